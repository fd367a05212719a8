#!/bin/bash
# Pipelined edge kernel with the col ids four chunks ahead (RC = 2): GPU parity,
# then the same-box A/B on Reddit, power-law Reddit and the Reddit training step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_parity.py tests/test_gpu_training.py tests/test_gpu_hubs.py tests/test_gpu_distributed.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for wl in reddit reddit_powerlaw; do
  timeout -k 10 400 python3 tools/edge_ab.py --workload $wl --rounds 7 --iters 10 --layer \
    --variants "base;GAT_EDGE_PIPECOL=0" > $O/edge_ab_pipecol_$wl.json 2> $O/edge_ab_pipecol_$wl.err || exit 3
done
timeout -k 10 400 python3 tools/train_ab.py --workload reddit --rounds 3 --steps 5 \
  --variants "base:;no_pipecol:GAT_EDGE_PIPECOL=0" > $O/train_ab_pipecol_reddit.json 2> $O/train_ab_pipecol_reddit.err || exit 4
echo "chain exit 0"
