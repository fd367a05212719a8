#!/bin/bash
# Row-batched col values for short rows (k_edge_grp RC): GPU parity (forward
# variants, training, hubs, distributed), then the same-box A/B against the
# one-chunk-ahead form on every short-row workload, and the PPI bisection.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_parity.py tests/test_gpu_training.py tests/test_gpu_hubs.py tests/test_gpu_distributed.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for wl in ppi arxiv cifar cifar_h8; do
  timeout -k 10 300 python3 tools/edge_ab.py --workload $wl --rounds 7 --iters 20 --layer \
    --variants "base;GAT_EDGE_ROWCOL=0" > $O/edge_ab_rowcol_$wl.json 2> $O/edge_ab_rowcol_$wl.err || exit 3
done
timeout -k 10 120 tools/edge_bisect > $O/edge_bisect.json 2> $O/edge_bisect.err || exit 4
echo "chain exit 0"
