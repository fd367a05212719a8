#!/bin/bash
# Row-batched col values gated to rows of >= 16 in-edges: GPU parity, then
# the same-box A/B on PPI (and arxiv / CIFAR, where the gate now keeps the
# one-chunk-ahead form: both arms should match), plus the PPI training step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_parity.py tests/test_gpu_training.py tests/test_gpu_hubs.py tests/test_gpu_distributed.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for wl in ppi arxiv cifar_h8; do
  timeout -k 10 300 python3 tools/edge_ab.py --workload $wl --rounds 9 --iters 20 --layer \
    --variants "base;GAT_EDGE_ROWCOL=0" > $O/edge_ab_rowcol_$wl.json 2> $O/edge_ab_rowcol_$wl.err || exit 3
done
timeout -k 10 300 python3 tools/train_ab.py --workload ppi --variants "base:;no_rowcol:GAT_EDGE_ROWCOL=0" > $O/train_ab_rowcol_ppi.json 2> $O/train_ab_rowcol_ppi.err || exit 4
echo "chain exit 0"
