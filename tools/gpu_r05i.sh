#!/bin/bash
# The lean short-row edge kernel (GAT_HINT_SHORT_ROWS: no Kahan / dropout code,
# 60 VGPRs, 8 waves per SIMD) against the full one, then the parity suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
for wl in ppi arxiv cifar cifar_h8; do
  timeout -k 10 300 python3 tools/edge_ab.py --workload $wl --rounds 7 --iters 20 --layer \
    --variants "base;GAT_EDGE_LEAN=1" > $O/edge_ab_lean_$wl.json 2> $O/edge_ab_lean_$wl.err || exit 2
done
echo "ab done"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_parity.txt 2>&1
rc=$?; tail -3 $O/pytest_parity.txt; exit $rc
