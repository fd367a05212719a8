#!/bin/bash
# The eval projection skips the s_src table when the fused edge kernels
# recompute it: forward parity (all variants incl. GAT_PROJ_SS=1), then the
# layer A/B at arxiv (row-major table: 5.4 MB of s_src stores) and CIFAR H=8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05ee
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_parity.py tests/test_gpu_gatnet.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/edge_ab.py --workload arxiv --rounds 11 --iters 20 --layer \
  --variants "base;GAT_PROJ_SS=1;GAT_WH_SLICES=2" > $O/edge_ab_projss_arxiv.json 2> $O/edge_ab_projss_arxiv.err || exit 3
echo "chain exit 0"
