#!/bin/bash
# k_project_wres_d (direct epilogue, 3 workgroups per CU) against k_project_wres:
# projection parity tests first (every variant incl. the new one), then
# proj_bench at arxiv and its rank shares.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_parity.txt 2>&1
rc=$?; tail -3 $O/pytest_parity.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/proj_bench.py --shapes "arxiv@21184,arxiv@42368,arxiv@84672,arxiv" \
  --variants "base;GAT_PROJ_WRES_DIRECT=1" --out $O/proj_wres_direct.json > $O/proj_wres_direct.txt 2>&1 || exit 2
echo "chain exit 0"
