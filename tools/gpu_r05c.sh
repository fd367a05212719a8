#!/bin/bash
# Round-5 evidence after adopting the A/B winners (x3 addressing restored, W
# pre-split, straight-line source pass, hub segments by source): tools/gpu_final.sh
# (full GPU suite, smoke, default bench, rocprofv3 of the bench and of the
# PPI-only bench, --dist at world 1), then a rank-share projection probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/gpu_final.sh r05c > gpurun_out/final_r05c.log 2>&1
tail -2 gpurun_out/final_r05c.log
grep -q "chain exit 0" gpurun_out/final_r05c.log || exit 3
timeout -k 10 300 python3 tools/proj_bench.py --shapes "ppi@5632,arxiv@21184,arxiv@42368,arxiv" \
  --variants "base;GAT_PROJ_WK_MAX=128;GAT_PROJ_WRES=0" --out gpurun_out/proj_share_r05c.json \
  > gpurun_out/proj_share_r05c.txt 2>&1 || exit 2
echo "r05c exit 0"
