#!/bin/bash
# Round-5 evidence at HEAD (workgroup hub merge): tools/gpu_final.sh (full GPU suite, smoke, default
# bench, rocprofv3 of the bench and of the PPI-only bench, --dist at world 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/gpu_final.sh r05s > gpurun_out/final_r05s.log 2>&1
tail -2 gpurun_out/final_r05s.log
grep -q "chain exit 0" gpurun_out/final_r05s.log
