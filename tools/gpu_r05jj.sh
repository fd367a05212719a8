#!/bin/bash
# Round-5 evidence at HEAD (final):
# tools/gpu_final.sh, then the host cost of one eval forward (PPI, CIFAR).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/gpu_final.sh r05jj > gpurun_out/final_r05jj.log 2>&1
tail -2 gpurun_out/final_r05jj.log
grep -q "chain exit 0" gpurun_out/final_r05jj.log || exit 2
for wl in ppi cifar; do
  timeout -k 10 120 python3 tools/host_overhead.py $wl > gpurun_out/host_overhead_$wl.txt 2>&1 || exit 3
done
echo "host ok"
