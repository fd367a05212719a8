#!/bin/bash
# Same-box A/B of two builds of libgat_amd.so: alternates old/new/old/new
# under tools/train_ab.py.  usage: bash tools/ab_swap.sh <old.so> <new.so> <workload> <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=atmlgraphattentionnetworks_amd/libgat_amd.so
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp "$1" $L; else cp "$2" $L; fi
    timeout -k 10 300 python3 tools/train_ab.py --workload $3 --variants base > gpurun_out/swap_${4}_${v}_${r}.json 2>/dev/null || exit 1
  done
done
cp "$2" $L
echo "chain exit 0"
