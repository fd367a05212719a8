#!/bin/bash
# Same-box A/B of two builds of libgat_amd.so on the PPI bench step and the
# P = 8 per-rank emulation: old/new/old/new.
# usage: bash tools/ab_bench.sh <old.so> <new.so> <tag>
# The in-tree library is restored on ANY exit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=atmlgraphattentionnetworks_amd/libgat_amd.so
BAK=$(mktemp /tmp/libgat_amd.XXXXXX.so)
cp "$L" "$BAK" || exit 1
trap 'cp "$BAK" "$L"; rm -f "$BAK"' EXIT
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp "$1" $L; else cp "$2" $L; fi
    timeout -k 10 300 python3 bench.py --workloads "${AB_WORKLOADS-cifar_h8}" --no-cpu-baseline --no-pmc --no-train --emulate-ranks 4,8 > gpurun_out/abb_${3}_${v}_${r}.json 2>/dev/null || exit 1
  done
done
echo "chain exit 0"
