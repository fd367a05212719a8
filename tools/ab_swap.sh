#!/bin/bash
# Same-box A/B of two builds of libgat_amd.so: alternates old/new/old/new
# under tools/train_ab.py.  usage: bash tools/ab_swap.sh <old.so> <new.so> <workload> <tag>
# The in-tree library is backed up first and restored on ANY exit (a failed
# run must not leave a candidate build installed for later tests or benches).
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
    timeout -k 10 300 python3 tools/train_ab.py --workload $3 --variants base > gpurun_out/swap_${4}_${v}_${r}.json 2>/dev/null || exit 1
  done
done
echo "chain exit 0"
