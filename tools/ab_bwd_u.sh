#!/bin/bash
# A/B of the recompute backward's edges-per-chunk (GAT_BWD_U) on PPI and Reddit.
export TMPDIR=/tmp; mkdir -p gpurun_out
for u in 4 8 16; do
  for w in ppi reddit; do
    st=30; [ $w = reddit ] && st=4
    GAT_BWD_U=$u timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abu_${w}_$u -o run -- python3 tools/train_probe.py $w $st 0.6 > gpurun_out/abu_${w}_$u.log 2>&1 || exit 1
  done
done
