#!/bin/bash
# Round-5 second A/B call (same box for every arm):
#  - projection: HEAD (x3 addressing restored) base / GAT_PROJ_PRESPLIT=1
#    against the bda929d tree, alternated;
#  - degree skew: hub segment order (GAT_HUB_ORDER=src) and whole-row order
#    (GAT_ROW_ORDER=asc) on power-law Reddit;
#  - short-row pipelined edge kernel (GAT_EDGE_PIPE=1) at PPI / arxiv / CIFAR;
#  - the training GPU tests (straight-line source pass now the default) and the
#    training step with and without it at dropout 0 (gradients cross-checked).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
OLD=abtree/bda929d
for r in 1 2; do
  (cd $OLD && timeout -k 10 300 python3 tools/proj_bench.py --shapes reddit,reddit@29120,arxiv,ppi --out /tmp/pb_old.json) > $O/proj_old_$r.txt 2>&1 || exit 2
  cp /tmp/pb_old.json $O/proj_old_$r.json
  timeout -k 10 300 python3 tools/proj_bench.py --shapes reddit,reddit@29120,arxiv,ppi \
    --variants "base;GAT_PROJ_PRESPLIT=1" --out $O/proj_new_$r.json > $O/proj_new_$r.txt 2>&1 || exit 2
done
echo "proj done"
timeout -k 10 400 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 5 --iters 5 \
  --variants "base;hubseg=2048;hubseg=2048,GAT_HUB_ORDER=src;hubseg=2048,GAT_ROW_ORDER=asc;hubseg=2048,GAT_HUB_ORDER=src,GAT_ROW_ORDER=asc" \
  > $O/edge_ab_hub_order_powerlaw.json 2> $O/edge_ab_hub_order_powerlaw.err || exit 2
echo "hub order done"
for wl in ppi arxiv cifar; do
  timeout -k 10 300 python3 tools/edge_ab.py --workload $wl --rounds 5 --iters 20 \
    --variants "base;GAT_EDGE_PIPE=1" > $O/edge_ab_pipe_short_$wl.json 2> $O/edge_ab_pipe_short_$wl.err || exit 2
done
echo "pipe done"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_training.txt 2>&1
rc=$?; tail -3 $O/pytest_training.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 tools/train_ab.py --workload reddit --dropout 0 \
  --variants "sl:;base:GAT_BWD_SL=0" > $O/train_ab_sl_reddit_p0.json 2> $O/train_ab_sl_reddit_p0.err || exit 2
echo "chain exit 0"
