#!/bin/bash
# Round-5 first GPU call: the full GPU suite once, then same-box A/Bs of the
# round-4 changes that were never timed:
#  - HEAD against the bda929d tree (abtree/bda929d, built in-tree there):
#    bench lines (projection + edge per workload) and proj_bench, alternated;
#  - GAT_BWD_SL=1 against the default source pass (train_ab, Reddit);
#  - GAT_PROJ_PRESPLIT=1 (proj_bench).
# Every GPU step has its own limit; a fault / abort / limit ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
ok() {  # continue after pass (0) or test failures (1); stop on anything else
  local rc=$1
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step rc=$rc: stopping"; exit $rc; fi
}
OLD=abtree/bda929d
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.txt 2>&1; ok $?
  tail -5 $O/pytest_gpu.txt
fi
BARGS="--no-cpu-baseline --no-pmc --emulate-ranks 2,4,8 --no-train --workloads reddit,reddit_powerlaw,arxiv --steps 20"
for r in 1 2; do
  (cd $OLD && timeout -k 10 300 python3 bench.py $BARGS --detail-out /tmp/old_detail.json) > $O/bench_old_$r.json 2> $O/bench_old_$r.err || exit 2
  cp /tmp/old_detail.json $O/bench_old_detail_$r.json
  timeout -k 10 300 python3 bench.py $BARGS --detail-out $O/bench_new_detail_$r.json > $O/bench_new_$r.json 2> $O/bench_new_$r.err || exit 2
  echo "bench round $r done"
done
for r in 1 2; do
  (cd $OLD && timeout -k 10 300 python3 tools/proj_bench.py --shapes reddit,reddit@29120,arxiv,ppi --out /tmp/pb_old.json) > $O/proj_old_$r.txt 2>&1 || exit 2
  cp /tmp/pb_old.json $O/proj_old_$r.json
  timeout -k 10 300 python3 tools/proj_bench.py --shapes reddit,reddit@29120,arxiv,ppi \
    --variants "base;GAT_PROJ_PRESPLIT=1" --out $O/proj_new_$r.json > $O/proj_new_$r.txt 2>&1 || exit 2
  echo "proj round $r done"
done
timeout -k 10 400 python3 tools/train_ab.py --workload reddit --dropout 0.6 \
  --variants "base:;sl:GAT_BWD_SL=1" > $O/train_ab_sl_reddit.json 2> $O/train_ab_sl_reddit.err || exit 2
timeout -k 10 300 python3 tools/train_ab.py --workload ppi --dropout 0.6 \
  --variants "base:;sl:GAT_BWD_SL=1" > $O/train_ab_sl_ppi.json 2> $O/train_ab_sl_ppi.err || exit 2
echo "chain exit 0"
