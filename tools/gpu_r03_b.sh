#!/bin/bash
# r03 batch: write-through / register-epilogue A/B, scheduled-CSR edge A/B, new parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03b}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 200 python3 tools/step_probe.py --workload ppi --variants "wt:GAT_STORE_WT=1;plain:GAT_STORE_WT=0;wt_ldsepi:GAT_PROJ_REGEPI=0;plain_ldsepi:GAT_STORE_WT=0,GAT_PROJ_REGEPI=0" > gpurun_out/step_wt_${TAG}_ppi.json 2>&1 &&
timeout -k 10 400 $PYT tests/test_gpu_parity.py -k "golden or random or non_finite" > gpurun_out/pytest_parity_${TAG}.log 2>&1 &&
timeout -k 10 200 python3 tools/edge_ab.py --workload ppi --variants "base;sched=1;GAT_STORE_WT=0;sched=1,GAT_EDGE_U=8" > gpurun_out/ab_sched_${TAG}_ppi.json 2>&1 &&
timeout -k 10 200 python3 tools/edge_ab.py --workload arxiv --variants "base;sched=1;GAT_STORE_WT=0;GAT_EDGE_V=2;sched=1,GAT_EDGE_V=2;sched=1,GAT_EDGE_U=8" > gpurun_out/ab_sched_${TAG}_arxiv.json 2>&1 &&
for v in 1 0 1 0; do
  GAT_STORE_WT=$v timeout -k 10 200 python3 bench.py --workloads '' --no-pmc --no-train --no-cpu-baseline --emulate-ranks '' > gpurun_out/bench_wt${v}_${TAG}.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/bench_wt${v}_${TAG}.json'));print('wt=$v', d['value']/1e9, d['ms_per_step']*1e3, d['breakdown_ms'])" >> gpurun_out/bench_wt_${TAG}.txt
done &&
timeout -k 10 200 $PYT tests/test_gpu_training.py -k "hub_row" > gpurun_out/pytest_hubbwd_${TAG}.log 2>&1 &&
timeout -k 10 400 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 3 --variants "base;hubseg=1024;hubseg=512;hubseg=256" > gpurun_out/ab_hubseg_${TAG}.json 2>&1
echo "chain exit $?"
