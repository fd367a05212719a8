#!/bin/bash
# One parameterised GPU-box driver (replaces the per-experiment gpu_*.sh
# scripts of rounds 1-5, which stay in git history).
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Steps, run in order; each GPU step has its own time limit, and the first
# failure (test failures included), fault, abort or time limit ends the call:
#   tests[=FILES]        GPU suite (or the listed test files / node ids, comma-separated)
#   smoke                __graft_entry__.smoke()
#   bench[=ARGS]         bench.py [ARGS] -> gpurun_out/<tag>/bench.json (+ detail)
#   profppi              rocprofv3 --kernel-trace --stats of the PPI-only bench
#   profbench            rocprofv3 --kernel-trace --stats of the default bench (no PMC)
#   dist1                bench.py --dist at world 1 (the RCCL path over a one-rank group)
#   edgeab=WL:VARIANTS   tools/edge_ab.py --workload WL --variants VARIANTS
#   projab=SHAPES:VARS   tools/proj_bench.py --shapes SHAPES --variants VARS
#   trainab=WL:VARIANTS  tools/train_ab.py --workload WL --dropout 0.6 --variants VARIANTS
#   py=SCRIPT ARGS       python3 SCRIPT ARGS (a probe), output to <tag>/py_<n>.txt
# Outputs go to gpurun_out/<tag>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?usage: tools/gpu.sh <tag> <step>...}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
PYT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
n=0
run() {  # run <limit-seconds> <log> <cmd...>: stop the call on any non-zero status
  local lim=$1 log=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2> "$log.err"
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step '$STEP' rc=$rc: stopping"
    tail -5 "$log" "$log.err"
    exit $rc
  fi
}
for STEP in "$@"; do
  n=$((n + 1))
  echo "[gpu.sh $(date +%H:%M:%S)] $STEP"
  case "$STEP" in
    tests) run 1500 "$O/pytest_gpu.txt" $PYT -m gpu tests; tail -1 "$O/pytest_gpu.txt" ;;
    tests=*) f=${STEP#tests=}
      run 900 "$O/pytest_$n.txt" $PYT -m gpu ${f//,/ }; tail -1 "$O/pytest_$n.txt" ;;
    smoke) run 180 "$O/smoke.txt" python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 600 "$O/bench.json" python3 bench.py --detail-out "$O/bench_detail.json"; cat "$O/bench.json" ;;
    bench=*) run 600 "$O/bench_$n.json" python3 bench.py ${STEP#bench=} --detail-out "$O/bench_detail_$n.json"; cat "$O/bench_$n.json" ;;
    profppi)
      run 300 "$O/profppi.json" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profppi" -o run -- \
        python3 bench.py --workloads '' --no-cpu-baseline --no-pmc --no-train --emulate-ranks '' \
        --detail-out "$O/profppi_detail.json"
      python3 tools/prof_summary.py "$O/profppi/run_kernel_stats.csv" > "$O/kernel_stats_ppi.csv" ;;
    profbench)
      run 500 "$O/profbench.json" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/profbench" -o run -- \
        python3 bench.py --no-cpu-baseline --no-pmc --detail-out "$O/profbench_detail.json"
      python3 tools/prof_summary.py "$O/profbench/run_kernel_stats.csv" > "$O/kernel_stats_bench.csv" ;;
    dist1) run 400 "$O/bench_dist1.json" python3 bench.py --dist --dist-workloads ppi,arxiv --steps 10 --warmup 3 \
             --detail-out "$O/bench_dist1_detail.json" ;;
    edgeab=*) a=${STEP#edgeab=}
      run 600 "$O/edge_ab_${a%%:*}_$n.json" python3 tools/edge_ab.py --workload "${a%%:*}" --rounds 5 --iters 10 --variants "${a#*:}" ;;
    projab=*) a=${STEP#projab=}
      run 400 "$O/proj_ab_$n.txt" python3 tools/proj_bench.py --shapes "${a%%:*}" --variants "${a#*:}" --out "$O/proj_ab_$n.json" ;;
    trainab=*) a=${STEP#trainab=}
      run 600 "$O/train_ab_${a%%:*}_$n.json" python3 tools/train_ab.py --workload "${a%%:*}" --dropout 0.6 --variants "${a#*:}" ;;
    py=*) run 600 "$O/py_$n.txt" python3 ${STEP#py=} ;;
    *) echo "unknown step '$STEP'"; exit 2 ;;
  esac
done
echo "chain exit 0"
