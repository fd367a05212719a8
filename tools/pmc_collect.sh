#!/bin/bash
# PMC passes for one workload (counters only, no tracing domains), then parse.
# usage: bash tools/pmc_collect.sh <workload> [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
W=${1:-ppi}; TAG=${2:-r01}
mkdir -p gpurun_out
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc_${W}_${TAG}_p$i -o run -- python3 tools/pmc_run.py --workload $W > gpurun_out/pmc_${W}_${TAG}_p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
PMC_OUT=gpurun_out/pmc_${W}_${TAG}.json python3 tools/pmc_traffic.py $W gpurun_out/pmc_${W}_${TAG}_p*
