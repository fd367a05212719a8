#!/bin/bash
# SQ/TA occupancy and stall counters (separate passes) + a kernel trace, one workload.
# usage: bash tools/sq_collect.sh <workload> <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
W=${1:-ppi}; TAG=${2:-r01}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${W}_${TAG} -o run -- python3 tools/pmc_run.py --workload $W --iters 10 > gpurun_out/kt_${W}_${TAG}.log 2>&1 || exit 1
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/sq_${W}_${TAG}_p$i -o run -- python3 tools/pmc_run.py --workload $W > gpurun_out/sq_${W}_${TAG}_p$i.log 2>&1 || { echo "sq pass $i failed"; exit 1; }
done
python3 tools/sq_summary.py gpurun_out/sq_${W}_${TAG}_p* > gpurun_out/sq_${W}_${TAG}.txt
python3 tools/prof_summary.py gpurun_out/kt_${W}_${TAG}/run_kernel_stats.csv > gpurun_out/kt_${W}_${TAG}.csv
