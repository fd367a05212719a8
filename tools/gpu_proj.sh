#!/bin/bash
# Projection timing (tools/proj_bench.py) over shapes and knob variants, then
# optional SQ counter passes of the projection at one shape.
# usage: bash tools/gpu_proj.sh <tag> "<variants>" "<shapes>" [sq_shape]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-proj}; V=${2:-base}; S=${3:-reddit,reddit@29120,arxiv,ppi}; SQ=${4:-}
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/proj_bench.py --shapes "$S" --variants "$V" --out gpurun_out/proj_bench_${TAG}.json > gpurun_out/proj_bench_${TAG}.log 2>&1 || { echo "proj_bench failed"; tail -20 gpurun_out/proj_bench_${TAG}.log; exit 1; }
cat gpurun_out/proj_bench_${TAG}.log
if [ -n "$SQ" ]; then
  i=0
  for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/sqp_${TAG}_p$i -o run -- python3 tools/proj_bench.py --shapes "$SQ" --variants "base" --rounds 1 --iters 4 > gpurun_out/sqp_${TAG}_p$i.log 2>&1 || { echo "sq pass $i failed"; exit 1; }
  done
  python3 tools/sq_summary.py gpurun_out/sqp_${TAG}_p* > gpurun_out/sqp_${TAG}.txt 2>&1
  cat gpurun_out/sqp_${TAG}.txt | head -60
fi
