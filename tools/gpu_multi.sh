#!/bin/bash
# Several measurement steps in one GPU call, each under its own time limit,
# stopping at the first failure.  Steps are given as arguments:
#   test:<pytest -k expr>   proj:<shapes>|<variants>   emu:<workload>|<ranks>|<variants>
#   bench:<bench.py args>   edge:<workload>|<variants>   train:<workload>|<variants>|<dropout>
#   trainstats:<workload>|<steps>   trainsq:<workload>|<steps>
# usage: bash tools/gpu_multi.sh <tag> <step> [<step> ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
i=0
for STEP in "$@"; do
  i=$((i+1))
  KIND=${STEP%%:*}; ARG=${STEP#*:}
  OUT=gpurun_out/${TAG}_${i}_${KIND}
  echo "== step $i: $KIND $ARG"
  case $KIND in
    test)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests -k "$ARG" > $OUT.log 2>&1 || { echo "FAILED"; tail -40 $OUT.log; exit 1; }
      tail -1 $OUT.log ;;
    proj)
      S=${ARG%%|*}; V=${ARG#*|}
      timeout -k 10 600 python3 -u tools/proj_bench.py --shapes "$S" --variants "$V" --out $OUT.json > $OUT.log 2>&1 || { echo "FAILED"; tail -20 $OUT.log; exit 1; }
      grep '^{' $OUT.log ;;
    emu)
      W=${ARG%%|*}; REST=${ARG#*|}; R=${REST%%|*}; V=${REST#*|}
      timeout -k 10 900 python3 -u tools/emu_probe.py --workload $W --ranks $R --variants "$V" > $OUT.json 2> $OUT.err || { echo "FAILED"; tail -20 $OUT.err; exit 1; }
      cat $OUT.json ;;
    bench)
      timeout -k 10 900 python3 -u bench.py $ARG --detail-out $OUT.detail.json > $OUT.json 2> $OUT.err || { echo "FAILED"; tail -20 $OUT.err; exit 1; }
      cat $OUT.json ;;
    edge)
      W=${ARG%%|*}; V=${ARG#*|}
      timeout -k 10 600 python3 -u tools/edge_ab.py --workload $W --variants "$V" > $OUT.json 2> $OUT.err || { echo "FAILED"; tail -20 $OUT.err; exit 1; }
      cat $OUT.json ;;
    sq)
      # SQ / TCP counters of the projection at one shape under one variant
      S=${ARG%%|*}; V=${ARG#*|}
      j=0
      for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
        j=$((j+1))
        timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d ${OUT}_p$j -o run -- python3 tools/proj_bench.py --shapes "$S" --variants "$V" --rounds 1 --iters 4 > ${OUT}_p$j.log 2>&1 || { echo "FAILED pass $j"; tail -5 ${OUT}_p$j.log; exit 1; }
      done
      python3 tools/sq_summary.py ${OUT}_p* > $OUT.txt 2>&1
      cat $OUT.txt ;;
    edgepmc)
      # edge A/B, then per variant: fabric reads + L2 hit, and SQ wait/active counters
      W=${ARG%%|*}; V=${ARG#*|}
      timeout -k 10 600 python3 -u tools/edge_ab.py --workload $W --rounds 5 --variants "$V" > $OUT.json 2> $OUT.err || { echo "FAILED"; tail -20 $OUT.err; exit 1; }
      cat $OUT.json
      IFS=';' read -ra VV <<< "$V"
      for vi in "${!VV[@]}"; do
        timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d ${OUT}_pmc_v$vi -o run -- python3 tools/edge_ab.py --workload $W --variants "$V" --only $vi --iters 3 > ${OUT}_pmc_v$vi.log 2>&1 || { echo "FAILED pmc $vi"; exit 1; }
        timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d ${OUT}_sq_v$vi -o run -- python3 tools/edge_ab.py --workload $W --variants "$V" --only $vi --iters 3 > ${OUT}_sq_v$vi.log 2>&1 || { echo "FAILED sq $vi"; exit 1; }
      done
      python3 tools/pmc_edge_summary.py ${OUT}_pmc_v* > $OUT.pmc.json 2>&1; cat $OUT.pmc.json
      python3 tools/sq_summary.py ${OUT}_sq_v* > $OUT.sq.txt 2>&1; cat $OUT.sq.txt ;;
    train)
      # training-step A/B (tools/train_ab.py): <workload>|<variants>|<dropout>
      W=${ARG%%|*}; REST=${ARG#*|}; V=${REST%%|*}; D=${REST#*|}
      timeout -k 10 900 python3 -u tools/train_ab.py --workload $W --variants "$V" --dropout $D > $OUT.json 2> $OUT.err || { echo "FAILED"; tail -20 $OUT.err; exit 1; }
      cat $OUT.json ;;
    trainstats)
      # kernel-trace stats of training steps (tools/train_probe.py <workload> <steps>)
      W=${ARG%%|*}; N=${ARG#*|}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d ${OUT}_kt -o run -- python3 tools/train_probe.py $W $N > $OUT.log 2>&1 || { echo "FAILED"; tail -20 $OUT.log; exit 1; }
      find ${OUT}_kt -name '*kernel_stats.csv' -exec head -12 {} \; ;;
    trainsq)
      # SQ / TCP / TCC counters over a training step (tools/train_probe.py)
      W=${ARG%%|*}; N=${ARG#*|}
      j=0
      for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE"; do
        j=$((j+1))
        timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d ${OUT}_p$j -o run -- python3 tools/train_probe.py $W $N > ${OUT}_p$j.log 2>&1 || { echo "FAILED pass $j"; tail -5 ${OUT}_p$j.log; exit 1; }
      done
      python3 tools/sq_summary.py ${OUT}_p* > $OUT.txt 2>&1
      cat $OUT.txt ;;
    *) echo "unknown step $KIND"; exit 2 ;;
  esac
done
echo "ALL OK"
