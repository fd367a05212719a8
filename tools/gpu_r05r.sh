#!/bin/bash
# Power-law vs uniform Reddit edge kernel: address-translation (UTCL1) and
# DRAM-vs-Infinity-Cache counters, one rocprofv3 --pmc pass per counter set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
for W in reddit_powerlaw reddit; do
  i=0
  for CTRS in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum" \
              "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum" \
              "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $O/${W}_p$i -o run -- python3 tools/pmc_run.py --workload $W --iters 3 > $O/${W}_p$i.log 2>&1 || { echo "pmc $W pass $i failed"; tail -5 $O/${W}_p$i.log; exit 2; }
  done
  python3 tools/pmc_kernel_summary.py --match k_edge_grp $O/${W}_p* > $O/pmc_${W}.json
done
echo "chain exit 0"
