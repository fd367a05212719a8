#!/bin/bash
# PPI projection: the whole-K fp32 kernel (k_project_wk) against the split-bf16
# W-resident kernels (k_project_wres_d / k_project_wres) at fin 50, full PPI and
# a P = 8 rank's share; arxiv as the control.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/proj_bench.py --shapes "ppi,ppi@5632,arxiv" \
  --variants "base;GAT_PROJ_WRES=1;GAT_PROJ_WRES=1,GAT_PROJ_WRES_DIRECT=0" \
  --rounds 7 --out gpurun_out/proj_wres_ppi.json
