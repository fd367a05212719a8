#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03f}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 1000 $PYT -m gpu tests > gpurun_out/pytest_full_${TAG}.log 2>&1 &&
timeout -k 10 120 python3 tools/host_overhead.py cifar > gpurun_out/host_${TAG}_cifar.txt 2>&1 &&
timeout -k 10 400 python3 bench.py --no-pmc --no-train --no-cpu-baseline --emulate-ranks '' --workloads arxiv,cifar,cifar_h8 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
echo "chain exit $?" &&
timeout -k 10 300 python3 tools/edge_ab.py --workload ppi --variants "base;GAT_EDGE_SCHED=0;GAT_WH_SLICES=4;GAT_WH_SLICES=8;GAT_WH_SLICES=8,GAT_EDGE_V=2;GAT_WH_SLICES=8,GAT_EDGE_U=8" > gpurun_out/ab_planes_r03f_ppi.json 2>&1
echo "chain2 exit $?"
timeout -k 10 300 python3 tools/proj_ab.py --workload arxiv --variants "base;GAT_PROJ_WRES_NW=16" > gpurun_out/proj_ab_nw_r03f_arxiv.json 2>&1
timeout -k 10 300 python3 tools/proj_ab.py --workload ppi --variants "base;GAT_PROJ_WRES=1;GAT_PROJ_WRES=1,GAT_PROJ_WRES_NW=16" > gpurun_out/proj_ab_nw_r03f_ppi.json 2>&1
echo "chain3 exit $?"
