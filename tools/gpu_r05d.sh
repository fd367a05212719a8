#!/bin/bash
# The --dist bench at world 1 over a one-rank RCCL group, with the graph-
# replayed sharded step; the gat_forward per-call probe (arxiv).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python3 tools/probe_gat_forward.py --workload arxiv > $O/probe_gat_forward_arxiv.txt 2>&1 || exit 2
timeout -k 10 400 python3 bench.py --dist --dist-workloads ppi,arxiv --steps 20 --warmup 5 \
  --detail-out $O/bench_dist1_detail.json > $O/bench_dist1.json 2> $O/bench_dist1.err || exit 2
echo "dist chain exit 0"
timeout -k 10 300 python3 tools/proj_bench.py --shapes "arxiv@10624,arxiv@21184,arxiv@42368,arxiv@84672,arxiv,cifar_h8" \
  --variants "base;GAT_PROJ_WRES=0,GAT_PROJ_WK_MAX=128" --out $O/proj_wk128.json > $O/proj_wk128.txt 2>&1 || exit 2
echo "proj chain exit 0"
