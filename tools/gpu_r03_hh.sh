#!/bin/bash
# S = 4 split rows: parity (golden + random variants, sharded segment passes),
# then per-rank edge passes at P = 2/4/8 (PPI) and the single-GPU A/B of the
# small workloads, split 1 / 2 / 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_distributed.py -k "split or sharded" > gpurun_out/pytest_split4.log 2>&1 &&
timeout -k 10 300 python3 tools/emu_probe.py --workload ppi --ranks 2,4,8 --variants "GAT_EDGE_SPLIT=1;GAT_EDGE_SPLIT=2;GAT_EDGE_SPLIT=4" > gpurun_out/emu_split4_ppi.json 2> gpurun_out/emu_split4_ppi.err &&
timeout -k 10 300 python3 tools/emu_probe.py --workload arxiv --ranks 4,8 --variants "GAT_EDGE_SPLIT=1;GAT_EDGE_SPLIT=2;GAT_EDGE_SPLIT=4" > gpurun_out/emu_split4_arxiv.json 2> gpurun_out/emu_split4_arxiv.err &&
timeout -k 10 300 python3 tools/edge_ab.py --workload cifar_h8 --variants "GAT_EDGE_SPLIT=1;GAT_EDGE_SPLIT=2;GAT_EDGE_SPLIT=4" > gpurun_out/edge_ab_split4_cifar_h8.json 2> gpurun_out/edge_ab_split4_cifar_h8.err
echo "chain exit $?"
