#!/bin/bash
# The fused small-Fin kernel with one vector load per x row, against the two
# launches: parity tests, then CIFAR H=4 / H=8 bench lines alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_parity.txt 2>&1
rc=$?; tail -3 $O/pytest_parity.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --workload cifar --workloads cifar_h8 --no-pmc --no-train --emulate-ranks "" --no-cpu-baseline --steps 50 \
    --detail-out $O/cifar_fused_$r.detail.json > $O/cifar_fused_$r.json 2> $O/cifar_fused_$r.err || exit 2
  GAT_EDGE_XPROJ=0 timeout -k 10 300 python3 bench.py --workload cifar --workloads cifar_h8 --no-pmc --no-train --emulate-ranks "" --no-cpu-baseline --steps 50 \
    --detail-out $O/cifar_two_$r.detail.json > $O/cifar_two_$r.json 2> $O/cifar_two_$r.err || exit 2
done
echo "chain exit 0"
