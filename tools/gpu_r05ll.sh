#!/bin/bash
# Training-path host trims (pointer arithmetic instead of per-call views; the
# gradient sums in their own buffer): the GPU training tests, the training
# probe (eager PPI step, torch profiler table), and the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=r05ll
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_training.py tests/test_gpu_gatnet.py > gpurun_out/pytest_train_${TAG}.txt 2>&1 &&
timeout -k 10 120 python3 tools/train_probe.py ppi 50 0.6 > gpurun_out/train_probe_${TAG}.json 2>&1 &&
TRAIN_PROBE_TORCHPROF=1 timeout -k 10 120 python3 tools/train_probe.py ppi 50 0.6 > gpurun_out/train_probe_prof_${TAG}.txt 2>&1 &&
timeout -k 10 600 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
echo "chain exit $?"
tail -1 gpurun_out/pytest_train_${TAG}.txt
cat gpurun_out/train_probe_${TAG}.json
