set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/step_probe.py --workload ppi --double-proj --variants "base:;sleep:PRED=sleep;fill:PRED=fill;read:PRED=read;tiny:PRED=tinyproj" > gpurun_out/step_probe_r03a.json 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_distributed.py -k "rccl or bench" > gpurun_out/pytest_dist_r03a.log 2>&1 &&
timeout -k 10 300 python bench.py --workloads arxiv --no-pmc --no-train --no-cpu-baseline > gpurun_out/bench_emu_r03a.json 2> gpurun_out/bench_emu_r03a.err
echo "chain exit $?"
