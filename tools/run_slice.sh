set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/host_tests.log 2>&1 &&
timeout -k 10 200 python tools/host_overhead.py > gpurun_out/host_overhead.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-train --no-cpu-baseline > gpurun_out/bench_single.json 2> gpurun_out/bench_single.err &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --dist --steps 50 --warmup 10 --no-train --no-cpu-baseline --no-strong-probe > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err
echo "exit $?"
