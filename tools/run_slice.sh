set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "sliced or golden" -p no:cacheprovider > gpurun_out/il_tests.log 2>&1 &&
timeout -k 10 200 python tools/slice_probe.py --workload ppi --slices 1,2 --vs 1 --us 4,8 --pipes 0,1 > gpurun_out/slice_ppi_il.json 2> gpurun_out/slice_ppi_il.err &&
timeout -k 10 300 python tools/slice_probe.py --workload reddit --slices 2 --vs 2 --us 8,16 --pipes 0,1 --rounds 3 --iters 5 > gpurun_out/slice_reddit_il.json 2> gpurun_out/slice_reddit_il.err
echo "exit $?"
