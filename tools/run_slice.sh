set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/qb_tests.log 2>&1 &&
timeout -k 10 200 python tools/slice_probe.py --workload ppi --slices 1,2 --vs 1 --us 4 > gpurun_out/slice_ppi_qb.json 2> gpurun_out/slice_ppi_qb.err &&
timeout -k 10 200 python tools/slice_probe.py --workload arxiv --slices 1 --vs 1 --us 4 > gpurun_out/slice_arxiv_qb.json 2> gpurun_out/slice_arxiv_qb.err &&
timeout -k 10 300 python tools/slice_probe.py --workload reddit --slices 2 --vs 2 --us 16 --pipes 1 --rounds 3 --iters 5 > gpurun_out/slice_reddit_qb.json 2> gpurun_out/slice_reddit_qb.err
echo "exit $?"
