set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/slice_probe.py --workload ppi --slices 1,2,4 --us 4,8,16 > gpurun_out/slice_ppi.json 2> gpurun_out/slice_ppi.err &&
timeout -k 10 200 python tools/slice_probe.py --workload arxiv --slices 1,2 --us 4,8 > gpurun_out/slice_arxiv.json 2> gpurun_out/slice_arxiv.err &&
timeout -k 10 300 python tools/slice_probe.py --workload reddit --slices 1,2,4 --us 8,16 --rounds 3 --iters 5 > gpurun_out/slice_reddit.json 2> gpurun_out/slice_reddit.err
echo "exit $?"
