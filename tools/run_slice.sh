set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bwdpipe_tests.log 2>&1 &&
timeout -k 10 400 python tools/train_ab.py --workload reddit --dropout 0 --variants 'base:;pipe:GAT_BWD_PIPE=1' > gpurun_out/train_ab_reddit2.json 2> gpurun_out/train_ab_reddit2.err &&
timeout -k 10 400 python tools/train_ab.py --workload reddit --variants 'base:;pipe:GAT_BWD_PIPE=1' > gpurun_out/train_ab_reddit3.json 2> gpurun_out/train_ab_reddit3.err
echo "exit $?"
