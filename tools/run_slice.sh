set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pipe2_tests.log 2>&1 &&
timeout -k 10 300 python tools/step_probe.py --workload arxiv --variants 'pipe2:;pipe1:GAT_PROJ_PIPE=1' > gpurun_out/step_arxiv2.json 2> gpurun_out/step_arxiv2.err &&
timeout -k 10 300 python tools/step_probe.py --workload reddit --rounds 3 --steps 10 --variants 'pipe2:;pipe1:GAT_PROJ_PIPE=1' > gpurun_out/step_reddit2.json 2> gpurun_out/step_reddit2.err
echo "exit $?"
