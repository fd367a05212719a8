set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/train_ab.py --workload reddit --variants 'base:;l54:GAT_BWD_LDS=54000;l82:GAT_BWD_LDS=81920;l160:GAT_BWD_LDS=160000' > gpurun_out/train_ab_reddit.json 2> gpurun_out/train_ab_reddit.err
echo "exit $?"
