set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/step_probe.py --workload ppi --double-proj --variants 'edge:;fill:PRED=fill;read:PRED=read;sleep:PRED=sleep' > gpurun_out/step_ppi3.json 2> gpurun_out/step_ppi3.err
echo "exit $?"
