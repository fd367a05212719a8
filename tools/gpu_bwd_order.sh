set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for M in natural outdeg; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bo_$M -o run -- python3 tools/bwd_order_probe.py reddit $M 8 > gpurun_out/bo_$M.json 2> gpurun_out/bo_$M.err || exit 1
  python3 tools/prof_summary.py gpurun_out/bo_$M/run_kernel_stats.csv > gpurun_out/bo_ks_$M.csv || exit 1
done
echo done
