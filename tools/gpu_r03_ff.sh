#!/bin/bash
# what does attention dropout cost the training step? kernel stats at p = 0.6 and 0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for P in 0.6 0.0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_drop${P} -o run -- python3 tools/train_ab.py --workload reddit --variants "base:" --rounds 1 --dropout $P > gpurun_out/kt_drop${P}.log 2>&1 || exit 1
  python3 tools/prof_summary.py gpurun_out/kt_drop${P}/run_kernel_stats.csv > gpurun_out/kt_drop${P}.csv || exit 1
done
echo "chain exit $?"
