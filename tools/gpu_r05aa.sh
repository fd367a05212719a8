#!/bin/bash
# Source pass with the target ids two chunks ahead (k_bwd_sources_sl PF2):
# the training tests, then the same-box A/B of the training step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_training.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 tools/train_ab.py --workload reddit --rounds 3 --steps 5 \
  --variants "base:;no_pf2:GAT_BWD_PF2=0" > $O/train_ab_pf2_reddit.json 2> $O/train_ab_pf2_reddit.err || exit 3
timeout -k 10 300 python3 tools/train_ab.py --workload ppi --rounds 5 --steps 20 --dropout 0 \
  --variants "base:;no_pf2:GAT_BWD_PF2=0" > $O/train_ab_pf2_ppi.json 2> $O/train_ab_pf2_ppi.err || exit 4
echo "chain exit 0"
