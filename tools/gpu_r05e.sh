#!/bin/bash
# Hub-segment length with the source-ordered segments (power-law and uniform
# Reddit), then the distributed GPU tests (graph-replayed sharded step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 400 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 5 --iters 5 \
  --variants "base;hubseg=256;hubseg=512;hubseg=1024;hubseg=4096" \
  > $O/edge_ab_hubseg_powerlaw.json 2> $O/edge_ab_hubseg_powerlaw.err || exit 2
timeout -k 10 400 python3 tools/edge_ab.py --workload reddit --rounds 5 --iters 5 \
  --variants "base;hubseg=128;hubseg=256" \
  > $O/edge_ab_hubseg_reddit.json 2> $O/edge_ab_hubseg_reddit.err || exit 2
echo "edge done"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_dist.txt 2>&1
rc=$?; tail -3 $O/pytest_dist.txt; exit $rc
