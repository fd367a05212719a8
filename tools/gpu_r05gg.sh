#!/bin/bash
# After the cheaper packed-parameter check: the full GPU suite, then the host
# cost of one eval forward (CIFAR, PPI).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05gg
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for wl in cifar ppi; do
  timeout -k 10 120 python3 tools/host_overhead.py $wl > $O/host_overhead_$wl.txt 2>&1 || exit 3
  grep "host enqueue" $O/host_overhead_$wl.txt
done
echo "chain exit 0"
