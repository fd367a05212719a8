#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT -m gpu tests/test_gpu_fullsize.py tests/test_gpu_hubs.py tests/test_gpu_distributed.py -k "reddit or powerlaw" > gpurun_out/pytest_reddit_rows.log 2>&1
echo "chain exit $?"
