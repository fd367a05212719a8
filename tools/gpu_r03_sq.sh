#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/sq_collect.sh ppi r03 && bash tools/sq_collect.sh arxiv r03
echo "chain exit $?"
