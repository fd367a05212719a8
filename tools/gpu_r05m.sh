#!/bin/bash
# gpu_r05k.sh (small-Fin fused kernel: parity + CIFAR A/B) then gpu_r05l.sh
# (edges per chunk for short rows) in one call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r05k.sh && bash tools/gpu_r05l.sh
