#!/bin/bash
# round 5: long-row parity + C2 at 4/3 waves per SIMD (gpu_r5ze.sh), then the
# NGTQG kernel at 4/3 waves per SIMD (gpu_r5zg.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r5ze.sh r5ze || exit 1
bash scripts/gpu_r5zg.sh r5zg || exit 1
