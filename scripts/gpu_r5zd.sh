#!/bin/bash
# round 5 final counters of the C2 headline (probe-and-resume fraction 0.25),
# then C3's long-row kernel at 4 / 3 / 2 waves per SIMD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5final}
EPS=0.058203125 bash scripts/gpu_r5final_pmc.sh r5final || exit 1
bash scripts/gpu_r5zc.sh r5zc || exit 1
