#!/bin/bash
# round 5 final (2): the committed tree after the C3 occupancy change -- smoke,
# the whole GPU suite, the driver's bench command; then C3's counter passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r5final.sh r5final2 || exit 1
bash scripts/gpu_r5zf.sh r5zf || exit 1
