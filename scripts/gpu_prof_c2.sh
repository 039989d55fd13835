#!/bin/bash
# rocprofv3 passes on the C2 bench (kernel trace + FETCH / WRITE / SQ in separate passes)
set -o pipefail
TAG=${1:-r2o}
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/prof_r2c.sh c2 || exit $?
mkdir -p gpurun_out/$TAG && mv gpurun_out/prof_c2/* gpurun_out/$TAG/
