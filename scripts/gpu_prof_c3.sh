#!/bin/bash
# rocprofv3 passes on the C3 bench (filtered cosine long-row search)
set -o pipefail
TAG=${1:-r2v}
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/prof_r2c.sh c3 || exit $?
mkdir -p gpurun_out/$TAG && mv gpurun_out/prof_c3/* gpurun_out/$TAG/
