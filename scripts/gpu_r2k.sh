#!/bin/bash
# Full GPU suite on the current tree, then rocprofv3 passes on the C2 bench
# (filtered graph search): kernel trace + FETCH/WRITE/SQ in separate passes.
set -o pipefail
TAG=${1:-r2k}
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_gpu.log
bash scripts/prof_r2c.sh c2 || exit $?
