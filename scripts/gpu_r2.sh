#!/bin/bash
# Round-2 GPU check: full pytest -m gpu (stops after 5 failures), then the
# default bench line (with the parity sample and the multi-core CPU baseline).
# usage: scripts/gpu_r2.sh <tag> [pytest selection]
TAG=${1:-r2a}
SEL=${2:-tests}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.log || exit $?
tail -4 gpurun_out/$TAG/bench.log
cat gpurun_out/$TAG/bench.json
