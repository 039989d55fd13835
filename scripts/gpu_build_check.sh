#!/bin/bash
# Construction parity (C1 byte-identical build) and the 1M construction timing.
TAG=${1:-r2h}
N=${2:-1000000}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_build.py tests/test_gpu_production.py -m gpu -v -x --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG/pytest_build.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_build.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_build.log
NGT_AMD_BUILD_PROFILE=1 timeout -k 10 900 python -u scripts/build_bench.py --n $N > gpurun_out/$TAG/build_$N.json \
  2> gpurun_out/$TAG/build_$N.log || { tail -20 gpurun_out/$TAG/build_$N.log; exit 1; }
grep build_insert gpurun_out/$TAG/build_$N.log; cat gpurun_out/$TAG/build_$N.json
