#!/bin/bash
# 1M-object ANNG construction timing with the per-stage split, plus the C++ facade tests.
TAG=${1:-r2g}
N=${2:-1000000}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_cxx_api.py -m gpu -v -x --timeout 240 --timeout-method thread \
  > gpurun_out/$TAG/pytest_cxx.log 2>&1 || { tail -20 gpurun_out/$TAG/pytest_cxx.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_cxx.log
NGT_AMD_BUILD_PROFILE=1 timeout -k 10 900 python -u scripts/build_bench.py --n $N > gpurun_out/$TAG/build_$N.json \
  2> gpurun_out/$TAG/build_$N.log || { tail -20 gpurun_out/$TAG/build_$N.log; exit 1; }
tail -4 gpurun_out/$TAG/build_$N.log; cat gpurun_out/$TAG/build_$N.json
