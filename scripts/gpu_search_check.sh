#!/bin/bash
# Exact-search parity (all graph-search tests), construction parity, 1M build timing, C2 bench line.
TAG=${1:-r2i}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_build.py tests/test_gpu_production.py \
  tests/test_gpu_api.py tests/test_gpu_shard.py tests/test_ngtpy.py -m gpu -v -x --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/pytest_search.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_search.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_search.log
NGT_AMD_BUILD_PROFILE=1 timeout -k 10 900 python -u scripts/build_bench.py --n 1000000 > gpurun_out/$TAG/build_1000000.json \
  2> gpurun_out/$TAG/build_1000000.log || { tail -20 gpurun_out/$TAG/build_1000000.log; exit 1; }
grep build_insert gpurun_out/$TAG/build_1000000.log; cat gpurun_out/$TAG/build_1000000.json
timeout -k 10 700 python bench.py > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.log || exit $?
tail -2 gpurun_out/$TAG/bench_c2.log; cut -c1-400 gpurun_out/$TAG/bench_c2.json
