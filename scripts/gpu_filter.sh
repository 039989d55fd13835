#!/bin/bash
# Distance-filter parity (filter on == off, production launch vs oracle) and the C2 bench line.
TAG=${1:-r2j}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py -m gpu -v -x --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG/pytest_filter.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_filter.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_filter.log
timeout -k 10 700 python bench.py > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.log || { tail -5 gpurun_out/$TAG/bench_c2.log; exit 1; }
tail -4 gpurun_out/$TAG/bench_c2.log; cut -c1-1500 gpurun_out/$TAG/bench_c2.json
