#!/bin/bash
# resident serving grid: its tests, the latency tests, then the C-API line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3o
timeout -k 10 300 python -u -m pytest tests/test_gpu_serve.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3o/pytest_serve.log 2>&1 || { tail -40 gpurun_out/r3o/pytest_serve.log; exit 1; }
tail -3 gpurun_out/r3o/pytest_serve.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_api.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3o/pytest.log 2>&1 || { tail -30 gpurun_out/r3o/pytest.log; exit 1; }
tail -1 gpurun_out/r3o/pytest.log
timeout -k 10 400 python -u bench.py --mode capi --no-cpu --eps 0.0703125 \
  > gpurun_out/r3o/capi.json 2> gpurun_out/r3o/capi.log || { tail -5 gpurun_out/r3o/capi.log; exit 1; }
grep -h "C client\|single" gpurun_out/r3o/capi.log
