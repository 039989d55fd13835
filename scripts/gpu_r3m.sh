#!/bin/bash
# latency kernel split into parts (exact rows only, two round trips per part):
# latency tests, C2 and ANNG single-query latency, the C-API line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3m
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookahead.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3m/pytest.log 2>&1 || { tail -20 gpurun_out/r3m/pytest.log; exit 1; }
tail -1 gpurun_out/r3m/pytest.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --eps 0.0703125 --latency-queries 200 \
  > gpurun_out/r3m/c2.json 2> gpurun_out/r3m/c2.log || { tail -5 gpurun_out/r3m/c2.log; exit 1; }
grep -h "single" gpurun_out/r3m/c2.log
timeout -k 10 300 python -u bench.py --mode capi --no-cpu --eps 0.0703125 \
  > gpurun_out/r3m/capi.json 2> gpurun_out/r3m/capi.log || { tail -5 gpurun_out/r3m/capi.log; exit 1; }
tail -c 1500 gpurun_out/r3m/capi.json
D=/tmp/anng1m
timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D --steps 3 --warmup 1 --no-cpu --eps 0.1279296875 \
  --latency-queries 50 > gpurun_out/r3m/anng.json 2> gpurun_out/r3m/anng.log || { tail -5 gpurun_out/r3m/anng.log; exit 1; }
grep -h "single" gpurun_out/r3m/anng.log
