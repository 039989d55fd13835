#!/bin/bash
# per-part readiness in the latency kernel: tests, C2 single-query latency,
# C-API line; then the suite order that failed (scan, production before serve)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_serve.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3s/pytest.log 2>&1 || { tail -30 gpurun_out/r3s/pytest.log; exit 1; }
tail -1 gpurun_out/r3s/pytest.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --eps 0.0703125 --latency-queries 200 \
  > gpurun_out/r3s/c2.json 2> gpurun_out/r3s/c2.log || { tail -5 gpurun_out/r3s/c2.log; exit 1; }
grep -h "single" gpurun_out/r3s/c2.log
timeout -k 10 400 python -u bench.py --mode capi --no-cpu --eps 0.0703125 \
  > gpurun_out/r3s/capi.json 2> gpurun_out/r3s/capi.log || { tail -5 gpurun_out/r3s/capi.log; exit 1; }
grep -h "C client" gpurun_out/r3s/capi.log
for set in "tests/test_gpu_scan.py tests/test_gpu_serve.py" "tests/test_gpu_production.py tests/test_gpu_serve.py"; do
  n=$(echo $set | tr ' /' '__')
  timeout -k 10 400 python -u -m pytest $set -q --timeout 200 --timeout-method thread > gpurun_out/r3s/$n.log 2>&1
  rc=$?
  echo "$set rc=$rc"; tail -2 gpurun_out/r3s/$n.log
  grep -h "batch search failed" gpurun_out/r3s/$n.log | head -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
