#!/bin/bash
# diagnose the batch-search error flag seen after the serving test in the full suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3r
for set in "tests/test_gpu_serve.py" "tests/test_gpu_scan.py tests/test_gpu_serve.py" "tests/test_gpu_production.py tests/test_gpu_serve.py"; do
  n=$(echo $set | tr ' /' '__')
  timeout -k 10 400 python -u -m pytest $set -q --timeout 200 --timeout-method thread > gpurun_out/r3r/$n.log 2>&1
  rc=$?
  echo "$set rc=$rc"; tail -3 gpurun_out/r3r/$n.log
  grep -h "batch search failed" gpurun_out/r3r/$n.log | head -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 400 python -u bench.py --mode capi --no-cpu --eps 0.0703125 \
  > gpurun_out/r3r/capi.json 2> gpurun_out/r3r/capi.log || { tail -5 gpurun_out/r3r/capi.log; exit 1; }
grep -h "C client\|single" gpurun_out/r3r/capi.log
