#!/bin/bash
# GPU check of the exact scans (run under gpurun): parity tests, stats, timings.
set -o pipefail
mkdir -p gpurun_out/lin
timeout -k 10 180 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_scan.py > gpurun_out/lin/pytest.log 2>&1 || exit 1
NGT_AMD_SCAN_STATS=1 timeout -k 10 120 python scripts/linear_check.py 1000000 10000 128 10 l2 mfma > gpurun_out/lin/s.json 2> gpurun_out/lin/err.log || exit 1
for d in ${SCAN_DBG:-2}; do
  NGT_AMD_SCAN_DBG=$d timeout -k 10 120 python scripts/linear_check.py 1000000 10000 128 10 l2 mfma > gpurun_out/lin/d$d.json 2>> gpurun_out/lin/err.log || exit 1
done
timeout -k 10 200 python scripts/linear_check.py 1000000 10000 128 10 l2 mfma,tiled > gpurun_out/lin/c2.json 2>> gpurun_out/lin/err.log || exit 1
if [ -n "$SCAN_C3" ]; then
  NGT_AMD_SCAN_STATS=1 timeout -k 10 300 python scripts/linear_check.py 1000000 10000 960 10 cosine mfma > gpurun_out/lin/c3.json 2>> gpurun_out/lin/err.log || exit 1
fi
