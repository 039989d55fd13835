#!/bin/bash
# GPU check of the exact scans (run under gpurun): parity tests, stats, timings.
# SCAN_MODES: NGT_AMD_SCAN_PASSES values to test (default "3 1"); SCAN_C3=1 adds the C3 shape.
set -o pipefail
mkdir -p gpurun_out/lin
for p in ${SCAN_MODES:-3 1}; do
  NGT_AMD_SCAN_PASSES=$p timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_scan.py > gpurun_out/lin/pytest_p$p.log 2>&1 || exit 1
  NGT_AMD_SCAN_PASSES=$p NGT_AMD_SCAN_STATS=1 timeout -k 10 120 python scripts/linear_check.py 1000000 10000 128 10 l2 mfma > gpurun_out/lin/c2_p$p.json 2>> gpurun_out/lin/err.log || exit 1
  if [ -n "$SCAN_C3" ]; then
    NGT_AMD_SCAN_PASSES=$p NGT_AMD_SCAN_STATS=1 timeout -k 10 300 python scripts/linear_check.py 1000000 10000 960 10 cosine mfma > gpurun_out/lin/c3_p$p.json 2>> gpurun_out/lin/err.log || exit 1
  fi
done
