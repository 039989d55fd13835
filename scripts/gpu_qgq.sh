#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/qgq
timeout -k 10 600 python -u -m pytest tests/test_gpu_qg.py -k quantize -m gpu -v -s --timeout 600 --timeout-method thread \
  > gpurun_out/qgq/pytest.log 2>&1; tail -4 gpurun_out/qgq/pytest.log; grep -E "sha256|assert" gpurun_out/qgq/pytest.log | head -5
