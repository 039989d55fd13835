#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/kmeans3
timeout -k 10 300 python scripts/km_diag.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_build.py tests/test_gpu_qg.py tests/test_cxx_api.py tests/test_gpu_api.py tests/test_ngtpy.py -m gpu -v --timeout 600 \
  --timeout-method thread > gpurun_out/kmeans3/pytest.log 2>&1; tail -6 gpurun_out/kmeans3/pytest.log; grep -E "FAILED|PASSED.*quantize" gpurun_out/kmeans3/pytest.log | head
