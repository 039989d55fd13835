#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/kmeans2
timeout -k 10 300 python scripts/km_diag.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_qg.py tests/test_gpu_build.py tests/test_cxx_api.py -m gpu -x -v --timeout 600 \
  --timeout-method thread > gpurun_out/kmeans2/pytest.log 2>&1 || { tail -40 gpurun_out/kmeans2/pytest.log; exit 1; }
tail -4 gpurun_out/kmeans2/pytest.log
