#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r2q
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r2q/pytest.log 2>&1 || { tail -30 gpurun_out/r2q/pytest.log; exit 1; }
tail -2 gpurun_out/r2q/pytest.log
bash scripts/gpu_anng.sh 10
