#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/kmeans
timeout -k 10 700 python -u -m pytest tests/test_gpu_qg.py -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/kmeans/pytest.log 2>&1 || { tail -40 gpurun_out/kmeans/pytest.log; exit 1; }
tail -6 gpurun_out/kmeans/pytest.log
