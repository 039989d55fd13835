#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/rccl
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/rccl/pytest.log 2>&1 || { tail -40 gpurun_out/rccl/pytest.log; exit 1; }
tail -8 gpurun_out/rccl/pytest.log
