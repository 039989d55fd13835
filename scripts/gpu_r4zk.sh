#!/bin/bash
# batchSizeForCreation parity (tests/test_gpu_build.py -k batch_size), then
# the 1M build-time / ANNG-line comparison of gpu_r4zj.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zk}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_build.py -m gpu \
  > $O/pytest_build.log 2>&1 || { tail -30 $O/pytest_build.log; exit 1; }
tail -3 $O/pytest_build.log
bash scripts/gpu_r4zj.sh ${1:-r4zk}
