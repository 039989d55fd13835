#!/bin/bash
# NGTQ IVF-ADC parity tests on the GPU.
TAG=${1:-r2f}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_ngtq.py -m gpu -v -x --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/pytest_ngtq.log 2>&1
rc=$?; tail -15 gpurun_out/$TAG/pytest_ngtq.log; exit $rc
