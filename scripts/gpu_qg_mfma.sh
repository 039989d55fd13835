#!/bin/bash
# QG kernel with the matrix-core ADC sum: QG parity tests, then the QG bench line.
TAG=${1:-r2d}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_qg.py tests/test_gpu_production.py -m gpu -v -x --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG/pytest_qg.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/pytest_qg.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python bench.py --mode qg > gpurun_out/$TAG/bench_qg.json 2> gpurun_out/$TAG/bench_qg.log || exit $?
tail -3 gpurun_out/$TAG/bench_qg.log; cat gpurun_out/$TAG/bench_qg.json
