#!/bin/bash
# Parity suite + a short default bench, each under its own limit.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_sanity.json 2> gpurun_out/bench_sanity.log
rc=$?
cat gpurun_out/bench_sanity.json | cut -c1-400
exit $rc
