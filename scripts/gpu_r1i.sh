#!/bin/bash
# ngtpy GPU tests, then the default C2 line and the QG line (finer epsilon bisection).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ngtpy.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1i_ngtpy.log 2>&1 || { tail -30 gpurun_out/r1i_ngtpy.log; exit 1; }
tail -2 gpurun_out/r1i_ngtpy.log
timeout -k 10 400 python -u bench.py > gpurun_out/r1i_bench_exact.json 2> gpurun_out/r1i_bench_exact.log || { tail -20 gpurun_out/r1i_bench_exact.log; exit 1; }
cut -c1-260 gpurun_out/r1i_bench_exact.json
timeout -k 10 400 python -u bench.py --mode qg --cpu-seconds 10 > gpurun_out/r1i_bench_qg.json 2> gpurun_out/r1i_bench_qg.log || { tail -20 gpurun_out/r1i_bench_qg.log; exit 1; }
cut -c1-260 gpurun_out/r1i_bench_qg.json
