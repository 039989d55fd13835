#!/bin/bash
# smoke(), then the NGTQG and C3 bench lines of the current tree (with CPU baselines).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r1h_smoke.log 2>&1 || { tail -20 gpurun_out/r1h_smoke.log; exit 1; }
tail -2 gpurun_out/r1h_smoke.log
timeout -k 10 400 python -u bench.py --mode qg --cpu-seconds 10 > gpurun_out/r1h_bench_qg.json 2> gpurun_out/r1h_bench_qg.log || { tail -20 gpurun_out/r1h_bench_qg.log; exit 1; }
cut -c1-300 gpurun_out/r1h_bench_qg.json
timeout -k 10 600 python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/r1h_bench_c3.json 2> gpurun_out/r1h_bench_c3.log || { tail -20 gpurun_out/r1h_bench_c3.log; exit 1; }
cut -c1-300 gpurun_out/r1h_bench_c3.json
