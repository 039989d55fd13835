#!/bin/bash
# Round-end style refresh: default bench (exact C2, with CPU baseline), QG and C3
# bench lines, then the rocprofv3 trace + PMC passes of the default workload.
# usage: scripts/gpu_refresh.sh <tag>; outputs under gpurun_out/
TAG=${1:-r1d}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench_exact.json 2> gpurun_out/${TAG}_bench_exact.log || { tail -20 gpurun_out/${TAG}_bench_exact.log; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench_exact.json
timeout -k 10 400 python -u bench.py --mode qg --cpu-seconds 10 > gpurun_out/${TAG}_bench_qg.json 2> gpurun_out/${TAG}_bench_qg.log || { tail -20 gpurun_out/${TAG}_bench_qg.log; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench_qg.json
timeout -k 10 600 python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.log || { tail -20 gpurun_out/${TAG}_bench_c3.log; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench_c3.json
bash scripts/profile.sh ${TAG}_exact --steps 5 --warmup 2 --no-cpu --eps 0.0703125
