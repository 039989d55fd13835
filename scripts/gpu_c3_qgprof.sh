#!/bin/bash
# C3 (1M x 960 cosine) bench + rocprofv3 kernel trace and PMC passes of the QG bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log || { tail -20 gpurun_out/bench_c3.log; exit 1; }
cut -c1-400 gpurun_out/bench_c3.json
bash scripts/profile.sh r1c_qg --mode qg --steps 3 --warmup 1 --no-cpu --eps 0.05625
