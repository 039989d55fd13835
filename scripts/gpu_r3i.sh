#!/bin/bash
# C3 line (1M x 960 cosine, cosine filter) and its trace + PMC passes at the
# line's epsilon (the C3 kernel changed after the round-2 counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3i
timeout -k 10 700 python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 10 --latency-queries 20 \
  > gpurun_out/r3i/bench_c3.json 2> gpurun_out/r3i/bench_c3.log || { tail -20 gpurun_out/r3i/bench_c3.log; exit 1; }
cut -c1-300 gpurun_out/r3i/bench_c3.json
EPS=$(python3 -c "import json; print(repr(json.load(open('gpurun_out/r3i/bench_c3.json'))['config']['epsilon']))")
bash scripts/pmc_r3.sh gpurun_out/r3i c3 --config c3 --eps $EPS --sweep-nq 10000 --pmc-launches 2 --no-cpu || exit 1
