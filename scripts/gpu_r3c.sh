#!/bin/bash
# QG line (kmeansWithNGT codebooks, oracle LUTs in the parity sample) + its
# trace/PMC passes at the line's epsilon; then C4's 10M index on one GPU as
# 8 shards of 1.25M
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3c
timeout -k 10 600 python -u bench.py --mode qg --cpu-seconds 10 > gpurun_out/r3c/bench_qg.json 2> gpurun_out/r3c/bench_qg.log \
  || { tail -20 gpurun_out/r3c/bench_qg.log; exit 1; }
cut -c1-300 gpurun_out/r3c/bench_qg.json
EPS=$(python3 -c "import json; print(repr(json.load(open('gpurun_out/r3c/bench_qg.json'))['config']['epsilon']))")
bash scripts/pmc_r3.sh gpurun_out/r3c qg --mode qg --eps $EPS --sweep-nq 10000 --pmc-launches 6 --no-cpu || exit 1
timeout -k 10 900 python -u bench.py --mode shard --n 1250000 --shards-per-gpu 8 --steps 10 --warmup 2 \
  > gpurun_out/r3c/bench_c4_1gpu.json 2> gpurun_out/r3c/bench_c4_1gpu.log || { tail -20 gpurun_out/r3c/bench_c4_1gpu.log; exit 1; }
cut -c1-400 gpurun_out/r3c/bench_c4_1gpu.json
