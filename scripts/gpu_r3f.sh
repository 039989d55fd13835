#!/bin/bash
# C4's 10M x 128 L2 index on one GPU (8 shards of 1.25M), then the QG trace
# and PMC passes at the QG line's epsilon
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3f
timeout -k 10 900 python -u bench.py --mode shard --n 1250000 --shards-per-gpu 8 --steps 10 --warmup 2 \
  > gpurun_out/r3f/bench_c4_1gpu.json 2> gpurun_out/r3f/bench_c4_1gpu.log || { tail -20 gpurun_out/r3f/bench_c4_1gpu.log; exit 1; }
cut -c1-400 gpurun_out/r3f/bench_c4_1gpu.json
bash scripts/pmc_r3.sh gpurun_out/r3f qg --mode qg --eps 0.05625 --sweep-nq 10000 --pmc-launches 6 --no-cpu || exit 1
