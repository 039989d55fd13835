#!/bin/bash
# C5's per-GPU share on one GPU: 12.5M x 128 NGTQG as 10 shards of 1.25M
# (kmeansWithNGT codebooks, encoder and quantized graph per shard)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3g
timeout -k 10 1100 python -u bench.py --mode shard --qg --n 1250000 --shards-per-gpu 10 --steps 10 --warmup 2 \
  --shard-sample 1000 > gpurun_out/r3g/bench_c5_1gpu.json 2> gpurun_out/r3g/bench_c5_1gpu.log \
  || { tail -20 gpurun_out/r3g/bench_c5_1gpu.log; exit 1; }
cut -c1-400 gpurun_out/r3g/bench_c5_1gpu.json
