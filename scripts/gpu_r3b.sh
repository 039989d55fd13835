#!/bin/bash
# counters for the C2 and ANNG search kernels; sharded-path GPU tests and a
# small multi-shard bench (the S-shards-per-GPU code path)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3b
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_shard.py \
  > gpurun_out/r3b/pytest_shard.log 2>&1 || { tail -20 gpurun_out/r3b/pytest_shard.log; exit 1; }
tail -1 gpurun_out/r3b/pytest_shard.log
timeout -k 10 300 python -u bench.py --mode shard --n 200000 --shards-per-gpu 4 --steps 3 --warmup 1 \
  > gpurun_out/r3b/shard_small.json 2> gpurun_out/r3b/shard_small.log || { tail -20 gpurun_out/r3b/shard_small.log; exit 1; }
cut -c1-400 gpurun_out/r3b/shard_small.json
D=/tmp/anng1m
timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D --steps 1 --warmup 1 --no-cpu --eps 0.1279296875 \
  --latency-queries 0 > gpurun_out/r3b/anng_build.json 2> gpurun_out/r3b/anng_build.log || { tail -5 gpurun_out/r3b/anng_build.log; exit 1; }
bash scripts/pmc_r3.sh gpurun_out/r3b c2 --eps 0.0703125 --sweep-nq 10000 --pmc-launches 6 --no-cpu || exit 1
bash scripts/pmc_r3.sh gpurun_out/r3b anng --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 \
  --pmc-launches 6 --no-cpu || exit 1
