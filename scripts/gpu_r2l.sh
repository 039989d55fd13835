#!/bin/bash
# Where a filtered C2 search spends its cycles (stamps build) and how long a
# single-stream step takes next to the 2-stream bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r2l
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --eps 0.0703125 \
  > gpurun_out/r2l/stamps.json 2> gpurun_out/r2l/stamps.log || { tail -5 gpurun_out/r2l/stamps.log; exit 1; }
grep -E "phase|expansions" gpurun_out/r2l/stamps.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --eps 0.0703125 --streams 1 \
  > gpurun_out/r2l/s1.json 2> gpurun_out/r2l/s1.log || { tail -5 gpurun_out/r2l/s1.log; exit 1; }
grep -E "expansions" gpurun_out/r2l/s1.log; cut -c1-400 gpurun_out/r2l/s1.json
