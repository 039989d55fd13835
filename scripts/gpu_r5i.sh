#!/bin/bash
# round 5: C3 phase split (stamps build) -- pop / adjacency + visited probes /
# filter codes / exact rows / accept, per query
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5i}; mkdir -p $O
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --config c3 --eps 0.0654296875 \
  --steps 2 --warmup 1 --no-cpu --latency-queries 0 --anng-line off --c3-line off > $O/stamps_c3.json \
  2> $O/stamps_c3.log || { tail -20 $O/stamps_c3.log; exit 1; }
grep -E "phase|expansions" $O/stamps_c3.log
