#!/bin/bash
# accepted-only lookahead line accounting (timed launches' counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4t}; mkdir -p $O
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_lacount.so timeout -k 10 400 python -u bench.py --graph anng --anng-line off --steps 2 --warmup 1 \
  --no-cpu --latency-queries 0 --eps 0.128 > $O/lacount_anng.json 2> $O/lacount_anng.log || { tail -20 $O/lacount_anng.log; exit 1; }
grep -E "accounting|evaluations" $O/lacount_anng.log
