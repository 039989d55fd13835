#!/bin/bash
# lookahead kernel phase split on the ANNG (stamps build, diagnostic only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4q}; mkdir -p $O
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --graph anng --anng-line off --steps 2 --warmup 1 \
  --no-cpu --latency-queries 0 --eps 0.128 > $O/stamps_anng.json 2> $O/stamps_anng.log || { tail -20 $O/stamps_anng.log; exit 1; }
grep -E "phase|expansions|discarded|eps|QPS" $O/stamps_anng.log
