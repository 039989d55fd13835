#!/bin/bash
# round 6 aa: the latency kernel's per-phase cycles on the ANNG line's lone
# queries (stamps build), for the commit wave's chain
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6aa}; mkdir -p $O
D=/tmp/ngt_aa_anng_$$
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 1 \
  --warmup 1 --no-cpu --latency-queries 100 --capi-line off --anng-line off > $O/prod.json 2> $O/prod.log \
  || { tail -5 $O/prod.log; exit 1; }
grep -E "single" $O/prod.log
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D \
  --eps 0.1279296875 --sweep-nq 10000 --steps 1 --warmup 1 --no-cpu --latency-queries 100 --capi-line off \
  --anng-line off > $O/stamps.json 2> $O/stamps.log || { tail -5 $O/stamps.log; exit 1; }
grep -E "single|phase" $O/stamps.log
rm -rf $D
