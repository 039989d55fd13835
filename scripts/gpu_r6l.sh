#!/bin/bash
# round 6 l: per-phase cycle split (stamps build, diagnostic only) of the
# NGTQG kernel on the qg key's configuration and of the lookahead kernel on
# the ANNG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6l}; mkdir -p $O
D=/tmp/ngt_st_anng_$$
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D \
  --eps 0.1279296875 --steps 2 --warmup 1 --no-cpu --latency-queries 0 --capi-line off > $O/anng.json 2> $O/anng.log \
  || { tail -20 $O/anng.log; exit 1; }
grep -h "phase" $O/anng.log
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --mode qg --graph anng --anng-dir $D \
  --eps 0.09772 --expansion 3 --steps 2 --warmup 1 --no-cpu --latency-queries 0 --anng-line off --c3-line off \
  --qg-line off > $O/qg.json 2> $O/qg.log || { tail -20 $O/qg.log; exit 1; }
grep -h "phase" $O/qg.log
rm -rf $D
