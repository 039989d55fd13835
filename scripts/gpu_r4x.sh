#!/bin/bash
# lookahead kernel phase split at 4 and 16 resident waves per CU (stamps build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4x}; mkdir -p $O
D=/tmp/anng_r4x
for w in 4 16; do
  NGT_AMD_WAVES_PER_CU=$w NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D \
    --steps 2 --warmup 1 --no-cpu --latency-queries 0 --eps 0.128 --anng-line off > $O/stamps_w$w.json 2> $O/stamps_w$w.log || { tail -20 $O/stamps_w$w.log; exit 1; }
  echo "waves/CU $w"; grep -E "phase|kernel .* \(10000" $O/stamps_w$w.log
done
