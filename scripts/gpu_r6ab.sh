#!/bin/bash
# round 6 ab: speculation slots (and so the head entries kept speculated,
# F = min(slots, 16)) against the lone ANNG query's latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6ab}; mkdir -p $O
D=/tmp/ngt_ab_anng_$$
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 1 \
  --warmup 1 --no-cpu --latency-queries 100 --capi-line off --anng-line off > $O/s32.json 2> $O/s32.log \
  || { tail -5 $O/s32.log; exit 1; }
grep -E "single" $O/s32.log
for sl in ${SLOTS:-8 12 16 24 32}; do
  NGT_AMD_TEST_KNOBS=1 NGT_AMD_LAT_SLOTS=$sl timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D \
    --eps 0.1279296875 --sweep-nq 10000 --steps 1 --warmup 1 --no-cpu --latency-queries 100 --capi-line off \
    --anng-line off > $O/s$sl.json 2> $O/s$sl.log || { tail -5 $O/s$sl.log; exit 1; }
  echo "slots $sl: $(grep -E 'single' $O/s$sl.log | tr '\n' ' ')"
done
rm -rf $D
