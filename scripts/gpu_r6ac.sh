#!/bin/bash
# round 6 ac: head entries kept speculated (NGT_AMD_LAT_FEED) against the lone
# ANNG query's latency, 32 slots
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6ac}; mkdir -p $O
D=/tmp/ngt_ac_anng_$$
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 1 \
  --warmup 1 --no-cpu --latency-queries 100 --capi-line off --anng-line off > $O/base.json 2> $O/base.log \
  || { tail -5 $O/base.log; exit 1; }
echo "base: $(grep -E 'single' $O/base.log | tr '\n' ' ')"
for f in ${FEEDS:-8 12 24 32 16}; do
  NGT_AMD_TEST_KNOBS=1 NGT_AMD_LAT_FEED=$f timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D \
    --eps 0.1279296875 --sweep-nq 10000 --steps 1 --warmup 1 --no-cpu --latency-queries 100 --capi-line off \
    --anng-line off > $O/f$f.json 2> $O/f$f.log || { tail -5 $O/f$f.log; exit 1; }
  echo "feed $f: $(grep -E 'single' $O/f$f.log | tr '\n' ' ')"
done
rm -rf $D
