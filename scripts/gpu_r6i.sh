#!/bin/bash
# round 6 i: stream-count A/B of the C2 headline, the ANNG line and the qg
# line (the same timed steps over 2..5 streams after the line's own)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6i}; mkdir -p $O
D=/tmp/ngt_ab_anng_$$
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu --latency-queries 0 --anng-line off --c3-line off \
  --qg-line off --streams-ab 2,3,4,5,3 > $O/c2.json 2> $O/c2.log || { tail -20 $O/c2.log; exit 1; }
grep "streams" $O/c2.log
timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D --steps 10 --warmup 2 --no-cpu --latency-queries 0 \
  --capi-line off --streams-ab 2,3,4,5,3 > $O/anng.json 2> $O/anng.log || { tail -20 $O/anng.log; exit 1; }
grep "streams" $O/anng.log
timeout -k 10 400 python -u bench.py --mode qg --graph anng --anng-dir $D --eps 0.09772 --expansion 3 --steps 10 \
  --warmup 2 --no-cpu --latency-queries 0 --anng-line off --c3-line off --qg-line off --streams-ab 2,3,4,5,3 \
  > $O/qg.json 2> $O/qg.log || { tail -20 $O/qg.log; exit 1; }
grep "streams" $O/qg.log
rm -rf $D
