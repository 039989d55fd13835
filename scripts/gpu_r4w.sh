#!/bin/bash
# ANNG line (lookahead kernel) against resident waves per CU: how the step time
# (and so the loaded memory latency) moves with the load
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4w}; mkdir -p $O
D=/tmp/anng_r4w
for w in 16 12 8 4; do
  NGT_AMD_WAVES_PER_CU=$w timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 \
    --steps 2 --warmup 1 --no-cpu --latency-queries 0 --anng-line off > $O/w$w.json 2> $O/w$w.log || { tail -5 $O/w$w.log; exit 1; }
  python3 scripts/jline.py $O/w$w.json "waves/CU $w"
done
