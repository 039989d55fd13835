#!/bin/bash
# counter passes (trace, FETCH_SIZE, WRITE_SIZE, SQ wave-cycle split, TCC hit/miss +
# memory-side reads) of the C2 headline (scheduled: 2 dispatches per search) and the ANNG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4h}; mkdir -p $O
PMC_LAST=12 bash scripts/pmc_r4.sh $O c2 --eps 0.0703125 --sweep-nq 10000 --pmc-launches 6 --no-cpu --anng-line off || exit 1
D=/tmp/anng_r4h
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 1 --warmup 1 \
  --no-cpu --latency-queries 0 --anng-line off > $O/anng_build.json 2> $O/anng_build.log || { tail -5 $O/anng_build.log; exit 1; }
PMC_LAST=6 bash scripts/pmc_r4.sh $O anng --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --pmc-launches 6 --no-cpu --anng-line off || exit 1
ls $O
