#!/bin/bash
# round 5: C3 graph mixes on the kNN-256 surrogate (max 256 edges per node):
# out 64 / in 224 (default) against out 96 / in 160, out 128 / in 128 and
# out 32 / in 224, each at the epsilon its own sweep picks
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5zm}; mkdir -p $O
for g in "64 224" "96 160" "128 128" "32 224"; do
  set -- $g
  timeout -k 10 400 python -u bench.py --config c3 --out-deg $1 --in-deg $2 --steps 3 --warmup 1 --no-cpu \
    --latency-queries 0 --anng-line off --c3-line off > $O/o$1_i$2.json 2> $O/o$1_i$2.log \
    || { tail -20 $O/o$1_i$2.log; exit 1; }
  python3 scripts/jline.py $O/o$1_i$2.json o$1_i$2
done
