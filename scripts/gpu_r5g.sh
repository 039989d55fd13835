#!/bin/bash
# round 5: counter passes (kernel trace, FETCH, WRITE, SQ, TCC) of the NGTQG
# kernel with the packed layout: the C2-graph QG line and the 2M one-ANNG QG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5g}; mkdir -p $O
PMC_LAST=3 bash scripts/pmc_r4.sh $O qg_c2 --mode qg --eps 0.05625 --pmc-launches 3 --no-cpu --latency-queries 0 \
  --anng-line off --c3-line off || exit 1
PMC_LAST=3 bash scripts/pmc_r4.sh $O qg_anng2m --mode qg --graph anng --n 2000000 --anng-batch 8000 --eps 0.10529 \
  --pmc-launches 3 --no-cpu --latency-queries 0 || exit 1
