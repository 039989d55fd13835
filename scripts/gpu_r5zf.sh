#!/bin/bash
# round 5: counter passes of C3's kernel at 3 waves per SIMD (kernel trace,
# FETCH / WRITE / SQ / TCC), 3 launches of the line's epsilon each
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5zf}; mkdir -p $O
PMC_LAST=3 bash scripts/pmc_r4.sh $O c3 --config c3 --eps 0.056640625 --pmc-launches 3 --no-cpu --latency-queries 0 \
  --anng-line off --c3-line off || exit 1
