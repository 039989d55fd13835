#!/bin/bash
# round 5: counter passes of C3 on the new default graph (single dispatch per search)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5n}; mkdir -p $O
PMC_LAST=3 bash scripts/pmc_r4.sh $O c3 --config c3 --eps 0.056640625 --sweep-nq 10000 --pmc-launches 3 --no-cpu \
  --anng-line off --c3-line off --latency-queries 0 || exit 1
