#!/bin/bash
# round 5 final: counter passes of the C2 headline kernel at the epsilon the
# final bench line chose (probe-and-resume fraction 0.25): kernel trace, then
# FETCH_SIZE / WRITE_SIZE / SQ / TCC passes of 6 searches (12 dispatches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5final}; mkdir -p $O
EPS=${EPS:?}
PMC_LAST=12 bash scripts/pmc_r4.sh $O c2 --eps $EPS --sweep-nq 10000 --pmc-launches 6 --no-cpu --anng-line off \
  --c3-line off || exit 1
