#!/bin/bash
# C2 overlapped steps, 2 vs 3 HIP streams, interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4v}; mkdir -p $O
for r in 1 2 3; do for st in 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 20 --streams $st \
    > $O/c2_st${st}_$r.json 2> $O/c2_st${st}_$r.log || { tail -5 $O/c2_st${st}_$r.log; exit 1; }
  python3 scripts/jline.py $O/c2_st${st}_$r.json "streams $st run $r"
done; done
