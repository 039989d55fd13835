#!/bin/bash
# round 5: C3 at 3 waves per SIMD (12 per CU: ~13 KB of LDS per wave) with
# 512 (default), 768 and 1024 unchecked keys in LDS, interleaved twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5zk}; mkdir -p $O
for rep in a b; do
  for cq in 512 768 1024; do
    NGT_AMD_TEST_KNOBS=1 NGT_AMD_CQ_CAP=$cq timeout -k 10 300 python -u bench.py --config c3 --eps 0.056640625 \
      --steps 3 --warmup 1 --no-cpu --latency-queries 0 --anng-line off --c3-line off > $O/cq${cq}_$rep.json \
      2> $O/cq${cq}_$rep.log || { tail -20 $O/cq${cq}_$rep.log; exit 1; }
    python3 scripts/jline.py $O/cq${cq}_$rep.json cq${cq}_$rep
  done
done
