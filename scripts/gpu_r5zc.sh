#!/bin/bash
# round 5: C3's long-row kernel at 4 (product, 128 VGPRs, spills), 3 (168) and
# 2 (256, no spills) waves per SIMD, at the line's epsilon
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5zc}; mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config c3 --eps 0.056640625 --steps 3 \
    --warmup 1 --no-cpu --latency-queries 0 --anng-line off --c3-line off > $O/$name.json 2> $O/$name.log \
    || { tail -20 $O/$name.log; exit 1; }
  python3 scripts/jline.py $O/$name.json $name
}
L=$PWD/ngt_amd
for rep in a b; do
  run w4_$rep NGT_AMD_LIB=$L/libngt_amd.so
  run w3_$rep NGT_AMD_LIB=$L/libngt_amd_w3.so
  run w2_$rep NGT_AMD_LIB=$L/libngt_amd_w2.so
done
