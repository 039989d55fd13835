#!/bin/bash
# A/B on one box: the current library vs ngt_amd/libngt_amd_ab.so (C2 bench,
# alternating), then the 1M construction with each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
B="python bench.py --steps 10 --warmup 2 --no-cpu --eps 0.0703125"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/ab/cur$i.json 2> gpurun_out/ab/cur$i.log || exit 1
  NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_ab.so timeout -k 10 300 $B > gpurun_out/ab/old$i.json 2> gpurun_out/ab/old$i.log || exit 1
done
for f in cur1 old1 cur2 old2; do python3 -c "import json; d=json.load(open('gpurun_out/ab/$f.json')); print('$f', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2))"; done
for L in cur ab; do
  LIBV=""; [ $L = ab ] && LIBV="NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_ab.so"
  env $LIBV NGT_AMD_BUILD_PROFILE=1 timeout -k 10 400 python scripts/build_bench.py --n 1000000 --check 200 \
    > gpurun_out/ab/build_$L.json 2> gpurun_out/ab/build_$L.log || exit 1
  grep build_insert gpurun_out/ab/build_$L.log | head -1
done
