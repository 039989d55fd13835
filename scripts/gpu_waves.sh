#!/bin/bash
# C2 at 16 vs 20 resident waves per CU (search variants built for 5 waves/SIMD,
# 16 Kbit LDS visited filter so 20 queries fit a CU's LDS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/waves
B="python bench.py --steps 10 --warmup 2 --no-cpu --eps 0.0703125"
NGT_AMD_VFILTER=14 timeout -k 10 300 $B > gpurun_out/waves/w4_vf14.json 2> gpurun_out/waves/w4_vf14.log || exit 1
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_w5.so NGT_AMD_VFILTER=14 NGT_AMD_WAVES_PER_CU=20 timeout -k 10 300 $B \
  > gpurun_out/waves/w5_vf14.json 2> gpurun_out/waves/w5_vf14.log || exit 1
for f in w4_vf14 w5_vf14; do python3 -c "import json; d=json.load(open('gpurun_out/waves/$f.json')); print('$f', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms'], d['config'].get('adjacency_prefetch_hits_per_expansion'))"; done
