#!/bin/bash
# C2 occupancy sweep: waves per CU vs LDS filter / unchecked-array sizes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A="--eps 0.0703125 --no-cpu --steps 6"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py $A > gpurun_out/occ_$tag.json 2> gpurun_out/occ_$tag.log || return 1
  python -c "
import json;d=json.load(open('gpurun_out/occ_$tag.json'));print('$tag',round(d['value']),d['config']['recall_at_10'],round(d['roofline']['kernel_ms'],2),round(d['roofline']['frac'],3))"; }
run base NGT_AMD_WAVES_PER_CU=16 &&
run w24 NGT_AMD_WAVES_PER_CU=24 NGT_AMD_VFILTER=14 NGT_AMD_CQ_CAP=384 &&
run w32 NGT_AMD_WAVES_PER_CU=32 NGT_AMD_VFILTER=14 NGT_AMD_CQ_CAP=256 &&
run w16f14 NGT_AMD_WAVES_PER_CU=16 NGT_AMD_VFILTER=14 &&
run w32g2 NGT_AMD_WAVES_PER_CU=32 NGT_AMD_VFILTER=14 NGT_AMD_CQ_CAP=256 NGT_AMD_GROUPS=2
