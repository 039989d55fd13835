#!/bin/bash
# Same-box A/B: C2 bench current vs ngt_amd/libngt_amd_ab.so (alternating);
# C-API single-query latency with the filter on (default) and forced off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab2
B="python bench.py --steps 10 --warmup 2 --no-cpu --eps 0.0703125"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/ab2/cur$i.json 2> gpurun_out/ab2/cur$i.log || exit 1
  NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_ab.so timeout -k 10 300 $B > gpurun_out/ab2/old$i.json 2> gpurun_out/ab2/old$i.log || exit 1
done
for f in cur1 old1 cur2 old2; do python3 -c "import json; d=json.load(open('gpurun_out/ab2/$f.json')); print('$f', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2))"; done
timeout -k 10 600 python bench.py --mode capi > gpurun_out/ab2/capi_on.json 2> gpurun_out/ab2/capi_on.log || exit 1
NGT_AMD_FILTER=0 timeout -k 10 600 python bench.py --mode capi > gpurun_out/ab2/capi_off.json 2> gpurun_out/ab2/capi_off.log || exit 1
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_ab.so timeout -k 10 600 python bench.py --mode capi > gpurun_out/ab2/capi_old.json 2> gpurun_out/ab2/capi_old.log || exit 1
for f in capi_on capi_off capi_old; do python3 -c "import json; d=json.load(open('gpurun_out/ab2/$f.json')); print('$f', round(d['value']), d['single_query_latency_ms'])"; done
