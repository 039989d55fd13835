#!/bin/bash
# C2 exact: LDS visited filter bits (NGT_AMD_VFILTER, log2) x unchecked-array
# capacity (NGT_AMD_CQ_CAP) at the fixed tuned epsilon.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in ${VF_CFGS:-"0 1024" "15 512" "16 512" "15 1024" "14 512"}; do
  set -- $cfg
  NGT_AMD_VFILTER=$1 NGT_AMD_CQ_CAP=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --eps 0.0703125 > gpurun_out/vf_$1_$2.json 2> gpurun_out/vf_$1_$2.log || { echo "failed $cfg"; tail -20 gpurun_out/vf_$1_$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/vf_$1_$2.json').read().strip().splitlines()[-1]); print('$cfg', round(d['value']), round(d['roofline']['frac'],4), d['config'].get('recall_at_10'), d['config'].get('distance_computations_per_query'))"
done
