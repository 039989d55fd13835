#!/bin/bash
# LDS visited filter bits (NGT_AMD_VFILTER, log2) x unchecked-array capacity
# (NGT_AMD_CQ_CAP) at a fixed epsilon.  VF_CFGS="bits,cap ..."; MODE=exact|qg.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MODE=${MODE:-exact}
EPS=${EPS:-0.0703125}
for cfg in ${VF_CFGS:-"0,1024 15,512"}; do
  set -- ${cfg/,/ }
  NGT_AMD_VFILTER=$1 NGT_AMD_CQ_CAP=$2 timeout -k 10 300 python -u bench.py --mode $MODE --steps 5 --warmup 2 --no-cpu --eps $EPS > gpurun_out/vf_${MODE}_$1_$2.json 2> gpurun_out/vf_${MODE}_$1_$2.log || { echo "failed $cfg"; tail -20 gpurun_out/vf_${MODE}_$1_$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/vf_${MODE}_$1_$2.json').read().strip().splitlines()[-1]); print('$MODE $cfg', round(d['value']), round(d['roofline']['frac'],4), d['config'].get('recall_at_10'), d['config'].get('distance_computations_per_query'))"
done
