#!/bin/bash
# C2 exact: the LDS visited cache in front of the HBM epochs (visited_hash_log2)
# x unchecked-array capacity, fixed epsilon, no CPU baseline.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "-1 1024" "10 512" "11 512" "10 1024" "9 768"; do
  set -- $cfg
  NGT_AMD_CQ_CAP=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --eps 0.0703125 --visited $1 > gpurun_out/vc_$1_$2.json 2> gpurun_out/vc_$1_$2.log || { echo "failed $cfg"; tail -20 gpurun_out/vc_$1_$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/vc_$1_$2.json').read().strip().splitlines()[-1]); print('$cfg', round(d['value']), d['roofline']['frac'], d['config'].get('recall'))"
done
