#!/bin/bash
# C2 A/B: touch loads in the pipelined filtered expansion (NGT_AMD_TOUCH
# 0/1/2/3 on the new build) against the committed build (libngt_amd_base.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3v
B="--steps 10 --warmup 2 --cpu-seconds 2 --eps 0.0703125 --latency-queries 0"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py $B > gpurun_out/r3v/$n.json 2> gpurun_out/r3v/$n.log || { tail -8 gpurun_out/r3v/$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r3v/$n.json')); r=d['roofline']; print('$n', round(d['value']), d['config']['recall_at_10'], 'kernel_ms', round(r['kernel_ms'],2), 'frac', round(r['frac'],3), 'step_ms', round(d['ms_per_step'],2), 'parity', d['parity_sample']['identical'])"
}
run base NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_base.so
run t0 NGT_AMD_TOUCH=0
run t1 NGT_AMD_TOUCH=1
run t3 NGT_AMD_TOUCH=3
run t7 NGT_AMD_TOUCH=7
run t5 NGT_AMD_TOUCH=5
exit 0
