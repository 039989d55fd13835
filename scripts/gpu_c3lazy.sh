#!/bin/bash
# C3 with the accepted-only visited set behind an LDS filter (experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c3lazy
B="python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu --eps 0.06523437500000001"
for VF in 15 14; do
  NGT_AMD_ACCEPTED_ONLY=1 NGT_AMD_VFILTER=$VF timeout -k 10 400 $B > gpurun_out/c3lazy/vf$VF.json 2> gpurun_out/c3lazy/vf$VF.log || { tail -5 gpurun_out/c3lazy/vf$VF.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c3lazy/vf$VF.json')); r=d['roofline']; print($VF, round(d['value']), d['config']['recall_at_10'], r['kernel_ms'], d['ms_per_step'], d['config'].get('evaluations_per_query'))"
done
