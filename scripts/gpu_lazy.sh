#!/bin/bash
# A/B: visited set holding every evaluated id vs accepted ids only (C2).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A="--eps 0.0703125 --no-cpu --steps 6"
timeout -k 10 300 python bench.py $A > gpurun_out/lazy0.json 2> gpurun_out/lazy0.log &&
NGT_AMD_ACCEPTED_ONLY=1 timeout -k 10 300 python bench.py $A > gpurun_out/lazy1.json 2> gpurun_out/lazy1.log &&
NGT_AMD_ACCEPTED_ONLY=1 NGT_AMD_VFILTER=16 NGT_AMD_CQ_CAP=512 timeout -k 10 300 python bench.py $A > gpurun_out/lazy2.json 2> gpurun_out/lazy2.log
rc=$?
for f in lazy0 lazy1 lazy2; do grep "eps" gpurun_out/$f.log | tail -1; python -c "
import json;d=json.load(open('gpurun_out/$f.json'));print('$f',round(d['value']),d['config']['recall_at_10'],d['config']['distance_computations_per_query'],d['roofline']['kernel_ms'])"; done
exit $rc
