#!/bin/bash
# QG: parity tests, then A/B: early probes (default) / no filter / two round trips.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qg.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_qg.log; [ $rc -eq 0 ] || exit $rc
A="--mode qg --eps 0.05625 --no-cpu --steps 6"
timeout -k 10 400 python bench.py $A > gpurun_out/qg_new.json 2> gpurun_out/qg_new.log &&
NGT_AMD_VFILTER=0 timeout -k 10 400 python bench.py $A > gpurun_out/qg_nof.json 2> gpurun_out/qg_nof.log &&
NGT_AMD_QG_TWO_TRIPS=1 NGT_AMD_VFILTER=0 timeout -k 10 400 python bench.py $A > gpurun_out/qg_old.json 2> gpurun_out/qg_old.log
rc=$?
for f in qg_new qg_nof qg_old; do python -c "
import json;d=json.load(open('gpurun_out/$f.json'));print('$f',round(d['value']),d['config']['recall_at_10'],d['roofline']['kernel_ms'],d['roofline']['frac'])"; done
exit $rc
