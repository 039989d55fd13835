#!/bin/bash
# GPU parity suite, then C2 and C3 bench lines (no CPU baseline).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --eps 0.0703125 --no-cpu --steps 6 > gpurun_out/c2.json 2> gpurun_out/c2.log || exit $?
timeout -k 10 900 python bench.py --config c3 --eps 0.065625 --no-cpu --steps 3 --warmup 1 > gpurun_out/c3.json 2> gpurun_out/c3.log
rc=$?
for f in c2 c3; do python -c "
import json;d=json.load(open('gpurun_out/$f.json'));print('$f',round(d['value']),d['config']['recall_at_10'],round(d['roofline']['kernel_ms'],2),round(d['roofline']['frac'],3))"; done
exit $rc
