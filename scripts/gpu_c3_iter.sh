#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 900 python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.log || { tail gpurun_out/bench_c3.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_c3.json')); print('c3', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3))"
