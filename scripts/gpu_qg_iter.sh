#!/bin/bash
# QG + exact parity, then QG bench (+ stamps) and the default bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --mode qg --steps 5 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_qg.json 2> gpurun_out/bench_qg.log || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_qg.json')); print('qg', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3))"
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python -u bench.py --mode qg --steps 2 --warmup 1 --no-cpu --eps 0.05625 > gpurun_out/qg_stamps.json 2> gpurun_out/qg_stamps.log || exit 1
grep -E "phase" gpurun_out/qg_stamps.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --eps 0.0703125 > gpurun_out/bench_exact.json 2> gpurun_out/bench_exact.log || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_exact.json')); print('exact', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3))"
