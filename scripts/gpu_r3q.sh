#!/bin/bash
# full GPU suite with the serving grid in the C-API path, smoke, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3q/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3q/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3q/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3q/smoke.log 2>&1 || { tail -5 gpurun_out/r3q/smoke.log; exit 1; }
tail -1 gpurun_out/r3q/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3q/bench_c2.json 2> gpurun_out/r3q/bench_c2.log || { tail -5 gpurun_out/r3q/bench_c2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3q/bench_c2.json')); print(round(d['value']), d['roofline']['frac'], d.get('single_query_latency'))"
