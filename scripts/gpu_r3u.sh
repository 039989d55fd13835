#!/bin/bash
# re-entry refresh of the committed tree (latency kernel with per-part
# readiness and hop pool): GPU suite, smoke, the default bench (C2 headline),
# the C-API line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3u/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3u/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3u/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3u/smoke.log 2>&1 || { tail -10 gpurun_out/r3u/smoke.log; exit 1; }
tail -1 gpurun_out/r3u/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3u/bench_c2.json 2> gpurun_out/r3u/bench_c2.log || { tail -10 gpurun_out/r3u/bench_c2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3u/bench_c2.json')); print('c2', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['frac'],3), d['roofline']['kernel_ms'], d['parity_sample']['identical'], d['single_query_latency']['mean_ms'])"
timeout -k 10 400 python -u bench.py --mode capi --no-cpu --eps 0.0703125 \
  > gpurun_out/r3u/capi.json 2> gpurun_out/r3u/capi.log || { tail -5 gpurun_out/r3u/capi.log; exit 1; }
grep -h "C client" gpurun_out/r3u/capi.log
exit 0
