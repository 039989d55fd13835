#!/bin/bash
# the speculating latency kernel (NGT_AMD_LAT=1) and the 4-wave lookahead
# variant (NGT_AMD_LA_WPE=4): lookahead/latency tests first, then the whole
# GPU suite, then the ANNG line (fresh build through the latency kernel, parity
# sample, reference fixture) and the C2 line with single-query latencies
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3e
export NGT_AMD_LAT=1 NGT_AMD_LA_WPE=4
timeout -k 10 400 python -u -m pytest tests/test_gpu_lookahead.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3e/pytest_la.log 2>&1 || { tail -30 gpurun_out/r3e/pytest_la.log; exit 1; }
tail -2 gpurun_out/r3e/pytest_la.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3e/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3e/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3e/pytest_gpu.log
timeout -k 10 600 python -u bench.py --graph anng --steps 5 --warmup 1 --cpu-seconds 10 --latency-queries 50 \
  > gpurun_out/r3e/bench_anng.json 2> gpurun_out/r3e/bench_anng.log || { tail -10 gpurun_out/r3e/bench_anng.log; exit 1; }
grep -E "built|construction|single|parity|reference|discarded" gpurun_out/r3e/bench_anng.log
timeout -k 10 400 python -u bench.py --cpu-seconds 5 --latency-queries 100 \
  > gpurun_out/r3e/bench_c2.json 2> gpurun_out/r3e/bench_c2.log || { tail -10 gpurun_out/r3e/bench_c2.log; exit 1; }
grep -E "single|parity" gpurun_out/r3e/bench_c2.log
for f in bench_anng bench_c2; do python3 -c "import json; d=json.load(open('gpurun_out/r3e/$f.json')); print('$f', round(d['value']), d['roofline']['frac'], d['single_query_latency'])"; done
