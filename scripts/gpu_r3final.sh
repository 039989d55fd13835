#!/bin/bash
# round-3 refresh on the committed tree: GPU suite, smoke, the default bench
# (C2 headline), the ANNG line (fresh reference-identical build, parity sample,
# reference fixture), the C-API line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3final/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3final/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3final/smoke.log 2>&1 || { tail -10 gpurun_out/r3final/smoke.log; exit 1; }
tail -1 gpurun_out/r3final/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3final/bench_c2.json 2> gpurun_out/r3final/bench_c2.log || { tail -10 gpurun_out/r3final/bench_c2.log; exit 1; }
timeout -k 10 600 python -u bench.py --graph anng --steps 5 --warmup 1 --cpu-seconds 10 --latency-queries 50 \
  > gpurun_out/r3final/bench_anng.json 2> gpurun_out/r3final/bench_anng.log || { tail -10 gpurun_out/r3final/bench_anng.log; exit 1; }
for f in bench_c2 bench_anng; do python3 -c "import json; d=json.load(open('gpurun_out/r3final/$f.json')); print('$f', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['frac'],3), d['roofline']['traffic'], d['parity_sample']['identical'], d['single_query_latency']['mean_ms'])"; done
