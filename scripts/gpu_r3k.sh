#!/bin/bash
# lookahead form at 2 targets per step (default now) vs 1; latency kernel with
# 9-10 filter groups in flight; lookahead/latency tests; ANNG PMC at the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3k
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_production.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3k/pytest.log 2>&1 || { tail -20 gpurun_out/r3k/pytest.log; exit 1; }
tail -1 gpurun_out/r3k/pytest.log
D=/tmp/anng1m
A="--graph anng --anng-dir $D --steps 3 --warmup 1 --no-cpu --eps 0.1279296875 --latency-queries 30"
timeout -k 10 400 python -u bench.py $A > gpurun_out/r3k/anng_p2.json 2> gpurun_out/r3k/anng_p2.log || { tail -5 gpurun_out/r3k/anng_p2.log; exit 1; }
NGT_AMD_LA_P=1 timeout -k 10 300 python -u bench.py $A > gpurun_out/r3k/anng_p1.json 2> gpurun_out/r3k/anng_p1.log || { tail -5 gpurun_out/r3k/anng_p1.log; exit 1; }
for f in anng_p2 anng_p1; do python3 -c "import json; d=json.load(open('gpurun_out/r3k/$f.json')); print('$f', round(d['value']), d['roofline']['kernel_ms'], d['single_query_latency']['mean_ms'])"; done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --eps 0.0703125 --latency-queries 100 \
  > gpurun_out/r3k/c2.json 2> gpurun_out/r3k/c2.log || { tail -5 gpurun_out/r3k/c2.log; exit 1; }
grep -h "single" gpurun_out/r3k/*.log
bash scripts/pmc_r3.sh gpurun_out/r3k anng --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 \
  --pmc-launches 6 --no-cpu || exit 1
