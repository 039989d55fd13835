#!/bin/bash
# ANNG (1M x 128, E=10, the prf's edge size 40, tree seeds) investigation: the
# product lookahead kernel, its per-phase stamps (diagnostic build), and the
# one-expansion kernel (NGT_AMD_LA=0) on the same index, built once per call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3a
D=/tmp/anng1m
EPS=${EPS:-0.1279296875}
timeout -k 10 420 python -u bench.py --graph anng --anng-dir $D --steps 3 --warmup 1 --no-cpu --eps $EPS \
  --latency-queries 20 > gpurun_out/r3a/anng.json 2> gpurun_out/r3a/anng.log || { tail -5 gpurun_out/r3a/anng.log; exit 1; }
grep -E "lookahead|single|eps" gpurun_out/r3a/anng.log
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python -u bench.py --graph anng --anng-dir $D --steps 1 \
  --warmup 1 --no-cpu --eps $EPS --latency-queries 20 > gpurun_out/r3a/anng_stamps.json 2> gpurun_out/r3a/anng_stamps.log \
  || { tail -5 gpurun_out/r3a/anng_stamps.log; exit 1; }
grep -E "phase|single|eps" gpurun_out/r3a/anng_stamps.log
NGT_AMD_LA=0 timeout -k 10 300 python -u bench.py --graph anng --anng-dir $D --steps 2 --warmup 1 --no-cpu --eps $EPS \
  --latency-queries 20 > gpurun_out/r3a/anng_la0.json 2> gpurun_out/r3a/anng_la0.log || { tail -5 gpurun_out/r3a/anng_la0.log; exit 1; }
grep -E "single|eps" gpurun_out/r3a/anng_la0.log
for f in anng anng_la0; do python3 -c "import json; d=json.load(open('gpurun_out/r3a/$f.json')); print('$f', round(d['value']), d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
