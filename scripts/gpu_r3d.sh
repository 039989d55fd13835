#!/bin/bash
# lookahead kernel without chunk minima (targets removed at step start, the
# commit guard from the pushed keys): GPU suite, ANNG A/B (3 vs 4 waves per
# SIMD, P 3 vs 4), stamps, C2 single-query latency; QG line with the oracle
# LUT fix
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3d/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3d/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3d/pytest_gpu.log
D=/tmp/anng1m
B="--graph anng --anng-dir $D --steps 3 --warmup 1 --no-cpu --eps 0.1279296875 --latency-queries 20"
timeout -k 10 420 python -u bench.py $B > gpurun_out/r3d/anng_w3.json 2> gpurun_out/r3d/anng_w3.log || { tail -5 gpurun_out/r3d/anng_w3.log; exit 1; }
NGT_AMD_LA_WPE=4 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3d/anng_w4.json 2> gpurun_out/r3d/anng_w4.log || { tail -5 gpurun_out/r3d/anng_w4.log; exit 1; }
NGT_AMD_LA_P=4 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3d/anng_p4.json 2> gpurun_out/r3d/anng_p4.log || { tail -5 gpurun_out/r3d/anng_p4.log; exit 1; }
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python -u bench.py $B > gpurun_out/r3d/anng_stamps.json 2> gpurun_out/r3d/anng_stamps.log || { tail -5 gpurun_out/r3d/anng_stamps.log; exit 1; }
for f in anng_w3 anng_w4 anng_p4; do python3 -c "import json; d=json.load(open('gpurun_out/r3d/$f.json')); print('$f', round(d['value']), d['roofline']['kernel_ms'], d['single_query_latency']['mean_ms'])"; done
grep -h "phase\|discarded" gpurun_out/r3d/*.log
timeout -k 10 600 python -u bench.py --mode qg --cpu-seconds 10 > gpurun_out/r3d/bench_qg.json 2> gpurun_out/r3d/bench_qg.log \
  || { tail -5 gpurun_out/r3d/bench_qg.log; exit 1; }
cut -c1-300 gpurun_out/r3d/bench_qg.json
