#!/bin/bash
# latency kernel: tests, single-query latencies with and without the
# adjacency-ordered filter codes, phase split (stamps build), C-API clients
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3h
D=/tmp/anng1m
S=$PWD/ngt_amd/libngt_amd_stamps.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookahead.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h/pytest_la.log 2>&1 || { tail -20 gpurun_out/r3h/pytest_la.log; exit 1; }
tail -1 gpurun_out/r3h/pytest_la.log
B="--steps 2 --warmup 1 --no-cpu --eps 0.0703125 --latency-queries 100"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h/c2.json 2> gpurun_out/r3h/c2.log || { tail -5 gpurun_out/r3h/c2.log; exit 1; }
NGT_AMD_NCODES=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h/c2_ncodes.json 2> gpurun_out/r3h/c2_ncodes.log || { tail -5 gpurun_out/r3h/c2_ncodes.log; exit 1; }
NGT_AMD_LIB=$S timeout -k 10 300 python -u bench.py $B > gpurun_out/r3h/c2_stamps.json 2> gpurun_out/r3h/c2_stamps.log || { tail -5 gpurun_out/r3h/c2_stamps.log; exit 1; }
A="--graph anng --anng-dir $D --steps 2 --warmup 1 --no-cpu --eps 0.1279296875 --latency-queries 30"
timeout -k 10 300 python -u bench.py $A > gpurun_out/r3h/anng.json 2> gpurun_out/r3h/anng.log || { tail -5 gpurun_out/r3h/anng.log; exit 1; }
NGT_AMD_LIB=$S timeout -k 10 300 python -u bench.py $A > gpurun_out/r3h/anng_stamps.json 2> gpurun_out/r3h/anng_stamps.log || { tail -5 gpurun_out/r3h/anng_stamps.log; exit 1; }
grep -h "single" gpurun_out/r3h/*.log
timeout -k 10 500 python -u bench.py --mode capi --threads 32 > gpurun_out/r3h/capi.json 2> gpurun_out/r3h/capi.log \
  || { tail -5 gpurun_out/r3h/capi.log; exit 1; }
grep -h "C client" gpurun_out/r3h/capi.log
