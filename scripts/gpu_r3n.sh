#!/bin/bash
# latency kernel (parts of 32 exact rows): phase split (stamps build) on C2
# and ANNG, and the slot count's effect on C2 single-query latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3n
D=/tmp/anng1m
S=$PWD/ngt_amd/libngt_amd_stamps.so
B="--steps 1 --warmup 1 --no-cpu --eps 0.0703125 --latency-queries 100"
NGT_AMD_LIB=$S timeout -k 10 300 python -u bench.py $B > gpurun_out/r3n/c2_stamps.json 2> gpurun_out/r3n/c2_stamps.log || { tail -5 gpurun_out/r3n/c2_stamps.log; exit 1; }
for n in 8 32; do
NGT_AMD_LAT_SLOTS=$n timeout -k 10 300 python -u bench.py $B > gpurun_out/r3n/c2_s$n.json 2> gpurun_out/r3n/c2_s$n.log || { tail -5 gpurun_out/r3n/c2_s$n.log; exit 1; }
done
A="--graph anng --anng-dir $D --steps 1 --warmup 1 --no-cpu --eps 0.1279296875 --latency-queries 20"
NGT_AMD_LIB=$S timeout -k 10 400 python -u bench.py $A > gpurun_out/r3n/anng_stamps.json 2> gpurun_out/r3n/anng_stamps.log || { tail -5 gpurun_out/r3n/anng_stamps.log; exit 1; }
grep -h "single" gpurun_out/r3n/*.log
