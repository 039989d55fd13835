#!/bin/bash
# latency kernel with per-part readiness and the hop pool: tests, single-query
# latency (pool 8 vs 0) on C2 and the ANNG, the C-API line, suite-order check
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3t
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_serve.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3t/pytest.log 2>&1 || { tail -30 gpurun_out/r3t/pytest.log; exit 1; }
tail -1 gpurun_out/r3t/pytest.log
B="--steps 1 --warmup 1 --no-cpu --eps 0.0703125 --latency-queries 200"
for pool in 8 0; do
NGT_AMD_LAT_POOL=$pool timeout -k 10 300 python -u bench.py $B > gpurun_out/r3t/c2_p$pool.json 2> gpurun_out/r3t/c2_p$pool.log || { tail -5 gpurun_out/r3t/c2_p$pool.log; exit 1; }
echo "pool $pool: $(grep -h 'single' gpurun_out/r3t/c2_p$pool.log | head -2 | tr '\n' ' ')"
done
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python -u bench.py $B > gpurun_out/r3t/c2_stamps.json 2> gpurun_out/r3t/c2_stamps.log || { tail -5 gpurun_out/r3t/c2_stamps.log; exit 1; }
grep -h "single-query phase" gpurun_out/r3t/c2_stamps.log
timeout -k 10 400 python -u bench.py --mode capi --no-cpu --eps 0.0703125 \
  > gpurun_out/r3t/capi.json 2> gpurun_out/r3t/capi.log || { tail -5 gpurun_out/r3t/capi.log; exit 1; }
grep -h "C client" gpurun_out/r3t/capi.log
A="--graph anng --anng-dir /tmp/anng1m --steps 1 --warmup 1 --no-cpu --eps 0.1279296875 --latency-queries 30"
for pool in 8 0; do
NGT_AMD_LAT_POOL=$pool timeout -k 10 400 python -u bench.py $A > gpurun_out/r3t/anng_p$pool.json 2> gpurun_out/r3t/anng_p$pool.log || { tail -5 gpurun_out/r3t/anng_p$pool.log; exit 1; }
echo "anng pool $pool: $(grep -h 'single' gpurun_out/r3t/anng_p$pool.log | head -2 | tr '\n' ' ')"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_serve.py -q --timeout 200 --timeout-method thread > gpurun_out/r3t/scan_serve.log 2>&1
echo "scan+serve rc=$?"; tail -2 gpurun_out/r3t/scan_serve.log; grep -h "batch search failed" gpurun_out/r3t/scan_serve.log | head -3
exit 0
