#!/bin/bash
# error 16 in the served latency kernel (test_cxx_search_matches_reference on
# the C1 ANNG, hop pool of 8): pool 8 with the own-slot steal vs off; then, with the pool off, the whole
# GPU suite, smoke, the C2 bench and the C-API line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3w
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for pool in 8 0; do
  NGT_AMD_LAT_POOL=$pool $T tests/test_cxx_api.py > gpurun_out/r3w/cxx_p$pool.log 2>&1
  echo "cxx pool $pool rc=$? $(tail -1 gpurun_out/r3w/cxx_p$pool.log)"
done
# the default is now 0 (no env needed)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3w/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3w/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3w/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3w/smoke.log 2>&1 || { tail -10 gpurun_out/r3w/smoke.log; exit 1; }
tail -1 gpurun_out/r3w/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3w/bench_c2.json 2> gpurun_out/r3w/bench_c2.log || { tail -10 gpurun_out/r3w/bench_c2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3w/bench_c2.json')); print('c2', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['frac'],3), d['roofline']['kernel_ms'], d['parity_sample']['identical'], d['single_query_latency']['mean_ms'])"
timeout -k 10 400 python -u bench.py --mode capi --no-cpu --eps 0.0703125 \
  > gpurun_out/r3w/capi.json 2> gpurun_out/r3w/capi.log || { tail -5 gpurun_out/r3w/capi.log; exit 1; }
grep -h "C client" gpurun_out/r3w/capi.log
# the pool with the own-slot steal: lookahead/latency and serving tests at 8 slots
NGT_AMD_LAT_POOL=8 $T tests/test_gpu_lookahead.py tests/test_gpu_serve.py tests/test_gpu_api.py > gpurun_out/r3w/la_p8.log 2>&1
echo "lookahead/serve/api pool 8 rc=$? $(tail -1 gpurun_out/r3w/la_p8.log)"
exit 0
