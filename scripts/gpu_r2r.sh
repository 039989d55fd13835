#!/bin/bash
# Pipelined filtered expansion with the full visited set / small launches:
# parity, the C-API single-query latency, the C2 line, the device-ANNG line.
set -o pipefail
TAG=${1:-r2r}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_api.py \
  tests/test_cxx_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 \
  || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 600 python bench.py --mode capi > gpurun_out/$TAG/bench_capi.json 2> gpurun_out/$TAG/bench_capi.log || { tail -5 gpurun_out/$TAG/bench_capi.log; exit 1; }
cut -c1-200 gpurun_out/$TAG/bench_capi.json; python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_capi.json')); print(d['single_query_latency_ms'], d['config'].get('mean_coalesced_batch'))"
timeout -k 10 700 python bench.py > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.log || { tail -5 gpurun_out/$TAG/bench_c2.log; exit 1; }
grep -E "parity|accepted" gpurun_out/$TAG/bench_c2.log
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c2.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['frac_per_step'], d['config'].get('adjacency_prefetch_hits_per_expansion'))"
timeout -k 10 900 python -u bench.py --graph anng --anng-edges 10 --steps 5 --warmup 1 --eps 0.11,0.12,0.13,0.14,0.15,0.16 \
  > gpurun_out/$TAG/bench_anng_e10.json 2> gpurun_out/$TAG/bench_anng_e10.log || { tail -5 gpurun_out/$TAG/bench_anng_e10.log; exit 1; }
grep -E "ANNG|eps|parity" gpurun_out/$TAG/bench_anng_e10.log | tail -9
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_anng_e10.json')); print(round(d['value']), d['config']['recall_at_10'], d['config']['epsilon'], d['roofline']['frac'], d['cpu_baseline']['value'])"
