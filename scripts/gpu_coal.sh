#!/bin/bash
# C-API group commit: batches in flight 2 (default) / 4 / 8
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/coal
for L in 2 4 8; do
  NGT_AMD_COALESCE_LEADERS=$L timeout -k 10 500 python bench.py --mode capi > gpurun_out/coal/l$L.json 2> gpurun_out/coal/l$L.log || { tail -5 gpurun_out/coal/l$L.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/coal/l$L.json')); print($L, round(d['value']), d['config']['mean_coalesced_batch'], d['single_query_latency_ms']['mean'])"
done
