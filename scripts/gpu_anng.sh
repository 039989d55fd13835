#!/bin/bash
# C2 search over this library's own ANNG (ngt_create_index on the device, E=10
# and E=40) instead of the setup kNN graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/anng
for E in ${@:-10}; do
  timeout -k 10 900 python -u bench.py --graph anng --anng-edges $E --steps 5 --warmup 1 \
    > gpurun_out/anng/bench_anng_e$E.json 2> gpurun_out/anng/bench_anng_e$E.log || { tail -5 gpurun_out/anng/bench_anng_e$E.log; exit 1; }
  grep -E "ANNG|eps|parity" gpurun_out/anng/bench_anng_e$E.log | tail -6
  python3 -c "import json; d=json.load(open('gpurun_out/anng/bench_anng_e$E.json')); print(round(d['value']), d['config']['recall_at_10'], d['config']['epsilon'], d['roofline']['frac'], d['cpu_baseline']['value'])"
done
