#!/bin/bash
# ANNG device construction against batchSizeForCreation (ngt create -b): 1M
# objects at -b 2000 and 8000 (-b 200: 41.8 s, profiles/r4final), build time,
# recall/QPS of the ANNG line at 0.95
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zj}; mkdir -p $O
for B in ${BATCHES:-2000 8000}; do
  timeout -k 10 420 python -u bench.py --graph anng --n ${N:-1000000} --anng-batch $B --steps 5 --warmup 1 --no-cpu \
    --latency-queries 0 --anng-line off > $O/anng_b$B.json 2> $O/anng_b$B.log || { tail -20 $O/anng_b$B.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/anng_b$B.json')); print('b$B', round(d['value']), d['config']['recall_at_10'], d['config'].get('epsilon'), round(d['roofline']['kernel_ms'],1), round(d['roofline']['frac'],3), d['config'].get('graph_build_s'), (d.get('parity_sample') or {}).get('identical'))"
done
