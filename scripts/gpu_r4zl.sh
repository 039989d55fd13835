#!/bin/bash
# C4's 10M x 128 as ONE device-built ANNG on one GPU with a larger creation
# batch (ngt create -b $B): build, tree seeds, prf edge size 40, recall 0.95
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zl}; mkdir -p $O
B=${B:-4000}
timeout -k 10 1050 python -u bench.py --graph anng --n ${N:-10000000} --anng-batch $B --steps 3 --warmup 1 \
  --cpu-seconds 10 --latency-queries 0 --anng-line off > $O/c4_onegraph_b$B.json 2> $O/c4_onegraph_b$B.log \
  || { tail -20 $O/c4_onegraph_b$B.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4_onegraph_b$B.json')); print('c4', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['kernel_ms'],1), round(d['roofline']['frac'],3), d['config'].get('graph_build_s'), (d.get('parity_sample') or {}).get('identical'))"
