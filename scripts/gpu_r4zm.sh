#!/bin/bash
# C5's per-GPU share (12.5M x 128 NGTQG) over ONE device-built ANNG on one GPU
# (ngt create -b $B, then ngtqg quantize on the device), after a 200k check run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zm}; mkdir -p $O
B=${B:-8000}
for N in ${NS:-200000 12500000}; do
  timeout -k 10 ${T:-960} python -u bench.py --mode qg --graph anng --n $N --anng-batch $B --steps 3 --warmup 1 \
    --cpu-seconds 10 --latency-queries 0 --anng-line off > $O/c5_onegraph_$N.json 2> $O/c5_onegraph_$N.log \
    || { tail -20 $O/c5_onegraph_$N.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_onegraph_$N.json')); print('c5', $N, round(d['value']), d['config']['recall_at_10'], round(d['roofline']['kernel_ms'],1), round(d['roofline']['frac'],3), d['config'].get('graph_build_s'), (d.get('parity_sample') or {}).get('identical'))"
done
