#!/bin/bash
# round 6 g: C5's per-GPU share as one graph (12.5M x 128 NGTQG over one device
# ANNG, -b 8000, tree seeds) after the visited-scratch fix, at the round-5
# epsilon, streams chosen by the bench (1 at this size), parity sample
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6g}; mkdir -p $O
timeout -k 10 900 python -u bench.py --mode qg --graph anng --n 12500000 --anng-batch 8000 --eps 0.12548828125 \
  --expansion 3 --steps 5 --warmup 1 --cpu-seconds 10 --latency-queries 0 --anng-line off --streams-ab 3 \
  > $O/c5.json 2> $O/c5.log || { tail -20 $O/c5.log; exit 1; }
python3 scripts/jline.py $O/c5.json c5
python3 -c "import json; d=json.load(open('$O/c5.json')); print(d['config']['streams'], d['config'].get('stream_ab_ms_per_step'), (d.get('parity_sample') or {}).get('identical'), (d.get('parity_sample') or {}).get('queries'))"
