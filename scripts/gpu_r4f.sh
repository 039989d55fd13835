#!/bin/bash
# probe-and-resume budget fraction sweep (C2 and ANNG)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4f}; mkdir -p $O
for f in 0.12 0.4; do
  NGT_AMD_SCHED_FRAC=$f timeout -k 10 300 python -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 10 \
    > $O/c2_f$f.json 2> $O/c2_f$f.log || { tail -5 $O/c2_f$f.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_f$f.json')); print('c2 f$f', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3))"
done
for f in 0.08 0.5; do
  NGT_AMD_SCHED_FRAC=$f timeout -k 10 400 python -u bench.py --graph anng --no-cpu --latency-queries 0 --anng-line off --steps 5 --warmup 2 \
    > $O/anng_f$f.json 2> $O/anng_f$f.log || { tail -5 $O/anng_f$f.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/anng_f$f.json')); print('anng f$f', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3))"
done
