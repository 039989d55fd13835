#!/bin/bash
# C2 single-launch time against resident waves per CU (the launch's tail:
# 10k queries over 256 x W slots), and the ANNG line at the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4w}; mkdir -p $O
for w in 16 12 14 10; do
  NGT_AMD_WAVES_PER_CU=$w timeout -k 10 300 python -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 10 \
    > $O/c2_w$w.json 2> $O/c2_w$w.log || { tail -5 $O/c2_w$w.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_w$w.json')); print('w$w', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3), d['config']['recall_at_10'])"
done
