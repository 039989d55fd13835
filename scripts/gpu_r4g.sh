#!/bin/bash
# the full GPU suite, smoke, the default driver bench, and C2 at a smaller budget fraction
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4g}; mkdir -p $O
bash scripts/gpu_r4.sh ${1:-r4g} || exit 1
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); a=d.get('anng') or {}
print('c2', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['frac'],3), round(d['roofline']['kernel_ms'],2), d['parity_sample']['identical'])
print('anng', round(a.get('value',0)), a.get('config',{}).get('recall_at_10'), round(a.get('roofline',{}).get('frac',0),3), a.get('parity_sample',{}).get('identical'), a.get('child_wall_s'))"
NGT_AMD_SCHED_FRAC=0.06 timeout -k 10 300 python -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 10 \
    > $O/c2_f0.06.json 2> $O/c2_f0.06.log || { tail -5 $O/c2_f0.06.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2_f0.06.json')); print('c2 f0.06', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3))"
