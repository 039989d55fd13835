#!/bin/bash
# the default driver bench (C2 headline + the ANNG child line), then C2's
# single launch against resident waves per CU
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4b}; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); a=d.get('anng') or {}
print('c2', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['frac'],3), round(d['roofline']['kernel_ms'],2), d['parity_sample']['identical'])
print('anng', round(a.get('value',0)), a.get('config',{}).get('recall_at_10'), round(a.get('roofline',{}).get('frac',0),3), a.get('parity_sample',{}).get('identical'), a.get('child_wall_s'))"
bash scripts/gpu_r4_waves.sh ${1:-r4b}
