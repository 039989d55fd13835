#!/bin/bash
# round-4 state: the full GPU suite, smoke, the driver's default bench (C2 headline + ANNG line)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4final}; mkdir -p $O
bash scripts/gpu_r4.sh ${1:-r4final} || exit 1
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 scripts/jline.py $O/bench.json c2
python3 -c "
import json; d=json.load(open('$O/bench.json')); a=d.get('anng') or {}
print('c2 parity', d['parity_sample'].get('identical'), 'cpu', d['cpu_baseline']['value'])
print('anng', round(a.get('value',0)), a.get('config',{}).get('recall_at_10'), round(a.get('roofline',{}).get('frac',0),3), round(a.get('roofline',{}).get('kernel_ms',0),2), (a.get('parity_sample') or {}).get('identical'), round(a.get('child_wall_s',0)))"
