#!/bin/bash
# round-4 state: the full GPU suite twice (flakiness), smoke, the driver's default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4p}; mkdir -p $O
bash scripts/gpu_r4.sh ${1:-r4p} || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_2.log 2>&1 || { tail -40 $O/pytest_gpu_2.log; exit 1; }
tail -1 $O/pytest_gpu_2.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); a=d.get('anng') or {}
print('c2', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['frac'],3), round(d['roofline']['kernel_ms'],2), d['roofline'].get('traffic'), d['parity_sample']['identical'])
print('anng', round(a.get('value',0)), a.get('config',{}).get('recall_at_10'), round(a.get('roofline',{}).get('frac',0),3), a.get('parity_sample',{}).get('identical'), a.get('child_wall_s'))"
