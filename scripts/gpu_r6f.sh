#!/bin/bash
# round 6 f: smoke, the whole GPU suite, and a one-rank rehearsal of the N>1
# shard line with C5's NGTQG form over the same shards (2 shards of 250k)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6f}; mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --shard-line on --shard-count 2 --shard-n 250000 --anng-line off --c3-line off \
  --qg-line off --steps 5 --warmup 1 --latency-queries 0 --cpu-seconds 5 > $O/shard.json 2> $O/shard.log \
  || { tail -30 $O/shard.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/shard.json')); s=d['shard']; q=s.get('qg_form') or {}
print('shard', round(s['value']), s['config']['recall_at_10'], s['parity_sample'], '| qg_form', round(q.get('value', 0)), q.get('config', {}).get('recall_at_10'), q.get('parity_sample'))"
