#!/bin/bash
# round 6: one rank's share of the N=2 scaling run (4 shards of 1.25M, exact
# then NGTQG form) on one GPU, to time what a driver --gpus 2 run asks of a rank
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 1000 python -u bench.py --gpus 1 --steps 20 --warmup 5 --shard-line on --shard-count 4 \
  --anng-line off --qg-line off --c3-line off > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('c2', round(d['value']))
s=d['shard']; print('shard', round(s['value']), s['config']['recall_at_10'], round(s['wall_s'],1), s['config']['setup_s'], (s.get('parity_sample') or {}).get('identical'))
q=s['qg_form']; print('qg_form', round(q['value']), q['config']['recall_at_10'], q['config']['quantize_s'], (q.get('parity_sample') or {}).get('identical'), q['scaling'])
"
