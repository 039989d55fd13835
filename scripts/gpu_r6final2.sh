#!/bin/bash
# round 6 final (2), the tree as committed after the issue-bound fields: smoke,
# the driver's bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=${1:-gpurun_out/r6final2}; case $O in gpurun_out/*) ;; *) O=gpurun_out/$O;; esac; mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log \
  || { tail -30 $O/bench.log; exit 1; }
python3 scripts/jline.py $O/bench.json bench
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('c2', d['roofline']['bound'])
for k in ('anng','qg','c3'):
    x=d[k]; print(k, round(x['value']), x['config']['recall_at_10'], round(x['roofline']['kernel_ms'],2), round(x['roofline']['frac'],3), x['roofline']['bound'], (x.get('parity_sample') or {}).get('identical'))
print('capi', d['anng']['capi']['qps_best'], d['anng']['capi']['threads_best'], d['anng']['capi']['single_thread_latency_ms']['mean'], d['anng']['capi']['reference_parity']['ids_identical_to_ngt_search'])
"
