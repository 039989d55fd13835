#!/bin/bash
# the probe's prediction: C2 single search against the schedule's predictor and budget
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4n}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_schedule.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "0 0.12" "1 0.12" "2 0.12" "1 0.18" "0 0.18"; do
  set -- $cfg
  NGT_AMD_SCHED_PRIO=$1 NGT_AMD_SCHED_FRAC=$2 timeout -k 10 300 python -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 10 \
    > $O/c2_p$1_f$2.json 2> $O/c2_p$1_f$2.log || { tail -5 $O/c2_p$1_f$2.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_p$1_f$2.json')); print('prio $1 frac $2', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3))"
done
