#!/bin/bash
# the one-launch probe-and-resume schedule: its tests and the parity suites, then C2 with and without
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_parity.py tests/test_gpu_production.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sc in 1 0; do
  NGT_AMD_SCHED=$sc timeout -k 10 300 python -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 10 \
    > $O/c2_s$sc.json 2> $O/c2_s$sc.log || { tail -5 $O/c2_s$sc.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_s$sc.json')); print('sched$sc', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3), d['config']['recall_at_10'])"
done
