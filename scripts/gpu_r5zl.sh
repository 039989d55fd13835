#!/bin/bash
# round 5: long cosine rows with 768 LDS unchecked keys -- parity suites, then
# the C3 line (sweep, parity sample, CPU baseline) as the driver's c3 key runs it
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5zl}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_production.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u bench.py --config c3 --steps 10 --warmup 2 --latency-queries 0 --anng-line off \
  --c3-line off > $O/c3.json 2> $O/c3.log || { tail -20 $O/c3.log; exit 1; }
python3 scripts/jline.py $O/c3.json c3
python3 -c "import json; d=json.load(open('$O/c3.json')); print(d['parity_sample'].get('identical'), d['cpu_baseline']['value'], d['roofline'].get('traffic'))"
