#!/bin/bash
# the deferred visited test (lookahead and one-expansion kernels): parity suites, then C2 and ANNG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4i}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_production.py tests/test_gpu_build.py tests/test_gpu_serve.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 10 > $O/c2.json 2> $O/c2.log || { tail -5 $O/c2.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3), d['config']['recall_at_10'], d['config'].get('evaluations_per_query'))"
timeout -k 10 400 python -u bench.py --graph anng --no-cpu --latency-queries 0 --anng-line off --steps 5 --warmup 2 \
    > $O/anng.json 2> $O/anng.log || { tail -5 $O/anng.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/anng.json')); print('anng', round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3), d['config']['recall_at_10'], d['config'].get('evaluations_per_query'))"
