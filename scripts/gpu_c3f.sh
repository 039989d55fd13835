#!/bin/bash
# Cosine filter parity and a C3 timing at the bench epsilon.
set -o pipefail
TAG=${1:-c3f}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests/test_gpu_production.py -k cosine -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 600 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu --eps 0.06523437500000001 > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.log || { tail -5 gpurun_out/$TAG/bench_c3.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c3.json')); r=d['roofline']; print(round(d['value']), d['config']['recall_at_10'], r['kernel_ms'], r['frac'], d['ms_per_step'])"
