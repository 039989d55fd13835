#!/bin/bash
# Cosine/angle long-row filter: parity, then the C3 bench line.
set -o pipefail
TAG=${1:-r2t}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 900 python -u bench.py --config c3 --steps 3 --warmup 1 > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.log || { tail -5 gpurun_out/$TAG/bench_c3.log; exit 1; }
grep -E "eps|parity" gpurun_out/$TAG/bench_c3.log | tail -8
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c3.json')); r=d['roofline']; print(round(d['value']), d['config']['recall_at_10'], d['config']['epsilon'], r['kernel_ms'], r['frac'], d['config'].get('exact_neighbour_distances_per_query'), d['config']['distance_computations_per_query'])"
