#!/bin/bash
# Long-row code copy on 128-B lines + 512-key LDS unchecked arrays for long
# rows: parity, the C3 and C2 bench lines.
set -o pipefail
TAG=${1:-r2w}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 900 python -u bench.py --config c3 --steps 3 --warmup 1 > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.log || { tail -5 gpurun_out/$TAG/bench_c3.log; exit 1; }
grep -E "parity" gpurun_out/$TAG/bench_c3.log
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c3.json')); r=d['roofline']; print('c3', round(d['value']), d['config']['recall_at_10'], d['config']['epsilon'], r['kernel_ms'], r['frac'], r['frac_per_step'])"
timeout -k 10 700 python bench.py > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.log || { tail -5 gpurun_out/$TAG/bench_c2.log; exit 1; }
grep -E "parity" gpurun_out/$TAG/bench_c2.log
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c2.json')); r=d['roofline']; print('c2', round(d['value']), d['ms_per_step'], r['kernel_ms'], r['frac'], r['frac_per_step'])"
