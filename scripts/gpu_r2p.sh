#!/bin/bash
# Adjacency prefetch in every padded search: search/build/API parity, the 1M
# construction time, then the C2 bench line.
set -o pipefail
TAG=${1:-r2p}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_build.py \
  tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 \
  || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
NGT_AMD_BUILD_PROFILE=1 timeout -k 10 400 python scripts/build_bench.py --n 1000000 --check 500 \
  > gpurun_out/$TAG/build_1000000.json 2> gpurun_out/$TAG/build_1000000.log || { tail -5 gpurun_out/$TAG/build_1000000.log; exit 1; }
cat gpurun_out/$TAG/build_1000000.json; grep build_insert gpurun_out/$TAG/build_1000000.log
timeout -k 10 700 python bench.py > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.log || { tail -5 gpurun_out/$TAG/bench_c2.log; exit 1; }
grep -E "parity|accepted" gpurun_out/$TAG/bench_c2.log
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c2.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['config'].get('adjacency_prefetch_hits_per_expansion'))"
