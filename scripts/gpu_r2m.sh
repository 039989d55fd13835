#!/bin/bash
# Pipelined filtered expansion: parity (filter on == off, production config vs
# oracle, search parity suite), stamps, then the C2 bench line.
set -o pipefail
TAG=${1:-r2m}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --eps 0.0703125 \
  > gpurun_out/$TAG/stamps.json 2> gpurun_out/$TAG/stamps.log || { tail -5 gpurun_out/$TAG/stamps.log; exit 1; }
grep -E "phase|expansions" gpurun_out/$TAG/stamps.log
timeout -k 10 700 python bench.py > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.log || { tail -5 gpurun_out/$TAG/bench_c2.log; exit 1; }
grep -E "parity|accepted" gpurun_out/$TAG/bench_c2.log; cut -c1-300 gpurun_out/$TAG/bench_c2.json
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c2.json')); print(d['roofline'])"
