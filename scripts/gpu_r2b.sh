#!/bin/bash
# Round-2 GPU pass: full pytest -m gpu, default bench line, the C-API
# latency/concurrency line and the 1-GPU C5-form (sharded NGTQG) line.
TAG=${1:-r2b}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.log || exit $?
tail -3 gpurun_out/$TAG/bench.log; cat gpurun_out/$TAG/bench.json
timeout -k 10 600 python bench.py --mode capi > gpurun_out/$TAG/bench_capi.json 2> gpurun_out/$TAG/bench_capi.log || exit $?
tail -3 gpurun_out/$TAG/bench_capi.log; cat gpurun_out/$TAG/bench_capi.json
timeout -k 10 600 python bench.py --mode shard --qg --no-cpu > gpurun_out/$TAG/bench_shard_qg.json \
  2> gpurun_out/$TAG/bench_shard_qg.log || exit $?
tail -3 gpurun_out/$TAG/bench_shard_qg.log; cat gpurun_out/$TAG/bench_shard_qg.json
