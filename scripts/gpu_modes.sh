#!/bin/bash
# GPU parity (QG + shard) then one short bench per mode, each under its own limit.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_qg.py tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_modes.log 2>&1 || { tail -30 gpurun_out/pytest_modes.log; exit 1; }
tail -2 gpurun_out/pytest_modes.log
for m in "exact" "qg" "shard"; do
  timeout -k 10 500 python -u bench.py --mode $m --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.log || { echo "bench $m failed"; tail -20 gpurun_out/bench_$m.log; exit 1; }
  cut -c1-600 gpurun_out/bench_$m.json
done
