#!/bin/bash
# one-expansion kernel: compaction only when expr changed -- its parity tests
# (small LDS arrays force the spill), the schedule tests, C3 and the C2 headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zo}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_schedule.py -m gpu > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 --cpu-seconds 5 --latency-queries 0 \
  > $O/bench_c3.json 2> $O/bench_c3.log || { tail -20 $O/bench_c3.log; exit 1; }
python3 scripts/jline.py $O/bench_c3.json
