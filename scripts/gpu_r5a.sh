#!/bin/bash
# round 5, first box: the serving-grid regression tests (mutations under
# served calls, fresh stream error words), schedule + shard suites, and the
# bench's shard line on a small index (one rank, 4 shards)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5a}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_serve.py \
  tests/test_gpu_schedule.py tests/test_gpu_shard.py tests/test_ngtpy.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u bench.py --n 200000 --shard-line on --shard-n 100000 --shard-count 4 --anng-line off \
  --steps 5 --warmup 2 --latency-queries 5 --cpu-seconds 3 > $O/bench_shard.json 2> $O/bench_shard.log \
  || { tail -30 $O/bench_shard.log; exit 1; }
python3 scripts/jline.py $O/bench_shard.json
