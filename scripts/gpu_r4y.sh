#!/bin/bash
# lookahead kernel (register head of the unchecked set; survivors collected in the filter pass), list
# offsets from registers -- parity, then the ANNG line's launch time
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4y}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lookahead.py \
  tests/test_gpu_parity.py tests/test_gpu_production.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
D=/tmp/anng_r4y
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 3 --warmup 1 \
  --no-cpu --latency-queries 0 --anng-line off > $O/anng.json 2> $O/anng.log || { tail -5 $O/anng.log; exit 1; }
python3 scripts/jline.py $O/anng.json anng
grep -E "identical|evaluations" $O/anng.log
