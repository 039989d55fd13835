#!/bin/bash
# the tree as committed at the round's end: smoke, the one-expansion parity
# tests, a short C2 headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zr}; mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_build.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --anng-line off --cpu-seconds 5 > $O/bench.json 2> $O/bench.log \
  || { tail -20 $O/bench.log; exit 1; }
python3 scripts/jline.py $O/bench.json
