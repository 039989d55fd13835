#!/bin/bash
# round 6 d: the spill-trim test, then the driver's bench command (C2 headline
# + anng/capi + qg + c3 keys)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6d}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_qg.py::test_qg_spill_trim_at_capacity -m gpu > $O/trim.log 2>&1; tail -3 $O/trim.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log \
  || { tail -30 $O/bench.log; exit 1; }
python3 scripts/jline.py $O/bench.json bench
