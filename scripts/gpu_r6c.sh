#!/bin/bash
# round 6 c: the spill-trim test, then the NGTQG line on the 1M ANNG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6c}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_qg.py::test_qg_spill_trim_at_capacity -m gpu > $O/trim.log 2>&1; tail -5 $O/trim.log
timeout -k 10 600 python -u bench.py --mode qg --graph anng --qg-expansions 2,3,4,6 --steps 5 --warmup 1 \
  --cpu-seconds 10 --latency-queries 0 --anng-line off --c3-line off --qg-line off > $O/qg.json 2> $O/qg.log \
  || { tail -30 $O/qg.log; exit 1; }
python3 scripts/jline.py $O/qg.json qg
