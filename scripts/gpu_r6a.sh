#!/bin/bash
# round 6 a: the changed kernels' suites (QG spill trim, latency kernel /
# serving grid at CUs-1 workers), then the new NGTQG line on the 1M ANNG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_qg.py \
  tests/test_gpu_serve.py tests/test_gpu_lookahead.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py --mode qg --graph anng --qg-expansions 2,3,4,6 --steps 5 --warmup 1 \
  --cpu-seconds 10 --latency-queries 0 --anng-line off --c3-line off --qg-line off > $O/qg.json 2> $O/qg.log \
  || { tail -30 $O/qg.log; exit 1; }
python3 scripts/jline.py $O/qg.json qg
