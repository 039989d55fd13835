#!/bin/bash
# NGTQG kernel with chunk minima over its HBM spill: the QG parity suite, the
# C2-graph NGTQG line (1M, kNN graph), then C5's 12.5M one-ANNG NGTQG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zn}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_qg.py -m gpu \
  > $O/pytest_qg.log 2>&1 || { tail -30 $O/pytest_qg.log; exit 1; }
tail -2 $O/pytest_qg.log
timeout -k 10 300 python -u bench.py --mode qg --steps 10 --warmup 2 --cpu-seconds 5 --latency-queries 0 \
  > $O/bench_qg.json 2> $O/bench_qg.log || { tail -20 $O/bench_qg.log; exit 1; }
python3 scripts/jline.py $O/bench_qg.json
NS=12500000 B=8000 T=${T:-720} bash scripts/gpu_r4zm.sh ${1:-r4zn}
