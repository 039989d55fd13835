#!/bin/bash
# NGTQG on a low-degree quantized graph (12.5M over one ANNG, ~42 edges per
# node of 128 slots): code blocks loaded with the id row (default) against
# ids first, then only the blocks of the degree (NGT_AMD_QG_TWO_TRIPS=1);
# the QG suite with the two-trip form first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zq}; mkdir -p $O
NGT_AMD_QG_TWO_TRIPS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_qg.py -m gpu > $O/pytest_qg_two.log 2>&1 || { tail -30 $O/pytest_qg_two.log; exit 1; }
tail -1 $O/pytest_qg_two.log
A="--mode qg --graph anng --n 12500000 --anng-batch 8000 --eps 0.12548828125 --steps 3 --warmup 1 --no-cpu --latency-queries 0 --anng-line off"
timeout -k 10 330 python -u bench.py $A > $O/c5_one.json 2> $O/c5_one.log || { tail -20 $O/c5_one.log; exit 1; }
python3 scripts/jline.py $O/c5_one.json
NGT_AMD_QG_TWO_TRIPS=1 timeout -k 10 330 python -u bench.py $A > $O/c5_two.json 2> $O/c5_two.log || { tail -20 $O/c5_two.log; exit 1; }
python3 scripts/jline.py $O/c5_two.json
