#!/bin/bash
# round 6 z (final): the whole GPU suite, the smoke, the driver's bench command,
# then a kernel trace of the C2 headline's timed configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6z}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash scripts/gpu_r6final2.sh $O || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/c2trace -o c2 --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --anng-line off --qg-line off --c3-line off --latency-queries 0 \
  > $R/$O/c2trace.json 2> $R/$O/c2trace.log || { tail -20 $R/$O/c2trace.log; exit 1; }
cd $R && find $O/c2trace -name "*kernel_stats.csv" -exec cp {} $O/c2_kernel_stats.csv \; && rm -rf $O/c2trace
head -5 $O/c2_kernel_stats.csv | cut -c1-200
