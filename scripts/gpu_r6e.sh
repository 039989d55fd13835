#!/bin/bash
# round 6 e: (1) counter passes of the qg key's configuration (NGTQG over the
# 1M ANNG, expansion 3, its epsilon); (2) C5's per-GPU share as one graph
# (12.5M NGTQG) under a kernel trace with the step timed over 3, 1 and 2
# streams (the step-inflation question of VERDICT r5 item 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6e}; mkdir -p $O
D=/tmp/ngt_pmc_anng_$$
PMC_LAST=3 bash scripts/pmc_r4.sh $O qg1m --mode qg --graph anng --anng-dir $D --eps 0.09772 \
  --expansion 3 --sweep-nq 10000 --pmc-launches 3 --no-cpu --anng-line off --c3-line off --qg-line off || exit 1
rm -rf $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5trace -o c5 --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --mode qg --graph anng --n 12500000 --anng-batch 8000 --eps 0.12548828125 \
  --expansion 3 --steps 3 --warmup 1 --no-cpu --latency-queries 0 --anng-line off --streams 3 --streams-ab 1,2,3 \
  > $GRAFT_REPO_ROOT/$O/c5.json 2> $GRAFT_REPO_ROOT/$O/c5.log || { tail -20 $GRAFT_REPO_ROOT/$O/c5.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/jline.py $O/c5.json c5
find $O/c5trace -name "*kernel_trace.csv" -exec cp {} $O/c5_kernel_trace.csv \;
find $O/c5trace -name "*kernel_stats.csv" -exec cp {} $O/c5_kernel_stats.csv \;
rm -rf $O/c5trace
grep "streams" $O/c5.log
