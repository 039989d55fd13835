#!/bin/bash
# round 6 v: why the serving grid relaunches under 256 C callers (grid log on)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=${1:-gpurun_out/r6v}; case $O in gpurun_out/*) ;; *) O=gpurun_out/$O;; esac; mkdir -p $O
D=/tmp/ngt_v_anng_$$
NGT_AMD_TEST_KNOBS=1 NGT_AMD_SERVE_LOG=1 timeout -k 10 600 python3 -u bench.py --graph anng --anng-dir $D \
  --eps 0.1279296875 --sweep-nq 10000 --steps 2 --warmup 1 --no-cpu --latency-queries 0 > $O/anng.json 2> $O/anng.log \
  || { tail -20 $O/anng.log; exit 1; }
grep "C client" $O/anng.log | tail -40
nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
rm -rf $D
