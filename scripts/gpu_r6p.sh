#!/bin/bash
# round 6 p: EXPERIMENT -- the lookahead kernel's second target only when its
# distance is within a ratio of the first's (NGT_AMD_LA_RATIO), ANNG line at
# its epsilon; the lookahead suite with a ratio forced
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6p}; mkdir -p $O
NGT_AMD_LA_RATIO=1.02 timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_gpu_lookahead.py -m gpu > $O/pytest_la.log 2>&1 || { tail -30 $O/pytest_la.log; exit 1; }
tail -1 $O/pytest_la.log
D=/tmp/ngt_ab_anng_$$
A="--graph anng --anng-dir $D --capi-line off --eps 0.1279296875 --steps 10 --warmup 2 --latency-queries 0 --no-cpu"
for r in 1 2; do
  for ratio in 0 1.01 1.03 1.06 1.1; do
    NGT_AMD_TEST_KNOBS=1 NGT_AMD_LA_RATIO=$ratio timeout -k 10 400 python -u bench.py $A > $O/r${ratio}_$r.json \
      2> $O/r${ratio}_$r.log || { tail -20 $O/r${ratio}_$r.log; exit 1; }
    python3 scripts/jline.py $O/r${ratio}_$r.json ratio_${ratio}_$r
    grep -h "discarded" $O/r${ratio}_$r.log || true
  done
done
rm -rf $D
