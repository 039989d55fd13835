#!/bin/bash
# round 6 j: the record-speculating NGTQG form (quarter records, NB = 4) --
# the QG suite with it forced on, then an interleaved A/B on the qg key's
# configuration (knob NGT_AMD_QG_SPEC), the speculating runs with parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6j}; mkdir -p $O
NGT_AMD_QG_SPEC=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_qg.py \
  -m gpu > $O/pytest_qg_spec.log 2>&1 || { tail -30 $O/pytest_qg_spec.log; exit 1; }
tail -1 $O/pytest_qg_spec.log
D=/tmp/ngt_ab_anng_$$
A="--mode qg --graph anng --anng-dir $D --eps 0.09772 --expansion 3 --steps 10 --warmup 2 --latency-queries 0 --anng-line off --c3-line off --qg-line off"
for r in 1 2; do
  for v in 0 1; do
    C="--no-cpu"; [ $v = 1 ] && [ $r = 1 ] && C="--cpu-seconds 8"
    NGT_AMD_TEST_KNOBS=1 NGT_AMD_QG_SPEC=$v timeout -k 10 400 python -u bench.py $A $C > $O/spec${v}_$r.json \
      2> $O/spec${v}_$r.log || { tail -20 $O/spec${v}_$r.log; exit 1; }
    python3 scripts/jline.py $O/spec${v}_$r.json spec${v}_$r
    grep -h "parity" $O/spec${v}_$r.log || true
  done
done
python3 -c "
import json, numpy as np
" 
rm -rf $D
