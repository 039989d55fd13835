#!/bin/bash
# round 5: long cosine/angle rows at 3 waves per SIMD (parity suites), then
# the C2 headline kernel at 4 (product) and 3 waves per SIMD (no spills),
# interleaved twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5ze}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_production.py tests/test_gpu_schedule.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$PWD/ngt_amd
for rep in a b; do
  for v in w4 w3; do
    lib=$L/libngt_amd.so; [ $v = w3 ] && lib=$L/libngt_amd_c2w3.so
    NGT_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --latency-queries 0 \
      --anng-line off --c3-line off > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.log || { tail -20 $O/c2_${v}_$rep.log; exit 1; }
    python3 scripts/jline.py $O/c2_${v}_$rep.json c2_${v}_$rep
  done
done
