#!/bin/bash
# round 5: C3's long rows -- (1) parity suites with the 16-lanes-per-row
# evaluator; (2) C3 at the line's epsilon with library variants: quad-per-row
# evaluator (v0, the round's start), 16 lanes per row in stages of 32 (the
# product build) or 64 loads per lane, and 2 or 4 filter rows per lane group;
# (3) the product build with an accepted-only visited set + LDS filter (which
# also turns the probe-and-resume schedule on)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5u}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_production.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  local name=$1; shift
  env NGT_AMD_TEST_KNOBS=1 "$@" timeout -k 10 300 python -u bench.py --config c3 --eps 0.056640625 --steps 3 \
    --warmup 1 --no-cpu --latency-queries 0 --anng-line off --c3-line off > $O/$name.json 2> $O/$name.log \
    || { tail -20 $O/$name.log; exit 1; }
  python3 scripts/jline.py $O/$name.json $name
}
L=$PWD/ngt_amd
run v0r2 NGT_AMD_LIB=$L/libngt_amd_v0r2.so
run v32r2 NGT_AMD_LIB=$L/libngt_amd.so
run v64r2 NGT_AMD_LIB=$L/libngt_amd_v64r2.so
run v32r4 NGT_AMD_LIB=$L/libngt_amd_v32r4.so
run v0r4 NGT_AMD_LIB=$L/libngt_amd_v0r4.so
run v32r2_acc15 NGT_AMD_ACCEPTED_ONLY=1 NGT_AMD_VFILTER=15
run v32r2_acc14c256 NGT_AMD_ACCEPTED_ONLY=1 NGT_AMD_VFILTER=14 NGT_AMD_CQ_CAP=256
