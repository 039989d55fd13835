#!/bin/bash
# round 5: C3's long rows -- library variants at the line's epsilon:
#   v0r2      the round's start (quad-per-row evaluator, 8 filter rows per step, chunk by chunk)
#   v32r2np   16 lanes per row (32 loads per lane per stage), chunk by chunk
#   p32r2w4   + the pipelined expansion (one adjacency read, all probes together, survivors batched) [product]
#   p32r2w3   the same at 3 waves per SIMD (168 VGPRs)
#   p32r4w4   16 filter rows per step
#   p0r2w4    pipelined with the quad evaluator
# then the product build with an accepted-only visited set + LDS filter
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5v}; mkdir -p $O
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
run p32r2w4 NGT_AMD_LIB=$L/libngt_amd.so
run v0r2 NGT_AMD_LIB=$L/libngt_amd_v0r2.so
run v32r2np NGT_AMD_LIB=$L/libngt_amd_v32r2np.so
run p32r2w3 NGT_AMD_LIB=$L/libngt_amd_p32r2w3.so
run p32r4w4 NGT_AMD_LIB=$L/libngt_amd_p32r4w4.so
run p0r2w4 NGT_AMD_LIB=$L/libngt_amd_p0r2w4.so
run p32r2w4_acc15 NGT_AMD_ACCEPTED_ONLY=1 NGT_AMD_VFILTER=15
