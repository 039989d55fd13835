#!/bin/bash
# Per-phase cycle split of the construction searches (stamps build, diagnostic only).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
N=${1:-300000}
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so NGT_AMD_BUILD_PROFILE=1 timeout -k 10 600 python -u scripts/build_bench.py \
  --n $N --check 100 > gpurun_out/build_stamps.json 2> gpurun_out/build_stamps.log
rc=$?; grep -E "build_insert" gpurun_out/build_stamps.log; cat gpurun_out/build_stamps.json; exit $rc
