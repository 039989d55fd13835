#!/bin/bash
# Per-phase cycle split of the QG search kernel (stamps build, diagnostic only).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python bench.py --mode qg --steps 2 --warmup 1 --no-cpu \
  --eps 0.056640625 > gpurun_out/stamps_qg.json 2> gpurun_out/stamps_qg.log
rc=$?; grep -E "phase|eps" gpurun_out/stamps_qg.log; exit $rc
