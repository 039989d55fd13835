#!/bin/bash
cd "$GRAFT_REPO_ROOT"
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --eps 0.0703 > gpurun_out/stamps.json 2> gpurun_out/stamps.log
grep -E "phase|eps|graph" gpurun_out/stamps.log
