#!/bin/bash
# serving grid diagnostics: why grids leave under load (C client + python)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3p
NGT_AMD_SERVE_LOG=1 timeout -k 10 400 python -u bench.py --mode capi --no-cpu --eps 0.0703125 \
  > gpurun_out/r3p/capi.json 2> gpurun_out/r3p/capi.log || { tail -5 gpurun_out/r3p/capi.log; exit 1; }
grep -h "C client\|single\|serve" gpurun_out/r3p/capi.log | head -80
