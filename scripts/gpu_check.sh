#!/bin/bash
# GPU parity suite + default bench line + stamps breakdown, each under its own limit.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log &&
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --eps 0.0703 > gpurun_out/stamps.json 2> gpurun_out/stamps.log
rc2=$?
grep -E "eps|phase" gpurun_out/bench_default.log gpurun_out/stamps.log
exit $(( rc | rc2 ))
