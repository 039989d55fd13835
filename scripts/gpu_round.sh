#!/bin/bash
# GPU parity suite, default bench line, then the rocprofv3 passes (profile.sh <tag>).
# usage: scripts/gpu_round.sh <tag>
TAG=${1:-r1f}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.log || exit $?
grep -E "accepted|eps" gpurun_out/bench_${TAG}.log | tail -3
scripts/profile.sh $TAG
