#!/bin/bash
# Round-2 bench lines: C2 (graph search + exact scan), NGTQG on C2, C3.
TAG=${1:-r2c}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
for m in "c2:" "qg:--mode qg" "c3:--config c3"; do
  name=${m%%:*}; args=${m#*:}
  timeout -k 10 700 python bench.py $args > gpurun_out/$TAG/bench_$name.json 2> gpurun_out/$TAG/bench_$name.log || exit $?
  tail -2 gpurun_out/$TAG/bench_$name.log
done
