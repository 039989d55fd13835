#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE)
# of the default C2 bench workload.  Outputs under gpurun_out/prof_r1*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--steps 3 --warmup 1 --no-cpu --eps 0.096"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1 -o trace -- python3 bench.py $ARGS > gpurun_out/prof_r1_bench.json 2> gpurun_out/prof_r1_bench.log && \
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_r1_fetch -o pmc -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/prof_r1_fetch.log && \
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_r1_write -o pmc -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/prof_r1_write.log
echo PROFILE_EXIT=$?
find gpurun_out/prof_r1* -name "*.csv" | head -20
