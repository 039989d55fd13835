#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE,
# L2 hit/miss) of the C2 bench workload at a fixed epsilon.
# usage: scripts/profile.sh <tag> [bench args...]; outputs under gpurun_out/prof_<tag>*
TAG=${1:-r1}; shift
ARGS=${@:-"--steps 3 --warmup 1 --no-cpu --eps 0.0703125"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d ${P} -o trace -- python3 bench.py $ARGS > ${P}_bench.json 2> ${P}_bench.log && \
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d ${P}_fetch -o pmc -- python3 bench.py $ARGS > /dev/null 2> ${P}_fetch.log && \
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d ${P}_write -o pmc -- python3 bench.py $ARGS > /dev/null 2> ${P}_write.log && \
timeout -k 10 500 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d ${P}_l2 -o pmc -- python3 bench.py $ARGS > /dev/null 2> ${P}_l2.log
rc=$?
echo PROFILE_EXIT=$rc
find gpurun_out/prof_${TAG}* -name "*.csv" | head -20
exit $rc
