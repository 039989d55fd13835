#!/bin/bash
# FETCH_SIZE of the ANNG line's kernel with the deferred visited test
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4j}; mkdir -p $O
R="$GRAFT_REPO_ROOT"; D=/tmp/anng_r4j
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 1 --warmup 1 \
  --no-cpu --latency-queries 0 --anng-line off > $O/anng_build.json 2> $O/anng_build.log || { tail -5 $O/anng_build.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/anng_fetch" -o fetch --output-format csv -- \
  python3 "$R/bench.py" --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --pmc-launches 6 --no-cpu --anng-line off \
  > "$R/$O/anng_fetch.json" 2> "$R/$O/anng_fetch.log" || exit 1
python3 "$R/scripts/pmc_summary.py" "$R/$O" anng_fetch --last 6
