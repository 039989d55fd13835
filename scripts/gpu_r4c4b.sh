#!/bin/bash
# C4 counter passes (FETCH_SIZE, WRITE_SIZE) at the line's epsilon: after the
# epsilon check, exactly 3 more steps of the timed configuration
# (--pmc-launches 3 = 24 shard searches = 48 dispatches, probe + resume)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4c4b}; mkdir -p $O
EPS=${2:-0.068359375}
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for pass in fetch write; do
  C=FETCH_SIZE; [ $pass = write ] && C=WRITE_SIZE
  timeout -k 10 420 rocprofv3 --pmc $C -d "$R/$O/c4_$pass" -o $pass --output-format csv -- \
    python3 "$R/bench.py" --mode shard --shards-per-gpu 8 --eps $EPS --pmc-launches 3 --no-cpu \
    --latency-queries 0 > "$R/$O/c4_$pass.json" 2> "$R/$O/c4_$pass.log" || exit 1
  python3 "$R/scripts/pmc_summary.py" "$R/$O" "c4_$pass" --last 48 > /dev/null || exit 1
done
echo "c4 pmc done"
