#!/bin/bash
# C4 on one GPU (10M x 128 as 8 shards of 1.25M): the line, then FETCH_SIZE and
# WRITE_SIZE passes of the same workload (3 steps: the last 48 dispatches =
# 24 shard searches of 2 dispatches each, probe and resume)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4c4}; mkdir -p $O
timeout -k 10 600 python3 -u bench.py --mode shard --shards-per-gpu 8 --steps 10 --warmup 2 --cpu-seconds 10 \
  --latency-queries 0 > $O/bench_c4_1gpu.json 2> $O/bench_c4_1gpu.log || { tail -20 $O/bench_c4_1gpu.log; exit 1; }
python3 scripts/jline.py $O/bench_c4_1gpu.json c4
EPS=$(python3 -c "import json; print(repr(json.load(open('$O/bench_c4_1gpu.json'))['config']['epsilon']))")
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for pass in fetch write; do
  C=FETCH_SIZE; [ $pass = write ] && C=WRITE_SIZE
  timeout -k 10 420 rocprofv3 --pmc $C -d "$R/$O/c4_$pass" -o $pass --output-format csv -- \
    python3 "$R/bench.py" --mode shard --shards-per-gpu 8 --eps $EPS --steps 3 --warmup 1 --no-cpu --shard-sample 16 \
    --latency-queries 0 > "$R/$O/c4_$pass.json" 2> "$R/$O/c4_$pass.log" || exit 1
  python3 "$R/scripts/pmc_summary.py" "$R/$O" "c4_$pass" --last 48 > /dev/null || exit 1
done
echo "c4 pmc done"
