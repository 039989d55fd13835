#!/bin/bash
# round 5: the shard key at full scale on one rank -- C4's 10M index as 8 shards
# of 1.25M on one GPU (what --gpus N spreads 8/N per rank), with the C2
# headline in the same run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5p}; mkdir -p $O
timeout -k 10 1000 python -u bench.py --shard-line on --anng-line off --c3-line off --steps 10 --warmup 3 \
  --latency-queries 0 --cpu-seconds 5 > $O/bench_shard10m.json 2> $O/bench_shard10m.log || { tail -30 $O/bench_shard10m.log; exit 1; }
python3 - $O/bench_shard10m.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); s = d["shard"]
print("c2", round(d["value"]), "shard", round(s["value"]), s["config"]["recall_at_10"], s["config"]["objects_total"],
      s["config"]["shards_per_gpu"], round(s["roofline"]["kernel_ms"], 2), round(s["roofline"]["frac"], 3),
      s["parity_sample"], round(s["wall_s"]), s["config"]["setup_s"])
PY
for f in 0.25 0.3 0.4; do
  NGT_AMD_TEST_KNOBS=1 NGT_AMD_SCHED_FRAC=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --anng-line off \
    --c3-line off --no-cpu --latency-queries 0 > $O/frac$f.json 2> $O/frac$f.log || { tail -20 $O/frac$f.log; exit 1; }
  python3 scripts/jline.py $O/frac$f.json frac$f
done
