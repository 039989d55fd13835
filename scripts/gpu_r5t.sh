#!/bin/bash
# round 5: latency kernel test bits on the 1M ANNG single query (launch and
# served): 1 hop prefetch (default), 3 the two nearest, 5 commit wave at raised
# issue priority, 7 both; interleaved twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5t}; mkdir -p $O
D=/tmp/anng_r5t
for rep in a b; do
for h in 1 3 5 7; do
  NGT_AMD_TEST_KNOBS=1 NGT_AMD_LAT_HOP=$h timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D --steps 1 \
    --warmup 1 --no-cpu --latency-queries 80 --capi-line off > $O/hop${h}_$rep.json 2> $O/hop${h}_$rep.log \
    || { tail -30 $O/hop${h}_$rep.log; exit 1; }
  python3 - $O/hop${h}_$rep.json hop${h}_$rep <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
l = d["single_query_latency"]
print(sys.argv[2], "lat", round(l["mean_ms"], 2), round(l["p50_ms"], 2), "served", round(l.get("served_mean_ms", 0), 2),
      round(l.get("served_p50_ms", 0), 2))
PY
done
done
