#!/bin/bash
# round 5: the latency kernel's hop cache -- the suites that run the latency
# kernel (lookahead/latency parity incl. the hop forms, serving grid, ANNG
# construction byte-identical to the reference, C API), then the 1M ANNG
# single query (launch + served) with the hop evaluated ahead (1), L2 prefetch
# only (2, round 5 before this) and off (0), interleaved twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5y}; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lookahead.py \
  tests/test_gpu_serve.py tests/test_gpu_build.py tests/test_gpu_api.py -m gpu > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
D=/tmp/anng_r5y
for rep in a b; do
for h in 1 2 0; do
  NGT_AMD_TEST_KNOBS=1 NGT_AMD_LAT_HOP=$h timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D --steps 1 \
    --warmup 1 --no-cpu --latency-queries 80 --capi-line off > $O/hop${h}_$rep.json 2> $O/hop${h}_$rep.log \
    || { tail -30 $O/hop${h}_$rep.log; exit 1; }
  python3 - $O/hop${h}_$rep.json hop${h}_$rep <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
l = d["single_query_latency"]
print(sys.argv[2], "lat", round(l["mean_ms"], 2), round(l["p50_ms"], 2), "served", round(l.get("served_mean_ms", 0), 2),
      round(l.get("served_p50_ms", 0), 2), "stalled", l.get("stalled_pops_mean"))
PY
done
done
