#!/bin/bash
# round 5: where a lone query's time goes on the 1M ANNG -- the product line
# (launch latency, the serving grid's per-call latency, the C-API key), then
# the stamps build's commit-wave phase split on the same saved index
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5q}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_schedule.py -m gpu > $O/pytest_sched.log 2>&1 || { tail -30 $O/pytest_sched.log; exit 1; }
tail -1 $O/pytest_sched.log
D=/tmp/anng_r5q
timeout -k 10 500 python -u bench.py --graph anng --anng-dir $D --steps 3 --warmup 1 --no-cpu \
  --latency-queries 60 > $O/anng.json 2> $O/anng.log || { tail -30 $O/anng.log; exit 1; }
grep -E "single|served" $O/anng.log
python3 - $O/anng.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
l = d["single_query_latency"]; c = d.get("capi") or {}
print(round(d["value"]), "lat", round(l["mean_ms"], 2), "served", l.get("served_mean_ms"), l.get("served_p50_ms"),
      "capi 1t", c.get("single_thread_latency_ms", {}).get("mean"), "best", c.get("qps_best"))
PY
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D \
  --steps 2 --warmup 1 --no-cpu --latency-queries 30 --capi-line off > $O/stamps.json 2> $O/stamps.log \
  || { tail -20 $O/stamps.log; exit 1; }
grep -E "phase|single" $O/stamps.log
