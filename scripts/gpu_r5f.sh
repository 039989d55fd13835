#!/bin/bash
# round 5: latency kernel hop prefetch -- latency/serve/build parity suites,
# then the 1M ANNG line (single-query latency + the C-API key) with the hop
# prefetch on and off (same saved index)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_lookahead.py \
  tests/test_gpu_serve.py tests/test_gpu_build.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
D=/tmp/anng_r5f
for hop in 1 0; do
  NGT_AMD_TEST_KNOBS=1 NGT_AMD_LAT_HOP=$hop timeout -k 10 500 python -u bench.py --graph anng --anng-dir $D \
    --steps 3 --warmup 1 --no-cpu --latency-queries 100 > $O/anng_hop$hop.json 2> $O/anng_hop$hop.log \
    || { tail -30 $O/anng_hop$hop.log; exit 1; }
  python3 - $O/anng_hop$hop.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
l = d["single_query_latency"]; c = d.get("capi") or {}
print(sys.argv[1], round(d["value"]), d["config"].get("graph_build_s"), "lat", round(l["mean_ms"], 2), round(l["p50_ms"], 2),
      "capi 1t", c.get("single_thread_latency_ms", {}).get("mean"), "best", c.get("qps_best"), c.get("reference_parity"))
PY
done
# QG kernel phase split (stamps build) on the 2M one-ANNG QG line
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --mode qg --graph anng --n 2000000 \
  --anng-batch 8000 --eps 0.10529 --steps 2 --warmup 1 --no-cpu --latency-queries 0 > $O/stamps_qg2m.json \
  2> $O/stamps_qg2m.log || { tail -20 $O/stamps_qg2m.log; exit 1; }
grep -E "phase|expansions" $O/stamps_qg2m.log
