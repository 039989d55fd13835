#!/bin/bash
# round 5: commit-wave tweaks in the latency kernel (slot generations in a
# register, list entries read with their count) -- the latency-kernel suites,
# then the 1M ANNG single query against the committed library, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5za}; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lookahead.py \
  tests/test_gpu_serve.py tests/test_gpu_build.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
D=/tmp/anng_r5za
for rep in a b c; do
for lib in new base; do
  L=$PWD/ngt_amd/libngt_amd.so; [ $lib = base ] && L=$PWD/ngt_amd/libngt_amd_base.so
  NGT_AMD_LIB=$L timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D --steps 1 --warmup 1 --no-cpu \
    --latency-queries 80 --capi-line off > $O/${lib}_$rep.json 2> $O/${lib}_$rep.log || { tail -30 $O/${lib}_$rep.log; exit 1; }
  python3 - $O/${lib}_$rep.json ${lib}_$rep <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
l = d["single_query_latency"]
print(sys.argv[2], "lat", round(l["mean_ms"], 2), round(l["p50_ms"], 2), "served", round(l.get("served_mean_ms", 0), 2),
      round(l.get("served_p50_ms", 0), 2))
PY
done
done
