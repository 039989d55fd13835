#!/bin/bash
# round 5: NGTQG kernel with the epoch probe after the ADC, only for entries within the radius -- the QG suite,
# then A/B against the library before the change (libngt_amd_base.so) on the
# C2-graph QG line and the 2M one-ANNG QG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5r}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_qg.py tests/test_gpu_shard.py tests/test_gpu_serve.py tests/test_gpu_api.py -m gpu \
  > $O/pytest_qg.log 2>&1 || { tail -40 $O/pytest_qg.log; exit 1; }
tail -2 $O/pytest_qg.log
for lib in new base; do
  L=$PWD/ngt_amd/libngt_amd.so; [ $lib = base ] && L=$PWD/ngt_amd/libngt_amd_base.so
  NGT_AMD_LIB=$L timeout -k 10 400 python -u bench.py --mode qg --eps 0.05548 --steps 10 --warmup 2 --no-cpu \
    --latency-queries 0 > $O/qg_c2_$lib.json 2> $O/qg_c2_$lib.log || { tail -20 $O/qg_c2_$lib.log; exit 1; }
  python3 scripts/jline.py $O/qg_c2_$lib.json qg_c2_$lib
  NGT_AMD_LIB=$L timeout -k 10 500 python -u bench.py --mode qg --graph anng --n 2000000 --anng-batch 8000 \
    --eps 0.10529 --steps 5 --warmup 1 --no-cpu --latency-queries 0 > $O/qg_2m_$lib.json 2> $O/qg_2m_$lib.log \
    || { tail -20 $O/qg_2m_$lib.log; exit 1; }
  python3 scripts/jline.py $O/qg_2m_$lib.json qg_2m_$lib
done
# the serving grid with relaxed polls (no cache invalidation per poll) against
# the base library: single-query launch and served latency on the 1M ANNG
D=/tmp/anng_r5r
for lib in new base; do
  L=$PWD/ngt_amd/libngt_amd.so; [ $lib = base ] && L=$PWD/ngt_amd/libngt_amd_base.so
  C=on; [ $lib = base ] && C=off
  NGT_AMD_LIB=$L timeout -k 10 500 python -u bench.py --graph anng --anng-dir $D --steps 3 --warmup 1 --no-cpu \
    --latency-queries 60 --capi-line $C > $O/anng_$lib.json 2> $O/anng_$lib.log || { tail -30 $O/anng_$lib.log; exit 1; }
  python3 - $O/anng_$lib.json $lib <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
l = d["single_query_latency"]; c = d.get("capi") or {}
print(sys.argv[2], round(d["value"]), "lat", round(l["mean_ms"], 2), "served", round(l.get("served_mean_ms", 0), 2),
      round(l.get("served_p50_ms", 0), 2), "capi 1t", c.get("single_thread_latency_ms", {}).get("mean"), "best", c.get("qps_best"))
PY
done
