#!/bin/bash
# round 5: the C2 surrogate graph's edge mix (kNN k, out-edges, in-edges, cap)
# against the headline QPS at recall 0.95 -- same kernel, same data
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5e}; mkdir -p $O
for cfg in "128 48 96 160" "128 32 96 128" "128 24 96 120" "128 16 112 128" "128 10 120 130" "128 64 96 160" "160 48 128 176"; do
  set -- $cfg
  n=k$1_o$2_i$3_m$4
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --anng-line off --c3-line off --no-cpu \
    --latency-queries 0 --knn $1 --out-deg $2 --in-deg $3 --max-deg $4 > $O/$n.json 2> $O/$n.log \
    || { tail -20 $O/$n.log; exit 1; }
  python3 scripts/jline.py $O/$n.json $n
done
for s in 4 5; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --anng-line off --c3-line off --no-cpu \
    --latency-queries 0 --streams $s > $O/streams$s.json 2> $O/streams$s.log || { tail -20 $O/streams$s.log; exit 1; }
  python3 scripts/jline.py $O/streams$s.json streams$s
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --anng-line off --c3-line off --no-cpu \
  --latency-queries 0 --streams 3 > $O/streams3.json 2> $O/streams3.log || { tail -20 $O/streams3.log; exit 1; }
python3 scripts/jline.py $O/streams3.json streams3
