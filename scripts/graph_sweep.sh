#!/bin/bash
# graph-construction parameter sweep for the C2 bench (kNN K, out, in, max degree)
cd "$GRAFT_REPO_ROOT"
for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --knn $1 --out-deg $2 --in-deg $3 --max-deg $4 \
     > gpurun_out/sweep_$1_$2_$3_$4.json 2> gpurun_out/sweep_$1_$2_$3_$4.log || break
  python3 -c "
import json; d=json.load(open('gpurun_out/sweep_$1_$2_$3_$4.json'))
print('$cfg', round(d['value']), d['config']['recall_at_10'], round(d['config']['epsilon'],4), round(d['config']['distance_computations_per_query']), round(d['roofline']['achieved']))"
done
