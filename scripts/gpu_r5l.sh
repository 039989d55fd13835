#!/bin/bash
# round 5: the densest C2 surrogate graphs the padded adjacency allows (<= 256
# edges per node), and the QG filter/tail setting on the C2-graph QG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5l}; mkdir -p $O
for cfg in "256 64 224 256" "256 96 224 256" "256 128 192 256" "224 96 192 256" "224 64 192 256"; do
  set -- $cfg
  n=k$1_o$2_i$3_m$4
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --anng-line off --c3-line off --no-cpu \
    --latency-queries 0 --knn $1 --out-deg $2 --in-deg $3 --max-deg $4 > $O/$n.json 2> $O/$n.log \
    || { tail -20 $O/$n.log; exit 1; }
  python3 scripts/jline.py $O/$n.json $n
done
export NGT_AMD_TEST_KNOBS=1
for cfg in "14 512" "15 256"; do
  set -- $cfg
  NGT_AMD_VFILTER=$1 NGT_AMD_CQ_CAP=$2 timeout -k 10 400 python -u bench.py --mode qg --eps 0.05625 --steps 10 \
    --warmup 2 --no-cpu --latency-queries 0 > $O/qgc2_vf$1_cq$2.json 2> $O/qgc2_vf$1_cq$2.log \
    || { tail -20 $O/qgc2_vf$1_cq$2.log; exit 1; }
  python3 scripts/jline.py $O/qgc2_vf$1_cq$2.json qgc2_vf$1_cq$2
done
