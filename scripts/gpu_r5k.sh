#!/bin/bash
# round 5: (1) the QG kernel's LDS visited filter size / tail capacity on the
# 2M one-ANNG line (visited probes are its excess traffic); (2) C2 surrogate
# graphs with more in-edges
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5k}; mkdir -p $O
export NGT_AMD_TEST_KNOBS=1
for cfg in "14 512" "15 256" "16 256" "17 256"; do
  set -- $cfg
  NGT_AMD_VFILTER=$1 NGT_AMD_CQ_CAP=$2 timeout -k 10 500 python -u bench.py --mode qg --graph anng --n 2000000 \
    --anng-batch 8000 --eps 0.10529 --steps 5 --warmup 1 --no-cpu --latency-queries 0 > $O/qg2m_vf$1_cq$2.json \
    2> $O/qg2m_vf$1_cq$2.log || { tail -20 $O/qg2m_vf$1_cq$2.log; exit 1; }
  python3 scripts/jline.py $O/qg2m_vf$1_cq$2.json qg2m_vf$1_cq$2
done
unset NGT_AMD_TEST_KNOBS
for cfg in "160 64 128 192" "192 48 160 208" "192 64 160 224" "224 64 192 256" "256 32 224 256"; do
  set -- $cfg
  n=k$1_o$2_i$3_m$4
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --anng-line off --c3-line off --no-cpu \
    --latency-queries 0 --knn $1 --out-deg $2 --in-deg $3 --max-deg $4 > $O/$n.json 2> $O/$n.log \
    || { tail -20 $O/$n.log; exit 1; }
  python3 scripts/jline.py $O/$n.json $n
done
