#!/bin/bash
# ANNG lookahead form: 2 vs 3 targets per step, and trace + PMC passes of the
# current (4-wave) kernel at the line's epsilon
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3j
D=/tmp/anng1m
A="--graph anng --anng-dir $D --steps 3 --warmup 1 --no-cpu --eps 0.1279296875 --latency-queries 0"
timeout -k 10 400 python -u bench.py $A > gpurun_out/r3j/anng_p3.json 2> gpurun_out/r3j/anng_p3.log || { tail -5 gpurun_out/r3j/anng_p3.log; exit 1; }
NGT_AMD_LA_P=2 timeout -k 10 300 python -u bench.py $A > gpurun_out/r3j/anng_p2.json 2> gpurun_out/r3j/anng_p2.log || { tail -5 gpurun_out/r3j/anng_p2.log; exit 1; }
for f in anng_p3 anng_p2; do python3 -c "import json; d=json.load(open('gpurun_out/r3j/$f.json')); print('$f', round(d['value']), d['roofline']['kernel_ms'])"; done
bash scripts/pmc_r3.sh gpurun_out/r3j anng --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 \
  --pmc-launches 6 --no-cpu || exit 1
# the lookahead form on the C2 kNN graph (long lists), forced
NGT_AMD_LA=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --eps 0.0703125 --latency-queries 0 \
  > gpurun_out/r3j/c2_la.json 2> gpurun_out/r3j/c2_la.log || { tail -5 gpurun_out/r3j/c2_la.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3j/c2_la.json')); print('c2_la', round(d['value']), d['roofline']['kernel_ms'])"
