#!/bin/bash
# lookahead kernel line accounting on the ANNG (diagnostic build), then the
# unchecked-set capacity knob on the product build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4r}; mkdir -p $O
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_lacount.so timeout -k 10 400 python -u bench.py --graph anng --anng-line off --steps 2 --warmup 1 \
  --no-cpu --latency-queries 0 --eps 0.128 > $O/lacount_anng.json 2> $O/lacount_anng.log || { tail -20 $O/lacount_anng.log; exit 1; }
grep -E "accounting|expansions|discarded|eps" $O/lacount_anng.log
for cq in 128 192; do
  NGT_AMD_CQ_CAP=$cq timeout -k 10 400 python -u bench.py --graph anng --anng-line off --steps 3 --warmup 1 \
    --no-cpu --latency-queries 0 --eps 0.128 > $O/cq$cq.json 2> $O/cq$cq.log || { tail -20 $O/cq$cq.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cq$cq.json')); print('cq $cq', round(d['value']), d['config']['recall_at_10'], round(d['roofline']['kernel_ms'],2))"
done
