#!/bin/bash
# C2 overlapped steps against the number of HIP streams consecutive steps alternate over
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4o}; mkdir -p $O
for st in 3 4 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 20 --streams $st \
    > $O/c2_st$st.json 2> $O/c2_st$st.log || { tail -5 $O/c2_st$st.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2_st$st.json')); print('streams $st', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2))"
done
