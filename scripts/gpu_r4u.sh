#!/bin/bash
# counter passes of the ANNG line (lookahead kernel)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4u}; mkdir -p $O
D=/tmp/anng_r4u
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 3 --warmup 1 \
  --no-cpu --latency-queries 0 --anng-line off > $O/anng_build.json 2> $O/anng_build.log || { tail -5 $O/anng_build.log; exit 1; }
python3 scripts/jline.py $O/anng_build.json anng
PMC_LAST=6 bash scripts/pmc_r4.sh $O anng --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --pmc-launches 6 --no-cpu --anng-line off || exit 1
python3 - <<PY
import json
f=json.load(open("$O/anng_fetch_pmc.json")); t=json.load(open("$O/anng_tcc_pmc.json"))
k=[x for x in f if "la_kernel" in x][0]; e=f[k]; tt=t[k]
print("fetch GB/launch", e["FETCH_SIZE"]/e["dispatches"]*2048/1e9, "rdreq/launch", tt["TCC_EA0_RDREQ_sum"]/tt["dispatches"])
PY
