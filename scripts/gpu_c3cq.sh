#!/bin/bash
# C3 filtered search with smaller LDS unchecked arrays (more resident waves per CU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c3cq
for CQ in 1024 512 384; do
  NGT_AMD_CQ_CAP=$CQ timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu --eps 0.06523437500000001 \
    > gpurun_out/c3cq/cq$CQ.json 2> gpurun_out/c3cq/cq$CQ.log || { tail -5 gpurun_out/c3cq/cq$CQ.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c3cq/cq$CQ.json')); r=d['roofline']; print($CQ, round(d['value']), d['config']['recall_at_10'], r['kernel_ms'], d['ms_per_step'])"
done
