#!/bin/bash
# C5-form NGTQG shard line (1 GPU, 1.25M rows) and the C-API line on the final tree.
set -o pipefail
TAG=${1:-r2fin}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 \
  bench.py --mode shard --qg --steps 5 --warmup 1 > gpurun_out/$TAG/bench_shard_qg.json 2> gpurun_out/$TAG/bench_shard_qg.log || { tail -5 gpurun_out/$TAG/bench_shard_qg.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_shard_qg.json')); print('shard_qg', round(d['value']), d['config']['recall_at_10'], d['roofline']['frac'])"
timeout -k 10 600 python bench.py --mode capi > gpurun_out/$TAG/bench_capi.json 2> gpurun_out/$TAG/bench_capi.log || { tail -5 gpurun_out/$TAG/bench_capi.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_capi.json')); print('capi', round(d['value']), d['single_query_latency_ms'], d.get('batched_capi_qps'))"
