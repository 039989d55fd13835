#!/bin/bash
# Bench lines on the current tree: C2 (default), NGTQG, and the one-rank
# torch.distributed.run launch of the default bench.
set -o pipefail
TAG=${1:-r2final}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 700 python bench.py > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.log || { tail -5 gpurun_out/$TAG/bench_c2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c2.json')); r=d['roofline']; print('c2', round(d['value']), d['ms_per_step'], r['kernel_ms'], r['frac'], d['parity_sample']['identical'])"
timeout -k 10 700 python bench.py --mode qg > gpurun_out/$TAG/bench_qg.json 2> gpurun_out/$TAG/bench_qg.log || { tail -5 gpurun_out/$TAG/bench_qg.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_qg.json')); r=d['roofline']; print('qg', round(d['value']), d['ms_per_step'], r['kernel_ms'], r['frac'], d['parity_sample']['identical'])"
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu > gpurun_out/$TAG/bench_dist1.json 2> gpurun_out/$TAG/bench_dist1.log || { tail -5 gpurun_out/$TAG/bench_dist1.log; exit 1; }
cut -c1-300 gpurun_out/$TAG/bench_dist1.json
