#!/bin/bash
# (1) per-query kernel cost vs batch size (tail effect of the persistent kernel)
# (2) QG phase stamps (diagnostic build)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for nq in 4096 8192 10000 20000 40000; do
  timeout -k 10 300 python -u bench.py --nq $nq --steps 3 --warmup 1 --no-cpu --eps 0.0703125 > gpurun_out/tail_$nq.json 2> gpurun_out/tail_$nq.log || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/tail_$nq.json'))
print($nq, round(d['value']), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],3), d['config']['recall_at_10'])"
done
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python -u bench.py --mode qg --steps 2 --warmup 1 --no-cpu --eps 0.05625 > gpurun_out/qg_stamps.json 2> gpurun_out/qg_stamps.log || exit 1
grep -E "phase|eps" gpurun_out/qg_stamps.log
python3 -c "
import json; d=json.load(open('gpurun_out/qg_stamps.json')); print(d['config'])"
