#!/bin/bash
# QG code-block-count prefetch: QG parity suites, then A/B against ngt_amd/libngt_amd_ab.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/qgpf
timeout -k 10 600 python -u -m pytest tests/test_gpu_qg.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/qgpf/pytest.log 2>&1 || { tail -30 gpurun_out/qgpf/pytest.log; exit 1; }
tail -2 gpurun_out/qgpf/pytest.log
B="python bench.py --mode qg --steps 10 --warmup 2 --no-cpu --eps 0.056640625"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/qgpf/cur$i.json 2> gpurun_out/qgpf/cur$i.log || exit 1
  NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_ab.so timeout -k 10 300 $B > gpurun_out/qgpf/old$i.json 2> gpurun_out/qgpf/old$i.log || exit 1
done
for f in cur1 old1 cur2 old2; do python3 -c "import json; d=json.load(open('gpurun_out/qgpf/$f.json')); print('$f', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), d['config']['recall_at_10'])"; done
