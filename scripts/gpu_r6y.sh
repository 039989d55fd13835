#!/bin/bash
# round 6 y: NGTQG record read-ahead (NGT_AMD_QG_PF) -- the QG GPU tests, then
# an interleaved A/B of the qg line (one saved 1M ANNG) against the build without it
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6y}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_qg.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
D=/tmp/ngt_y_anng_$$
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 1 \
  --warmup 1 --no-cpu --latency-queries 0 --capi-line off --anng-line off > $O/build.json 2> $O/build.log \
  || { tail -5 $O/build.log; exit 1; }
for r in 1 2 3; do for v in A B; do
  L=ngt_amd/libngt_amd_base.so; [ $v = B ] && L=ngt_amd/libngt_amd.so
  NGT_AMD_LIB=$PWD/$L timeout -k 10 300 python3 -u bench.py --mode qg --graph anng --anng-dir $D --eps 0.09772 \
    --expansion 3 --sweep-nq 10000 --steps 5 --warmup 1 --no-cpu --latency-queries 0 --anng-line off --c3-line off \
    --qg-line off > $O/$v$r.json 2> $O/$v$r.log || { tail -5 $O/$v$r.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$v$r.json')); c=d['config']
print('$v$r', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), c['recall_at_10'], c.get('expansions_per_query'))"
done; done
rm -rf $D
