#!/bin/bash
# round 6: 16-byte filter-code loads in the C2 filter -- GPU parity of
# the C2 paths, then an interleaved A/B of the C2 line against the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6r}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_production.py tests/test_gpu_schedule.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do for v in A B; do
  L=ngt_amd/libngt_amd_base.so; [ $v = B ] && L=ngt_amd/libngt_amd.so
  NGT_AMD_LIB=$PWD/$L timeout -k 10 300 python3 -u bench.py --eps 0.058203125 --steps 20 --warmup 5 --no-cpu \
    --latency-queries 0 --anng-line off --qg-line off --c3-line off > $O/$v$r.json 2> $O/$v$r.log || { tail -5 $O/$v$r.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$v$r.json')); c=d['config']
print('$v$r', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), c['recall_at_10'], c['exact_neighbour_distances_per_query'], c['evaluations_per_query'])"
done; done
