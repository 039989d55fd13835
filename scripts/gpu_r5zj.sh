#!/bin/bash
# round 5: lookahead kernel next-step adjacency prefetch (NGT_AMD_LA_PF=1) --
# the lookahead suite with it on, then the 1M ANNG line: the committed
# library (base), this one with the prefetch off and on, interleaved twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5zj}; mkdir -p $O
NGT_AMD_LA_PF=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_gpu_lookahead.py -m gpu > $O/pytest_la_pf.log 2>&1 || { tail -30 $O/pytest_la_pf.log; exit 1; }
tail -1 $O/pytest_la_pf.log
D=/tmp/anng_r5zj
L=$PWD/ngt_amd
for rep in a b; do
  for v in base pf0 pf1; do
    lib=$L/libngt_amd.so; [ $v = base ] && lib=$L/libngt_amd_base.so
    pf=0; [ $v = pf1 ] && pf=1
    NGT_AMD_TEST_KNOBS=1 NGT_AMD_LA_PF=$pf NGT_AMD_LIB=$lib timeout -k 10 400 python -u bench.py --graph anng \
      --anng-dir $D --steps 5 --warmup 1 --no-cpu --latency-queries 0 --capi-line off > $O/anng_${v}_$rep.json \
      2> $O/anng_${v}_$rep.log || { tail -30 $O/anng_${v}_$rep.log; exit 1; }
    python3 scripts/jline.py $O/anng_${v}_$rep.json anng_${v}_$rep
  done
done
