#!/bin/bash
# round 5: NGTQG next-record prefetch (NGT_AMD_QG_PF=1: the head's next key's
# packed record read towards L2 by LDS-DMA under each expansion) -- the QG
# suite with it on, then A/B on the C2-graph QG line and the 2M one-ANNG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5zi}; mkdir -p $O
NGT_AMD_QG_PF=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_qg.py \
  -m gpu > $O/pytest_qg_pf.log 2>&1 || { tail -30 $O/pytest_qg_pf.log; exit 1; }
tail -1 $O/pytest_qg_pf.log
for rep in a b; do
  for pf in 0 1; do
    NGT_AMD_TEST_KNOBS=1 NGT_AMD_QG_PF=$pf timeout -k 10 300 python -u bench.py --mode qg --eps 0.05548 --steps 10 \
      --warmup 2 --no-cpu --latency-queries 0 --anng-line off --c3-line off > $O/qgc2_pf${pf}_$rep.json \
      2> $O/qgc2_pf${pf}_$rep.log || { tail -20 $O/qgc2_pf${pf}_$rep.log; exit 1; }
    python3 scripts/jline.py $O/qgc2_pf${pf}_$rep.json qgc2_pf${pf}_$rep
  done
done
for pf in 0 1; do
  NGT_AMD_TEST_KNOBS=1 NGT_AMD_QG_PF=$pf timeout -k 10 400 python -u bench.py --mode qg --graph anng --n 2000000 \
    --anng-batch 8000 --eps 0.10529 --steps 5 --warmup 1 --no-cpu --latency-queries 0 > $O/qg2m_pf$pf.json \
    2> $O/qg2m_pf$pf.log || { tail -20 $O/qg2m_pf$pf.log; exit 1; }
  python3 scripts/jline.py $O/qg2m_pf$pf.json qg2m_pf$pf
done
