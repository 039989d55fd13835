#!/bin/bash
# round 5: NGTQG packed search layout -- the QG suite, then the C2-graph QG
# line and a 2M one-ANNG QG line with the packed layout and (A/B) the fixed slabs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_qg.py -m gpu \
  > $O/pytest_qg.log 2>&1 || { tail -40 $O/pytest_qg.log; exit 1; }
tail -3 $O/pytest_qg.log
timeout -k 10 400 python -u bench.py --mode qg --steps 10 --warmup 2 --cpu-seconds 5 > $O/qg.json 2> $O/qg.log \
  || { tail -30 $O/qg.log; exit 1; }
python3 scripts/jline.py $O/qg.json qg_packed
export NGT_AMD_TEST_KNOBS=1
NGT_AMD_QG_PACKED=0 timeout -k 10 400 python -u bench.py --mode qg --steps 10 --warmup 2 --no-cpu > $O/qg_fixed.json \
  2> $O/qg_fixed.log || { tail -30 $O/qg_fixed.log; exit 1; }
python3 scripts/jline.py $O/qg_fixed.json qg_fixed
timeout -k 10 500 python -u bench.py --mode qg --graph anng --n 2000000 --anng-batch 8000 --steps 5 --warmup 1 \
  --cpu-seconds 5 > $O/qg_anng2m.json 2> $O/qg_anng2m.log || { tail -30 $O/qg_anng2m.log; exit 1; }
python3 scripts/jline.py $O/qg_anng2m.json qg_anng2m_packed
NGT_AMD_QG_PACKED=0 timeout -k 10 500 python -u bench.py --mode qg --graph anng --n 2000000 --anng-batch 8000 \
  --steps 5 --warmup 1 --no-cpu > $O/qg_anng2m_fixed.json 2> $O/qg_anng2m_fixed.log || { tail -30 $O/qg_anng2m_fixed.log; exit 1; }
python3 scripts/jline.py $O/qg_anng2m_fixed.json qg_anng2m_fixed
