#!/bin/bash
# round 5: NGTQG kernel with the register-head unchecked set -- the QG suite,
# then A/B against the library before the change (libngt_amd_r5base.so) on the
# C2-graph QG line and the 2M one-ANNG QG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_qg.py tests/test_gpu_shard.py -m gpu \
  > $O/pytest_qg.log 2>&1 || { tail -40 $O/pytest_qg.log; exit 1; }
tail -2 $O/pytest_qg.log
for lib in new base; do
  L=$PWD/ngt_amd/libngt_amd.so; [ $lib = base ] && L=$PWD/ngt_amd/libngt_amd_r5base.so
  NGT_AMD_LIB=$L timeout -k 10 400 python -u bench.py --mode qg --eps 0.05625 --steps 10 --warmup 2 --no-cpu \
    --latency-queries 0 > $O/qg_c2_$lib.json 2> $O/qg_c2_$lib.log || { tail -20 $O/qg_c2_$lib.log; exit 1; }
  python3 scripts/jline.py $O/qg_c2_$lib.json qg_c2_$lib
  NGT_AMD_LIB=$L timeout -k 10 500 python -u bench.py --mode qg --graph anng --n 2000000 --anng-batch 8000 \
    --eps 0.10529 --steps 5 --warmup 1 --no-cpu --latency-queries 0 > $O/qg_2m_$lib.json 2> $O/qg_2m_$lib.log \
    || { tail -20 $O/qg_2m_$lib.log; exit 1; }
  python3 scripts/jline.py $O/qg_2m_$lib.json qg_2m_$lib
done
