#!/bin/bash
# round 5: the NGTQG search kernel at 4 (product, 128 VGPRs, 112 B of spills
# per lane) and 3 waves per SIMD (152 VGPRs, none): the 2M one-ANNG QG line
# and the C2-graph QG line, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5zg}; mkdir -p $O
L=$PWD/ngt_amd
for rep in a b; do
  for v in w4 w3; do
    lib=$L/libngt_amd.so; [ $v = w3 ] && lib=$L/libngt_amd_qgw3.so
    NGT_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --mode qg --eps 0.05548 --steps 10 --warmup 2 --no-cpu \
      --latency-queries 0 --anng-line off --c3-line off > $O/qgc2_${v}_$rep.json 2> $O/qgc2_${v}_$rep.log \
      || { tail -20 $O/qgc2_${v}_$rep.log; exit 1; }
    python3 scripts/jline.py $O/qgc2_${v}_$rep.json qgc2_${v}_$rep
  done
done
for v in w4 w3; do
  lib=$L/libngt_amd.so; [ $v = w3 ] && lib=$L/libngt_amd_qgw3.so
  NGT_AMD_LIB=$lib timeout -k 10 400 python -u bench.py --mode qg --graph anng --n 2000000 --anng-batch 8000 \
    --eps 0.10529 --steps 5 --warmup 1 --no-cpu --latency-queries 0 > $O/qg2m_$v.json 2> $O/qg2m_$v.log \
    || { tail -20 $O/qg2m_$v.log; exit 1; }
  python3 scripts/jline.py $O/qg2m_$v.json qg2m_$v
done
