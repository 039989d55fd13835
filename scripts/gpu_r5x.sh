#!/bin/bash
# round 5: C5's per-GPU share (12.5M x 128 NGTQG over one device ANNG, -b 8000,
# tree seeds) with the epoch probe after the ADC (product) against the library
# before it (libngt_amd_base.so), at the line's epsilon, with the oracle parity sample
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5x}; mkdir -p $O
for lib in new base; do
  L=$PWD/ngt_amd/libngt_amd.so; [ $lib = base ] && L=$PWD/ngt_amd/libngt_amd_base.so
  C="--cpu-seconds 10"; [ $lib = base ] && C="--no-cpu"
  NGT_AMD_LIB=$L timeout -k 10 540 python -u bench.py --mode qg --graph anng --n 12500000 --anng-batch 8000 \
    --eps 0.12548828125 --steps 3 --warmup 1 $C --latency-queries 0 --anng-line off > $O/c5_$lib.json \
    2> $O/c5_$lib.log || { tail -20 $O/c5_$lib.log; exit 1; }
  python3 scripts/jline.py $O/c5_$lib.json c5_$lib
done
python3 -c "import json; d=json.load(open('$O/c5_new.json')); print((d.get('parity_sample') or {}).get('identical'), (d.get('parity_sample') or {}).get('queries'))"
