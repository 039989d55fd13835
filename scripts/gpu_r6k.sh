#!/bin/bash
# round 6 k: NGTQG entry speculation (the next key's entries under the
# current expansion, its probes beside its code loads) -- the QG suite, then an
# interleaved A/B against the committed library on the qg key's configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6k}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_qg.py -m gpu \
  > $O/pytest_qg.log 2>&1 || { tail -30 $O/pytest_qg.log; exit 1; }
tail -1 $O/pytest_qg.log
D=/tmp/ngt_ab_anng_$$
A="--mode qg --graph anng --anng-dir $D --eps 0.09772 --expansion 3 --steps 10 --warmup 2 --latency-queries 0 --anng-line off --c3-line off --qg-line off"
for r in 1 2; do
  for lib in base spec; do
    L=$PWD/ngt_amd/libngt_amd.so; [ $lib = base ] && L=$PWD/ngt_amd/libngt_amd_base.so
    C="--no-cpu"; [ $lib = spec ] && [ $r = 1 ] && C="--cpu-seconds 8"
    NGT_AMD_LIB=$L timeout -k 10 400 python -u bench.py $A $C > $O/${lib}_$r.json 2> $O/${lib}_$r.log \
      || { tail -20 $O/${lib}_$r.log; exit 1; }
    python3 scripts/jline.py $O/${lib}_$r.json ${lib}_$r
    grep -h "parity" $O/${lib}_$r.log || true
  done
done
rm -rf $D
