#!/bin/bash
# round 6 h: NGTQG record speculation -- the QG suite, then an interleaved A/B
# against the library without it on the qg key's configuration (1M ANNG,
# expansion 3, its epsilon), the speculating run with the oracle parity sample
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6h}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_qg.py -m gpu \
  > $O/pytest_qg.log 2>&1 || { tail -30 $O/pytest_qg.log; exit 1; }
tail -1 $O/pytest_qg.log
D=/tmp/ngt_ab_anng_$$
A="--mode qg --graph anng --anng-dir $D --eps 0.09772 --expansion 3 --steps 10 --warmup 2 --latency-queries 0 --anng-line off --c3-line off --qg-line off"
for r in 1 2; do
  for lib in nospec spec; do
    L=$PWD/ngt_amd/libngt_amd.so; [ $lib = nospec ] && L=$PWD/ngt_amd/libngt_amd_nospec.so
    C="--no-cpu"; [ $lib = spec ] && [ $r = 1 ] && C="--cpu-seconds 8"
    NGT_AMD_LIB=$L timeout -k 10 400 python -u bench.py $A $C > $O/${lib}_$r.json 2> $O/${lib}_$r.log \
      || { tail -20 $O/${lib}_$r.log; exit 1; }
    python3 scripts/jline.py $O/${lib}_$r.json ${lib}_$r
    grep -h "speculation\|parity" $O/${lib}_$r.log || true
  done
done
rm -rf $D
