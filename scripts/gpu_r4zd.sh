#!/bin/bash
# lookahead kernel, targets from registers in phase B, 16-byte hash clears, unconditional commit reads: parity, ANNG launch time, phase split
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zd}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lookahead.py \
  tests/test_gpu_parity.py tests/test_gpu_production.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
D=/tmp/anng_r4zd
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 3 --warmup 1 \
  --no-cpu --latency-queries 0 --anng-line off > $O/anng.json 2> $O/anng.log || { tail -5 $O/anng.log; exit 1; }
python3 scripts/jline.py $O/anng.json anng
grep -E "identical|evaluations" $O/anng.log
for w in 4 16; do
  NGT_AMD_WAVES_PER_CU=$w NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D \
    --steps 2 --warmup 1 --no-cpu --latency-queries 0 --eps 0.128 --anng-line off > $O/stamps_w$w.json 2> $O/stamps_w$w.log || { tail -20 $O/stamps_w$w.log; exit 1; }
  echo "waves/CU $w"; grep -E "phase|kernel .* \(10000" $O/stamps_w$w.log
done
