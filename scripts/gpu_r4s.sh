#!/bin/bash
# accepted-only lookahead: the visited test moved from every list entry to the
# survivors (rides with their exact rows) -- parity, the ANNG line, accounting
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4s}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lookahead.py \
  tests/test_gpu_parity.py -k "lookahead or accepted or reference" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --graph anng --anng-line off --steps 3 --warmup 1 \
  --no-cpu --latency-queries 0 --eps 0.128 > $O/anng.json 2> $O/anng.log || { tail -20 $O/anng.log; exit 1; }
python3 scripts/jline.py $O/anng.json anng
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_lacount.so timeout -k 10 400 python -u bench.py --graph anng --anng-line off --steps 2 --warmup 1 \
  --no-cpu --latency-queries 0 --eps 0.128 > $O/lacount_anng.json 2> $O/lacount_anng.log || { tail -20 $O/lacount_anng.log; exit 1; }
grep -E "accounting" $O/lacount_anng.log
