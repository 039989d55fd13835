#!/bin/bash
# parity subset on build B, then the ANNG line A/B (A = committed, B = working tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zi}; mkdir -p $O
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_b.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_schedule.py tests/test_gpu_lookahead.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/gpu_ab.sh ${1:-r4zi}_anng ngt_amd/libngt_amd_a.so ngt_amd/libngt_amd_b.so ${2:-3}
