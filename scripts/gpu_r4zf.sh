#!/bin/bash
# lookahead parity subset on build A, then A/B of A vs B on the ANNG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zf}; mkdir -p $O
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_a.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_lookahead.py tests/test_gpu_parity.py tests/test_gpu_production.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/gpu_ab.sh ${1:-r4zf}_ab ngt_amd/libngt_amd_a.so ngt_amd/libngt_amd_b.so ${2:-2}
