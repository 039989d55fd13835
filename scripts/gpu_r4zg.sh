#!/bin/bash
# filter threshold cached per exploration radius (C2 and lookahead kernels):
# parity on build B, A/B on C2 and on the ANNG line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zg}; mkdir -p $O
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_b.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_lookahead.py tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_schedule.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/gpu_ab_c2.sh ${1:-r4zg}_c2 ngt_amd/libngt_amd_a.so ngt_amd/libngt_amd_b.so 2 || exit 1
bash scripts/gpu_ab.sh ${1:-r4zg}_anng ngt_amd/libngt_amd_a.so ngt_amd/libngt_amd_b.so 2
