#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6x; mkdir -p $O
NGT_AMD_LIB=${LIBX:-$PWD/ngt_amd/libngt_amd.so} timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_serve.py -k grid_stays \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
