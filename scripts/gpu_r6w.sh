#!/bin/bash
# round 6 w: serving grid idle counted from the last answer -- the serving
# tests, then the C client runs with the grid log
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6w}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_serve.py \
  tests/test_capi_host.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash scripts/gpu_r6v.sh $O
