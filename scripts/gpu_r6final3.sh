#!/bin/bash
# round 6 final (3): the whole GPU suite, the smoke and the driver's bench
# command on the committed tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r6final3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash scripts/gpu_r6final2.sh $O
