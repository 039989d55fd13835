#!/bin/bash
# round 5: the driver's default bench command as it now is (C2 headline +
# anng key with the C-API line + c3 key)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5b}; mkdir -p $O
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log \
  || { tail -30 $O/bench.log; exit 1; }
python3 scripts/jline.py $O/bench.json
