#!/bin/bash
# A/B of two library builds on the C2 headline (interleaved, 20 overlapped steps each)
#   scripts/gpu_ab_c2.sh <out> <libA> <libB> [rounds]
set -o pipefail
export NGT_AMD_TEST_KNOBS=1  # the library reads NGT_AMD_* knobs only with this set (csrc/knobs.h)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; mkdir -p $O
for r in $(seq 1 ${4:-2}); do for v in A B; do
  L=$2; [ $v = B ] && L=$3
  NGT_AMD_LIB=$PWD/$L timeout -k 10 300 python3 -u bench.py --no-cpu --latency-queries 0 --anng-line off --steps 20 \
    > $O/$v$r.json 2> $O/$v$r.log || { tail -5 $O/$v$r.log; exit 1; }
  python3 scripts/jline.py $O/$v$r.json "C2 $v run $r"
done; done
