#!/bin/bash
# A/B of two library builds on the ANNG line (interleaved runs, one built graph):
#   scripts/gpu_ab.sh <out> <libA> <libB> [rounds]
set -o pipefail
export NGT_AMD_TEST_KNOBS=1  # the library reads NGT_AMD_* knobs only with this set (csrc/knobs.h)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; mkdir -p $O
D=/tmp/anng_ab
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 1 --warmup 1 \
  --no-cpu --latency-queries 0 --anng-line off > $O/build.json 2> $O/build.log || { tail -5 $O/build.log; exit 1; }
for r in $(seq 1 ${4:-3}); do for v in A B; do
  L=$2; [ $v = B ] && L=$3
  NGT_AMD_LIB=$PWD/$L timeout -k 10 300 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 \
    --steps 5 --warmup 1 --no-cpu --latency-queries 0 --anng-line off > $O/$v$r.json 2> $O/$v$r.log || { tail -5 $O/$v$r.log; exit 1; }
  python3 scripts/jline.py $O/$v$r.json "$v run $r"
done; done
