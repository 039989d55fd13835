#!/bin/bash
# Interleaved runs of the ANNG line under environment variants (one built graph):
#   scripts/gpu_abenv.sh <out> <rounds> "<envA>" "<envB>" ["<envC>" ...]   (env "" = defaults)
set -o pipefail
export NGT_AMD_TEST_KNOBS=1  # the library reads NGT_AMD_* knobs only with this set (csrc/knobs.h)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
D=/tmp/anng_abenv
timeout -k 10 400 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 --steps 1 --warmup 1 \
  --no-cpu --latency-queries 0 --anng-line off > $O/build.json 2> $O/build.log || { tail -5 $O/build.log; exit 1; }
for r in $(seq 1 $R); do i=0; for e in "$@"; do i=$((i+1))
  env $e timeout -k 10 300 python3 -u bench.py --graph anng --anng-dir $D --eps 0.1279296875 --sweep-nq 10000 \
    --steps 5 --warmup 1 --no-cpu --latency-queries 0 --anng-line off > $O/v${i}_$r.json 2> $O/v${i}_$r.log || { tail -5 $O/v${i}_$r.log; exit 1; }
  python3 scripts/jline.py $O/v${i}_$r.json "[$e] run $r"
done; done
