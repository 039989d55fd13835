#!/bin/bash
# round 5: the probe-and-resume budget fraction on the new C2 graph (327
# expansions per query), and the C2-graph QG line on the new graph with parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5o}; mkdir -p $O
for f in 0.06 0.12 0.2; do
  NGT_AMD_TEST_KNOBS=1 NGT_AMD_SCHED_FRAC=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --anng-line off \
    --c3-line off --no-cpu --latency-queries 0 > $O/frac$f.json 2> $O/frac$f.log || { tail -20 $O/frac$f.log; exit 1; }
  python3 scripts/jline.py $O/frac$f.json frac$f
done
timeout -k 10 400 python -u bench.py --mode qg --steps 10 --warmup 2 --cpu-seconds 5 --latency-queries 0 \
  > $O/qg.json 2> $O/qg.log || { tail -20 $O/qg.log; exit 1; }
python3 scripts/jline.py $O/qg.json qg_c2graph
