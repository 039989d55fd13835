#!/bin/bash
# round 5: C3 on the denser surrogate graph against round 4's, then counter
# passes of the C2 headline on the new default graph at the epsilon its sweep picks
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5m}; mkdir -p $O
for g in new old; do
  G=""; [ $g = old ] && G="--knn 128 --out-deg 48 --in-deg 96 --max-deg 160"
  timeout -k 10 500 python -u bench.py --config c3 $G --steps 3 --warmup 1 --no-cpu --latency-queries 0 \
    --anng-line off --c3-line off > $O/c3_$g.json 2> $O/c3_$g.log || { tail -20 $O/c3_$g.log; exit 1; }
  python3 scripts/jline.py $O/c3_$g.json c3_$g
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --anng-line off --c3-line off --no-cpu \
  --latency-queries 0 > $O/c2.json 2> $O/c2.log || { tail -20 $O/c2.log; exit 1; }
python3 scripts/jline.py $O/c2.json c2
EPS=$(python3 -c "import json; print(repr(json.load(open('$O/c2.json'))['config']['epsilon']))")
echo "c2 epsilon $EPS"
PMC_LAST=12 bash scripts/pmc_r4.sh $O c2 --eps $EPS --sweep-nq 10000 --pmc-launches 6 --no-cpu --anng-line off \
  --c3-line off || exit 1
