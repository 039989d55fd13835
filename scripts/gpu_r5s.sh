#!/bin/bash
# round 5: (1) the latency kernel's commit-wave phase split on the 1M ANNG
# (stamps build: waits for list parts apart from the list/visited work and the
# accepts); (2) FETCH_SIZE of the 2M one-ANNG NGTQG search with the epoch probe
# after the ADC (new) and before it (base)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5s}; mkdir -p $O
D=/tmp/anng_r5s
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 400 python -u bench.py --graph anng --anng-dir $D \
  --steps 2 --warmup 1 --no-cpu --latency-queries 30 --capi-line off > $O/stamps.json 2> $O/stamps.log \
  || { tail -20 $O/stamps.log; exit 1; }
grep -E "phase|single" $O/stamps.log
R=$PWD
cd /tmp && export TMPDIR=/tmp
for lib in new base; do
  L=$R/ngt_amd/libngt_amd.so; [ $lib = base ] && L=$R/ngt_amd/libngt_amd_base.so
  NGT_AMD_LIB=$L timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/qg2m_${lib}_fetch" -o fetch --output-format csv -- \
    python3 "$R/bench.py" --mode qg --graph anng --n 2000000 --anng-batch 8000 --eps 0.10529 --pmc-launches 3 --no-cpu \
    --latency-queries 0 > "$R/$O/qg2m_${lib}_fetch.json" 2> "$R/$O/qg2m_${lib}_fetch.log" || exit 1
  python3 "$R/scripts/pmc_summary.py" "$R/$O" "qg2m_${lib}_fetch" --last 3 > /dev/null || exit 1
  python3 -c "import json; d=json.load(open(\"$R/$O/qg2m_${lib}_fetch_pmc.json\")); print(\"$lib\", {k: round(v[\"FETCH_SIZE\"] * 1024 / 3 / 1e9, 1) for k, v in d.items() if \"qg_search\" in k})" || exit 1
done
