#!/bin/bash
# round 5: (1) the C2 kernel's phase split (stamps build) on the kNN256 graph;
# (2) FETCH_SIZE of the C5 one-graph NGTQG search (12.5M, device ANNG -b 8000,
# tree seeds) with the epoch probe after the ADC, plus its kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r5w}; mkdir -p $O
NGT_AMD_LIB=$PWD/ngt_amd/libngt_amd_stamps.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu \
  --latency-queries 0 --anng-line off --c3-line off > $O/stamps_c2.json 2> $O/stamps_c2.log || { tail -20 $O/stamps_c2.log; exit 1; }
grep -E "phase|expansions" $O/stamps_c2.log
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/c5_fetch" -o fetch --output-format csv -- \
  python3 "$R/bench.py" --mode qg --graph anng --n 12500000 --anng-batch 8000 --eps 0.12548828125 --pmc-launches 3 \
  --no-cpu --latency-queries 0 --anng-line off > "$R/$O/c5_fetch.json" 2> "$R/$O/c5_fetch.log" || exit 1
python3 "$R/scripts/pmc_summary.py" "$R/$O" c5_fetch --last 3 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$R/$O/c5_fetch_pmc.json')); print({k: v['FETCH_SIZE'] for k, v in d.items() if 'qg_search' in k})"
python3 -c "import json; d=json.load(open('$R/$O/c5_fetch.json')); print(d.get('pmc_launches'), d.get('kernel_ms_last'), d.get('recall_at_10'))"
