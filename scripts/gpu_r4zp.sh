#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the one-graph C4 (10M ANNG) and C5 (12.5M
# NGTQG over one ANNG) lines at their committed epsilons, one launch each
# (--pmc-launches 1, PMC_LAST=1: only the last dispatch of the search kernel)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4zp}; mkdir -p "$R/$O"
cd /tmp && export TMPDIR=/tmp
run_pass() {  # name pass counter bench-args...
  local name=$1 pass=$2 C=$3; shift 3
  timeout -k 10 ${PT:-270} rocprofv3 --pmc $C -d "$R/$O/${name}_$pass" -o $pass --output-format csv -- \
    python3 "$R/bench.py" "$@" > "$R/$O/${name}_$pass.json" 2> "$R/$O/${name}_$pass.log" || return 1
  python3 "$R/scripts/pmc_summary.py" "$R/$O" "${name}_$pass" --last 1 > /dev/null
}
C4="--graph anng --n 10000000 --anng-batch 8000 --eps 0.16082763671875 --pmc-launches 1 --no-cpu --latency-queries 0 --anng-line off"
C5="--mode qg --graph anng --n 12500000 --anng-batch 8000 --eps 0.12548828125 --pmc-launches 1 --no-cpu --latency-queries 0 --anng-line off"
run_pass c4 fetch FETCH_SIZE $C4 && run_pass c4 write WRITE_SIZE $C4 && echo "c4 passes done" && \
run_pass c5 fetch FETCH_SIZE $C5 && run_pass c5 write WRITE_SIZE $C5 && echo "c5 passes done"
