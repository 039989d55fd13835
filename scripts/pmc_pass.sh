#!/bin/bash
# One rocprofv3 PMC pass over a bench command (MI355X_MICROARCH.md: counters in
# their own run, --kernel-trace off, one block's slots per pass).
#   scripts/pmc_pass.sh <outdir> <name> "<counters>" -- <bench args...>
set -e
out=$1; name=$2; ctr=$3; shift 4
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --pmc $ctr -d "$GRAFT_REPO_ROOT/$out/$name" -o "$name" --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" "$@" > "$GRAFT_REPO_ROOT/$out/$name.json" 2> "$GRAFT_REPO_ROOT/$out/$name.log"
python3 "$GRAFT_REPO_ROOT/scripts/pmc_summary.py" "$GRAFT_REPO_ROOT/$out" "$name" > /dev/null
