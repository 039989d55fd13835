#!/bin/bash
# Kernel trace + PMC passes of one bench workload (MI355X_MICROARCH.md: counters
# in their own runs, one block's slots per pass; FETCH_SIZE and WRITE_SIZE
# apart).  The bench runs with a fixed epsilon and --pmc-launches, so every
# dispatch of the search kernel is the timed configuration.  The tcc pass: L2
# hits/misses and the L2 memory-side read requests (all of them, and those
# destined for DRAM -- Infinity-Cache hits included: no TCC counter separates
# them).
#   [PMC_LAST=N] scripts/pmc_r4.sh <outdir> <name> <bench args...>
# (PMC_LAST: count only each kernel's last N dispatches -- the --pmc-launches
# searches; a scheduled search is two dispatches, probe and resume)
# writes <outdir>/<name>_{trace,fetch,write,sq,tcc}{.json,.log,_pmc.json} and the
# trace's kernel_stats.csv.
set -o pipefail
out=$1; name=$2; shift 2
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
TCC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$out/${name}_trace" -o trace --output-format csv -- \
  python3 "$R/bench.py" "$@" > "$R/$out/${name}_trace.json" 2> "$R/$out/${name}_trace.log" || exit 1
find "$R/$out/${name}_trace" -name "*kernel_stats.csv" -exec cp {} "$R/$out/${name}_kernel_stats.csv" \;
find "$R/$out/${name}_trace" -name "*kernel_trace.csv" -exec cp {} "$R/$out/${name}_kernel_trace.csv" \;
rm -rf "$R/$out/${name}_trace"
for pass in fetch write sq tcc; do
  case $pass in fetch) C="FETCH_SIZE";; write) C="WRITE_SIZE";; sq) C="$SQ";; tcc) C="$TCC";; esac
  timeout -k 10 400 rocprofv3 --pmc $C -d "$R/$out/${name}_$pass" -o $pass --output-format csv -- \
    python3 "$R/bench.py" "$@" > "$R/$out/${name}_$pass.json" 2> "$R/$out/${name}_$pass.log" || exit 1
  python3 "$R/scripts/pmc_summary.py" "$R/$out" "${name}_$pass" --last ${PMC_LAST:-0} > /dev/null || exit 1
done
echo "pmc $name done"
