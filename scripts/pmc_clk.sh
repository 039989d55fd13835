#!/bin/bash
# One counter pass of a bench workload: the SQ issue counters beside the GRBM
# clock (GRBM_GUI_ACTIVE / 8 = the dispatch's cycles, summed over the 8 XCDs;
# MI355X_MICROARCH.md 'DVFS give-back'), so that the SIMDs' issue and VALU
# utilisation come out in measured cycles, not an assumed clock.
#   [PMC_LAST=N] [PMC_SET="counters"] [PMC_TAG=tag] scripts/pmc_clk.sh <outdir> <name> <bench args...>
# (PMC_SET / PMC_TAG: another counter set beside the clock, e.g. the texture
# address / data units' busy cycles, written as <name>_<tag>*)
set -o pipefail
out=$1; name=$2; shift 2
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
C=${PMC_SET:-"SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"}
T=${PMC_TAG:-clk}
timeout -k 10 400 rocprofv3 --pmc $C -d "$R/$out/${name}_$T" -o $T --output-format csv -- \
  python3 "$R/bench.py" "$@" > "$R/$out/${name}_$T.json" 2> "$R/$out/${name}_$T.log" || exit 1
python3 "$R/scripts/pmc_summary.py" "$R/$out" "${name}_$T" --last ${PMC_LAST:-0} > /dev/null || exit 1
echo "$T pass $name done"
