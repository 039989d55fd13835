#!/bin/bash
# FETCH_SIZE calibration of the search kernels' load shapes (scripts/calib)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r4k}; mkdir -p $O; R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/fetch" -o fetch --output-format csv -- "$R/scripts/calib/fetch_calib" > "$R/$O/calib.txt" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_MISS_sum -d "$R/$O/tcc" -o tcc --output-format csv -- "$R/scripts/calib/fetch_calib" > /dev/null 2>&1 || exit 1
cd "$R"
python3 scripts/pmc_summary.py $O fetch --match k_
python3 scripts/pmc_summary.py $O tcc --match k_
cat $O/calib.txt
