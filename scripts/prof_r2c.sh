#!/bin/bash
# rocprofv3 passes on one bench mode at its bench-chosen epsilon:
# kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and the SQ VALU counters
# in separate --pmc passes (never combined with other tracing).
# usage: prof_r2c.sh qg|c3|c2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
M=$1; OUT=gpurun_out/prof_$M; mkdir -p $OUT
case $M in
  qg) ARGS="--mode qg --eps 0.056640625"; K="ngt_qg_search_kernel" ;;
  c3) ARGS="--config c3 --eps 0.06523437500000001"; K="ngt_graph_search_kernel" ;;
  c2) ARGS="--eps 0.0703125"; K="ngt_graph_search_kernel|ngt_scan_mfma_kernel" ;;
esac
B="bench.py $ARGS --steps 5 --warmup 1 --no-cpu"
timeout -k 10 500 rocprofv3 --output-format csv --kernel-trace --stats -d $OUT/trace -o run -- python3 $B > $OUT/trace.json 2> $OUT/trace.log || exit $?
python3 scripts/prof_extract.py $OUT/trace "$K" $OUT/${M}_trace || exit 1
timeout -k 10 500 rocprofv3 --output-format csv --kernel-include-regex "$K" --pmc FETCH_SIZE -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.json 2> $OUT/fetch.log || exit $?
python3 scripts/prof_extract.py $OUT/fetch "$K" $OUT/${M}_pmc_fetch || exit 1
timeout -k 10 500 rocprofv3 --output-format csv --kernel-include-regex "$K" --pmc WRITE_SIZE -d $OUT/write -o run -- python3 $B > $OUT/write.json 2> $OUT/write.log || exit $?
python3 scripts/prof_extract.py $OUT/write "$K" $OUT/${M}_pmc_write || exit 1
timeout -k 10 500 rocprofv3 --output-format csv --kernel-include-regex "$K" --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $OUT/sq -o run -- python3 $B > $OUT/sq.json 2> $OUT/sq.log || exit $?
python3 scripts/prof_extract.py $OUT/sq "$K" $OUT/${M}_pmc_sq || exit 1
ls -la $OUT
