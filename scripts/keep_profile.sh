#!/bin/bash
# Copy a GPU run's summaries from gpurun_out/<src> into profiles/<dst>:
# JSON lines, logs, *_pmc.json, and the kernel trace/stats CSVs reduced to
# the header + this library's kernels (the raw traces also hold torch's setup).
src=$1; dst=$2
mkdir -p "profiles/$dst"
for f in gpurun_out/$src/*; do
  b=$(basename "$f")
  case "$b" in
    *_kernel_stats.csv) { head -1 "$f"; grep "ngt_amd" "$f"; } > "profiles/$dst/$b" ;;
    *_kernel_trace.csv) { head -1 "$f"; grep -E "search_(la_|lat_)?kernel|qg_search_kernel|scan_mfma_kernel" "$f"; } > "profiles/$dst/$b" ;;
    *.json|*.log) cp "$f" "profiles/$dst/$b" ;;
  esac
done
