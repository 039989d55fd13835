#!/usr/bin/env python3
"""Keep what a rocprofv3 output directory says about the kernels we judge:
the kernel-stats summary (all rows, small), and the kernel-trace / counter
rows whose kernel name matches a regex; remove the raw directory.
usage: prof_extract.py DIR REGEX OUTPREFIX"""
import csv
import glob
import os
import re
import shutil
import sys

d, rx, out = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3]
for path in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
    base = os.path.basename(path)
    kind = ("kernel_stats" if base.endswith("kernel_stats.csv") else
            "kernel_trace" if base.endswith("kernel_trace.csv") else
            "counter_collection" if base.endswith("counter_collection.csv") else None)
    if kind is None:
        continue
    with open(path, newline="") as f:
        rows = list(csv.reader(f))
    if not rows:
        continue
    head, body = rows[0], rows[1:]
    if kind != "kernel_stats":
        col = head.index("Kernel_Name") if "Kernel_Name" in head else None
        if col is not None:
            body = [r for r in body if rx.search(r[col])]
    with open("%s_%s.csv" % (out, kind), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(head)
        w.writerows(body)
    print("%s_%s.csv: %d rows" % (out, kind, len(body)))
shutil.rmtree(d, ignore_errors=True)
