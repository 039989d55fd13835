#!/usr/bin/env python3
"""Condense rocprofv3 counter_collection CSVs to per-kernel sums (the raw
per-dispatch files exceed what a GPU run may bring back).  Writes
<dir>/<name>_pmc.json: {kernel: {"dispatches": n, counter: sum, ...}} for the
kernels matching --match (default: ngt_), then deletes the raw directory."""
import argparse
import csv
import glob
import json
import os
import shutil

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("name")
ap.add_argument("--match", default="ngt_")
ap.add_argument("--keep", action="store_true")
ap.add_argument("--last", type=int, default=0,
                help="per kernel, only its last N dispatches (the timed configuration's, after the setup launches)")
a = ap.parse_args()
raw = os.path.join(a.dir, a.name)
out = {}
rows = []
for f in glob.glob(os.path.join(raw, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        rows += [r for r in csv.DictReader(fh) if a.match in r.get("Kernel_Name", "")]
keep = None
if a.last:
    ids = {}
    for r in rows:
        ids.setdefault(r["Kernel_Name"].split("(")[0], set()).add(int(r["Dispatch_Id"]))
    keep = {k: set(sorted(v)[-a.last:]) for k, v in ids.items()}
for row in rows:
    k = row["Kernel_Name"].split("(")[0]
    if keep is not None and int(row["Dispatch_Id"]) not in keep[k]:
        continue
    e = out.setdefault(k, {"dispatches": set()})
    e["dispatches"].add(row.get("Dispatch_Id"))
    c = row.get("Counter_Name")
    e[c] = e.get(c, 0.0) + float(row.get("Counter_Value", 0))
for k, e in out.items():
    e["dispatches"] = len(e["dispatches"])
json.dump(out, open(os.path.join(a.dir, a.name + "_pmc.json"), "w"), indent=1)
if not a.keep:
    shutil.rmtree(raw, ignore_errors=True)
print(json.dumps(out, indent=1))
