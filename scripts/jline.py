#!/usr/bin/env python3
"""One summary line of a bench.py JSON result: label, QPS, recall, per-launch ms, frac."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d.get("roofline") or {}
print(sys.argv[2] if len(sys.argv) > 2 else sys.argv[1], round(d["value"]), d["config"].get("recall_at_10"),
      round(r.get("kernel_ms", float("nan")), 2), round(r.get("frac", float("nan")), 3), round(d["ms_per_step"], 2))
