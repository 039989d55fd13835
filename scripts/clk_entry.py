#!/usr/bin/env python3
"""Add the SIMD issue figures of a pmc_clk.sh pass to the matching
profiles/traffic.json entry: cycles per dispatch = GRBM_GUI_ACTIVE / 8 (summed
over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'); SIMD quad-cycles =
cycles / 4 x 1024 SIMDs; SQ_* cycle counters are quad-cycles summed over
waves.  simd_issue_util = SQ_ACTIVE_INST_ANY / SIMD quad-cycles (a quad-cycle
in which two waves of one SIMD issue counts twice, so it can pass 1);
simd_valu_util = SQ_ACTIVE_INST_VALU / SIMD quad-cycles; waves_per_simd =
SQ_WAVE_CYCLES / SIMD quad-cycles.
  clk_entry.py <dir> <name> <kernel-substring> key=value ...  (the entry's workload key)"""
import json
import os
import sys

d, name, ksub = sys.argv[1:4]
key = {}
for kv in sys.argv[4:]:
    k, v = kv.split("=", 1)
    try:
        v = json.loads(v)
    except ValueError:
        pass
    key[k] = v
js = json.load(open(os.path.join(d, "%s_clk_pmc.json" % name)))
ks = [k for k in js if ksub in k]
assert len(ks) == 1, ks
e = js[ks[0]]
cycles = e["GRBM_GUI_ACTIVE"] / 8.0
quads = cycles / 4.0 * 1024
clk = {"source": "%s/%s_clk_pmc.json (scripts/pmc_clk.sh: one --pmc pass of %s and GRBM_GUI_ACTIVE "
                 "GRBM_COUNT over %d dispatches of the timed configuration)" % (
                     d, name, " ".join(sorted(c for c in e if c.startswith("SQ_"))), e["dispatches"]),
       "cycles_per_dispatch": cycles / e["dispatches"],
       "simd_issue_util": e["SQ_ACTIVE_INST_ANY"] / quads,
       "simd_valu_util": e["SQ_ACTIVE_INST_VALU"] / quads,
       "waves_per_simd": e["SQ_WAVE_CYCLES"] / quads,
       "salu_per_valu": e["SQ_INSTS_SALU"] / e["SQ_INSTS_VALU"]}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
t = json.load(open(path))
DEF = {"mode": "exact", "config": "c2", "graph": None, "epsilon": None, "visited": -1, "filtered": False}
hit = [x for x in t["entries"] if all(x.get(k, v) == key.get(k, v) for k, v in DEF.items())]
assert len(hit) == 1, (key, len(hit))
ms = hit[0].get("trace_avg_kernel_ms")
if ms:
    clk["effective_clock_ghz"] = cycles / e["dispatches"] * hit[0].get("dispatches_per_search", 1) / (ms * 1e-3) / 1e9
hit[0]["simd_issue"] = clk
json.dump(t, open(path, "w"), indent=1)
print(json.dumps(clk, indent=1))
