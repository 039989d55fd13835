#!/usr/bin/env python3
"""Add the texture-address-unit figures of a pmc_clk.sh pass (PMC_TAG=ta:
TA_BUSY_avr, SQ_INSTS_VMEM_RD/WR beside GRBM_GUI_ACTIVE) to the
profiles/traffic.json entry that carries the same kernel's simd_issue pass
(matched by its simd_issue source file name <dir>/<name>_clk_pmc.json):
ta_busy_frac = TA_BUSY_avr / (GRBM_GUI_ACTIVE / 8), the mean TA instance's
busy share of the dispatch's cycles; vmem_per_cu_cycle = vector-memory
instructions per CU per cycle.
  ta_entry.py <ta-dir> <name> <kernel-substring> <clk-source-substring>"""
import json
import os
import sys

d, name, ksub, src = sys.argv[1:5]
js = json.load(open(os.path.join(d, "%s_ta_pmc.json" % name)))
ks = [k for k in js if ksub in k]
assert len(ks) == 1, ks
e = js[ks[0]]
cycles = e["GRBM_GUI_ACTIVE"] / 8.0
ta = {"source": "%s/%s_ta_pmc.json (scripts/pmc_clk.sh with PMC_TAG=ta: TA_BUSY_avr SQ_INSTS_VMEM_RD "
                "SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT over %d dispatches of the timed "
                "configuration)" % (d, name, e["dispatches"]),
      "ta_busy_frac": e["TA_BUSY_avr"] / cycles,
      "vmem_per_cu_cycle": (e["SQ_INSTS_VMEM_RD"] + e["SQ_INSTS_VMEM_WR"]) / (cycles * 256)}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
t = json.load(open(path))
hit = [x for x in t["entries"] if src in (x.get("simd_issue") or {}).get("source", "")]
assert len(hit) == 1, (src, len(hit))
hit[0]["texture_address"] = ta
json.dump(t, open(path, "w"), indent=1)
print(json.dumps(ta, indent=1))
