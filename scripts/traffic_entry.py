#!/usr/bin/env python3
"""Per-launch counter figures of one search kernel from the pmc_r3.sh
summaries (<dir>/<name>_{fetch,write,sq}_pmc.json + <name>_kernel_stats.csv),
appended to profiles/traffic.json (an entry with the same workload key is
replaced); with a <name>_tcc_pmc.json (scripts/pmc_r4.sh) also the L2 hit rate
and the DRAM-destined share of the L2's memory-side reads.  Units
(MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE and
WRITE_SIZE are KiB; FETCH_SIZE is doubled (gfx950 tallies 128-B requests at
64 B); SQ_* cycle counters are quad-cycles.
  traffic_entry.py <dir> <name> <kernel-substring> key=value ...  (graph=..., epsilon=..., mode=..., config=...)"""
import csv
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


def pick(p):
    js = json.load(open(os.path.join(d, "%s_%s_pmc.json" % (name, p))))
    ks = [k for k in js if ksub in k]
    assert len(ks) == 1, (p, ks)
    return ks[0], js[ks[0]]


kname, fe = pick("fetch")
_, wr = pick("write")
_, sq = pick("sq")
n = fe["dispatches"]
assert wr["dispatches"] == n and sq["dispatches"] == n
# a search may be several dispatches of the kernel (the probe-and-resume
# schedule: 2); figures are per search
dps = int(key.pop("dispatches_per_search", 1))
n = n / dps
fetch = fe["FETCH_SIZE"] / n * 1024 * 2
write = wr["WRITE_SIZE"] / n * 1024
per = {c: v / n for c, v in sq.items() if c.startswith("SQ_")}
tcc = None
if os.path.exists(os.path.join(d, "%s_tcc_pmc.json" % name)):
    # L2 hit rate and the share of L2 memory-side read requests destined for
    # DRAM (the Infinity Cache sits behind that interface: its hits count)
    _, tc = pick("tcc")
    assert tc["dispatches"] == round(n * dps)
    tcc = {c: v / n for c, v in tc.items() if c.startswith("TCC_")}
    per.update(tcc)
avg_ns = None
with open(os.path.join(d, name + "_kernel_stats.csv")) as f:
    for row in csv.DictReader(f):
        if ksub in row["Name"]:
            avg_ns = float(row["AverageNs"])
search_ns = None
tpath = os.path.join(d, name + "_kernel_trace.csv")
if os.path.exists(tpath):
    # per search, over the timed configuration's dispatches only (the last
    # searches' in the trace, summed per search): the stats file's average
    # also covers the epsilon sweep's launches of other sizes
    with open(tpath) as f:
        rs = [r for r in csv.DictReader(f) if ksub in r["Kernel_Name"]]
    rs.sort(key=lambda r: int(r["Dispatch_Id"]))
    last = rs[-int(round(n * dps)):]
    search_ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last) / n
e = dict(key)
e.update({"kernel": kname.replace("void ngt_amd::", ""), "fetch_bytes": fetch, "write_bytes": write,
          "traffic_bytes": fetch + write, "counters_per_launch": per,
          "trace_avg_kernel_ms": (search_ns if search_ns else avg_ns) / 1e6 if avg_ns else None,
          "dispatches_per_search": dps,
          "source": "%s/%s_{fetch,write,sq}_pmc.json, %s_kernel_stats.csv (scripts/pmc_r4.sh: rocprofv3 "
                    "--kernel-trace --stats, then separate --pmc passes FETCH_SIZE | WRITE_SIZE | %s%s; %d dispatches "
                    "of the timed configuration each, %d per search; FETCH_SIZE x1024 x2, WRITE_SIZE x1024)" % (
                        d, name, name, " ".join(sorted(c for c in per if c.startswith("SQ_"))),
                        (" | " + " ".join(sorted(tcc))) if tcc else "", round(n * dps), dps)})
if tcc:
    e["l2_hit_rate"] = tcc["TCC_HIT_sum"] / max(1.0, tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"])
    e["dram_destined_read_frac"] = tcc["TCC_EA0_RDREQ_DRAM_sum"] / max(1.0, tcc["TCC_EA0_RDREQ_sum"])
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
t = json.load(open(path))
DEF = {"mode": "exact", "config": "c2", "graph": None, "epsilon": None, "visited": -1, "filtered": False}


def wkey(x):
    return tuple(x.get(k, v) for k, v in DEF.items())


t["entries"] = [x for x in t["entries"] if wkey(x) != wkey(e)]
t["entries"].append(e)
json.dump(t, open(path, "w"), indent=1)
print(json.dumps({k: v for k, v in e.items() if k != "counters_per_launch"}, indent=1))
print("active_any %.3f wait_any %.3f wait_inst %.3f valu_active %.3f" % tuple(
    per[c] / per["SQ_WAVE_CYCLES"] for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                             "SQ_ACTIVE_INST_VALU")))
