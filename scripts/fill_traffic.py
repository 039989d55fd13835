#!/usr/bin/env python3
"""Fill `roofline.traffic` of committed bench lines from the PMC passes that
were taken of the same workload (MI355X_MICROARCH.md: FETCH_SIZE is KiB and
half-counts 16-B/lane reads on gfx950 -> x1024 x2; WRITE_SIZE KiB -> x1024),
per dispatch of the line's search kernel.
  fill_traffic.py <line.json> <fetch_pmc.json> <write_pmc.json> <kernel-substring> [note]"""
import json
import sys

line_p, fetch_p, write_p, ksub = sys.argv[1:5]
note = sys.argv[5] if len(sys.argv) > 5 else ""


def pick(p, c):
    js = json.load(open(p))
    ks = [k for k in js if ksub in k]
    assert len(ks) == 1, ks
    e = js[ks[0]]
    return ks[0], e[c] / e["dispatches"], e["dispatches"]


k, fe, n = pick(fetch_p, "FETCH_SIZE")
_, wr, n2 = pick(write_p, "WRITE_SIZE")
traffic = fe * 1024 * 2 + wr * 1024
d = json.load(open(line_p))
r = d["roofline"]
r["traffic"] = traffic
r["traffic_over_algorithmic"] = traffic / r["algorithmic_bytes_per_launch"]
r["traffic_source"] = ("%s / %s: %s, FETCH_SIZE x1024 x2 + WRITE_SIZE x1024 per dispatch (%d and %d dispatches)%s"
                       % (fetch_p, write_p, k.replace("void ngt_amd::", ""), n, n2, ("; " + note) if note else ""))
json.dump(d, open(line_p, "w"))
print(line_p, "traffic %.4g B per launch = %.2f x algorithmic" % (traffic, r["traffic_over_algorithmic"]))
