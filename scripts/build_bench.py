#!/usr/bin/env python3
"""Time ANNG construction on the device (DeviceIndex.build_anng) on synthetic
clustered 128-d float rows, and check the structural invariants of the result:
edge lists sorted by (distance, id), no self loops or duplicates, stored
distances equal to recomputed L2, every object in exactly one DVP-tree leaf,
and graph search recall against the exact linear search.

    python scripts/build_bench.py --n 100000
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ngt_amd.device import DeviceIndex  # noqa: E402


def synth(n, dim, seed):
    rng = np.random.default_rng(seed)
    nc = max(16, n // 500)
    centers = rng.uniform(0, 120, size=(nc, dim)).astype(np.float32)
    lab = rng.integers(0, nc, size=n)
    x = centers[lab] + rng.normal(0, 12, size=(n, dim)).astype(np.float32)
    return np.clip(np.rint(x), 0, 255).astype(np.float32)


def check(offs, ids, ds, tree, rows, n, sample, rng):
    deg = np.diff(offs.astype(np.int64))
    assert deg[0] == 0 and (deg[1:] > 0).all(), "every object gets a node with edges"
    for v in rng.choice(np.arange(1, n + 1), size=min(sample, n), replace=False):
        a, b = int(offs[v]), int(offs[v + 1])
        e, d = ids[a:b].astype(np.int64), ds[a:b]
        assert (e != v).all() and len(set(e.tolist())) == len(e), v
        assert all(d[i] < d[i + 1] or (d[i] == d[i + 1] and e[i] < e[i + 1]) for i in range(len(e) - 1)), v
        ref = np.sqrt(((rows[e].astype(np.float64) - rows[v].astype(np.float64)) ** 2).sum(1))
        assert np.allclose(d, ref, rtol=1e-5, atol=1e-3), v
    lid = np.sort(tree["leaf_ids"].astype(np.int64))
    assert np.array_equal(lid, np.arange(1, n + 1)), "tree leaves hold every object once"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--edges", type=int, default=10)
    ap.add_argument("--batch", type=int, default=200, help="batchSizeForCreation")
    ap.add_argument("--check", type=int, default=2000, help="nodes whose edge lists are checked")
    ap.add_argument("--queries", type=int, default=200)
    args = ap.parse_args()
    x = synth(args.n + args.queries, args.dim, args.seed)
    data, qs = x[:args.n], x[args.n:]
    rows = np.zeros((args.n + 1, args.dim), np.float32)
    rows[1:] = data
    ix = DeviceIndex("l2", "float", args.dim)
    ix.set_objects(rows)
    t0 = time.perf_counter()
    (offs, ids, ds), tree = ix.build_anng(edge_size_for_creation=args.edges,
                                             batch_size_for_creation=args.batch)
    t1 = time.perf_counter()
    check(offs, ids, ds, tree, rows, args.n, args.check, np.random.default_rng(1))
    ix.set_tree(tree)
    gi, _, _, _ = ix.search(qs, k=10, epsilon=0.1)
    li, _, _ = ix.linear_search(qs, k=10)
    recall = float(np.mean([len(set(gi[i]) & set(li[i])) / 10.0 for i in range(len(qs))]))
    out = {"n": args.n, "dim": args.dim, "edge_size_for_creation": args.edges, "batch": args.batch,
           "build_s": t1 - t0,
           "objects_per_s": args.n / (t1 - t0), "edges": int(len(ids)),
           "mean_degree": float(len(ids)) / args.n, "recall_at_10_eps0.1": recall}
    print(json.dumps(out))
    ix.close()


if __name__ == "__main__":
    main()
