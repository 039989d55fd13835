#!/usr/bin/env python3
"""C2-scale reference fixture and CPU-baseline calibration (development container only).

The reference NGT 1.13.8 CLI (built from /root/reference by oracle/ref.mk into
oracle/_ref/; this script only *runs* it) builds the index a user of
``ngt create -d 128 -o f -D 2 -E 10`` gets (ANNG, EdgeSizeForSearch 40, tree
seeds; Command.cpp:26-170) over the C2 data (1M x 128 splitmix64 U[0,1),
bench.py's generator), and then:

* ``build``   -- times ``ngt create`` (24 creation threads, the CLI default)
  and records the sha256 of the obj/grp/tre/prf files it writes;
* ``truth``   -- exact top-10 of the first ``--nq`` queries with the
  reference's own linear search (``ngt search -i s``);
* ``sweep``   -- ``ngt search -o e`` (read-only, tree seeds, EdgeSizeForSearch
  from the prf) over epsilon until mean recall@10 >= 0.95 (ngt eval semantics);
* ``time``    -- the reference's QPS at that epsilon: one query thread (the
  mean of its per-query Timer, Command.cpp:305-323) and P concurrent
  ``ngt search`` processes on disjoint query shards, next to
  the oracle restatement (oracle/ngt_oracle.c, what bench.py's cpu_baseline
  runs on the GPU box) on the same index, queries, epsilon and threads, whose
  ids and distances must equal the reference's -- the calibration ratio;
* ``fixture`` -- writes tests/golden/c2_anng_ref.json + c2_anng_ref.npz: the
  sha256s, the epsilon, the reference's ids/distances for the first 200
  queries, and the timings.  bench.py --graph anng and the GPU tests check the
  device-built index and its searches against them.

    python3 tests/golden/make_c2_anng_fixture.py --stage all
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from bench import BASE_SEED, splitmix_uniform  # noqa: E402
import ngt_files  # noqa: E402

N, D = 1_000_000, 128


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def write_tsv(path, a):
    # values are j * 2^-24: %.9g round-trips every float32 exactly
    with open(path, "w") as f:
        for s in range(0, a.shape[0], 20000):
            blk = a[s:s + 20000]
            f.write("\n".join("\t".join("%.9g" % v for v in r) for r in blk.tolist()))
            f.write("\n")


def env_of(args):
    return dict(os.environ, LD_LIBRARY_PATH=os.path.join(ROOT, "oracle", "_ref"))


def run(cmd, env, out=None):
    r = subprocess.run(cmd, env=env, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("%s failed:\n%s\n%s" % (cmd, r.stdout[-2000:], r.stderr[-2000:]))
    if out:
        with open(out, "w") as f:
            f.write(r.stdout)
    return r.stdout


def stage_data(args):
    os.makedirs(args.work, exist_ok=True)
    dpath = os.path.join(args.work, "data.tsv")
    if not os.path.exists(dpath):
        t0 = time.time()
        write_tsv(dpath + ".tmp", splitmix_uniform(N, D, BASE_SEED))
        os.rename(dpath + ".tmp", dpath)
        print("data.tsv written in %.1f s" % (time.time() - t0), flush=True)
    qpath = os.path.join(args.work, "queries.tsv")
    if not os.path.exists(qpath):
        write_tsv(qpath, splitmix_uniform(args.nq, D, BASE_SEED + 1))


def stage_build(args):
    idx = os.path.join(args.work, "anng")
    meta = os.path.join(args.work, "build.json")
    if os.path.exists(meta):
        return json.load(open(meta))
    env = env_of(args)
    t0 = time.time()
    run([args.ngt, "create", "-d", str(D), "-o", "f", "-D", "2", "-E", "10", idx,
         os.path.join(args.work, "data.tsv")], env, out=os.path.join(args.work, "create.log"))
    el = time.time() - t0
    m = {"build_s": el, "threads": 24, "cpus": os.cpu_count(),
         "sha256": {f: sha256(os.path.join(idx, f)) for f in ("prf", "obj", "grp", "tre")}}
    json.dump(m, open(meta, "w"), indent=1)
    print("ngt create: %.1f s" % el, flush=True)
    return m


def parse(text):
    return ngt_files.parse_search_output(text)


def search(args, idx, qpath, eps, mode="t", k=10, extra=()):
    out = run([args.ngt, "search", "-n", str(k), "-e", str(eps), "-i", mode, "-o", "e", *extra, idx, qpath],
              env_of(args))
    return parse(out)


def recall(ids, gt, k=10):
    return float(np.mean([len(set(a[:k]) & set(b[:k])) / k for a, b in zip(ids, gt)]))


def stage_truth(args):
    path = os.path.join(args.work, "truth.npz")
    if os.path.exists(path):
        return np.load(path)["ids"]
    t0 = time.time()
    r = search(args, os.path.join(args.work, "anng"), os.path.join(args.work, "queries.tsv"), 0.0, mode="s")
    ids = np.array([q["ids"] for q in r], np.int64)
    np.savez(path, ids=ids, dists=np.array([q["dists"] for q in r], np.float64))
    print("linear ground truth of %d queries in %.1f s" % (len(ids), time.time() - t0), flush=True)
    return ids


def stage_sweep(args, gt):
    path = os.path.join(args.work, "sweep.json")
    if os.path.exists(path):
        return json.load(open(path))
    idx, q = os.path.join(args.work, "anng"), os.path.join(args.work, "queries.tsv")
    pts = []
    eps = 0.0
    chosen = None
    for eps in [0.0, 0.02, 0.04, 0.06, 0.08, 0.1, 0.12, 0.14, 0.16, 0.18, 0.2, 0.25, 0.3, 0.4, 0.5]:
        r = search(args, idx, q, eps)
        rc = recall([x["ids"] for x in r], gt)
        pts.append({"epsilon": eps, "recall": rc, "ms": float(np.mean([x["time_ms"] for x in r]))})
        print("eps %.3f recall %.4f %.3f ms/query" % (eps, rc, pts[-1]["ms"]), flush=True)
        if rc >= args.target:
            chosen = eps
            break
    # bisect between the last two points to 0.005
    if chosen is not None and len(pts) > 1:
        lo, hi = pts[-2]["epsilon"], chosen
        while hi - lo > 0.0051:
            mid = round(0.5 * (lo + hi), 4)
            r = search(args, idx, q, mid)
            rc = recall([x["ids"] for x in r], gt)
            pts.append({"epsilon": mid, "recall": rc, "ms": float(np.mean([x["time_ms"] for x in r]))})
            print("eps %.4f recall %.4f" % (mid, rc), flush=True)
            if rc >= args.target:
                hi = mid
            else:
                lo = mid
        chosen = hi
    s = {"points": pts, "epsilon": chosen}
    json.dump(s, open(path, "w"), indent=1)
    return s


def stage_time(args, eps, gt):
    """Reference QPS (1 thread; P processes) and the oracle port on the same
    index, queries and epsilon; ids/distances must match the reference."""
    import oracle_py as O
    idx, q = os.path.join(args.work, "anng"), os.path.join(args.work, "queries.tsv")
    env = env_of(args)
    r1 = search(args, idx, q, eps)
    ref_ms = float(np.mean([x["time_ms"] for x in r1]))
    # P concurrent processes over disjoint query shards
    P = args.procs
    qs = np.loadtxt(q, dtype=np.float32)
    parts = np.array_split(np.arange(len(qs)), P)
    paths = []
    for p, sel in enumerate(parts):
        pp = os.path.join(args.work, "q_part%d.tsv" % p)
        write_tsv(pp, qs[sel])
        paths.append(pp)
    # each process's busy time = the sum of its per-query Timer values (the
    # index load, seconds per process, is not search time)
    outs = [open(pp + ".out", "w") for pp in paths]
    procs = [subprocess.Popen([args.ngt, "search", "-n", "10", "-e", str(eps), "-o", "e", idx, pp], env=env,
                              stdout=o, stderr=subprocess.DEVNULL) for pp, o in zip(paths, outs)]
    for pr, o in zip(procs, outs):
        pr.wait()
        o.close()
    busy = [sum(x["time_ms"] for x in parse(open(pp + ".out").read())) / 1e3 for pp in paths]
    ref_qps_p = len(qs) / max(busy)
    # the oracle restatement on the reference's own index files
    prf = ngt_files.read_prf(os.path.join(idx, "prf"))
    rows = ngt_files.read_obj(os.path.join(idx, "obj"), D, np.float32)[0]
    offs, edges = ngt_files.read_grp(os.path.join(idx, "grp"))[:2]
    tree = ngt_files.read_tre(os.path.join(idx, "tre"), D, np.float32)
    qp = np.zeros((len(qs), ngt_files.padded_dim(D)), np.float32)
    qp[:, :D] = qs
    es = int(prf.get("EdgeSizeForSearch", 40))
    seeds = [O.tree_seeds("l2", tree, qp[i], 10, seed_size=int(prf.get("SeedSize", 10)))[0] for i in range(len(qp))]
    sm = max(len(s) for s in seeds)
    sarr = np.zeros((len(qp), sm), np.uint32)
    for i, s in enumerate(seeds):
        sarr[i, :len(s)] = s
    L = O.native_lib(O.host_isa())
    out = {}
    for th in (1, P):
        t0 = time.perf_counter()
        oi, od, on, oc = O.search_batch("l2", rows, offs.astype(np.uint64), edges.astype(np.uint32), qp, sarr, 10,
                                         np.float32(eps), edge_size=es, threads=th, L=L)
        out[th] = (len(qp) / (time.perf_counter() - t0), oi, od, on)
    oi, od, on = out[1][1:]
    same = True
    for i, x in enumerate(r1):
        n = int(on[i])
        if list(oi[i, :n]) != list(x["ids"]) or not np.allclose(od[i, :n], x["dists"], rtol=2e-6, atol=0):
            same = False
            print("query %d differs: oracle %s ref %s" % (i, list(oi[i, :n]), x["ids"]), flush=True)
            break
    t = {"epsilon": eps, "queries": len(qs), "reference_ms_per_query_1thread": ref_ms,
         "reference_qps_1thread": 1000.0 / ref_ms, "reference_qps_%dproc" % P: ref_qps_p,
         "port_qps_1thread": out[1][0], "port_qps_%dthread" % P: out[P][0],
         "ratio_port_over_reference_1thread": out[1][0] / (1000.0 / ref_ms),
         "ratio_port_over_reference_%d" % P: out[P][0] / ref_qps_p,
         "port_identical_to_reference": same, "container_cores": os.cpu_count(),
         "recall_at_10": recall([x["ids"] for x in r1], gt)}
    print(json.dumps(t, indent=1), flush=True)
    return t, r1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", default="all", choices=["data", "build", "truth", "sweep", "time", "all"])
    ap.add_argument("--work", default="/tmp/c2anng")
    ap.add_argument("--ngt", default=os.path.join(ROOT, "oracle", "_ref", "ngt"))
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--fixture-nq", type=int, default=200)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--target", type=float, default=0.95)
    args = ap.parse_args()
    stage_data(args)
    if args.stage == "data":
        return
    b = stage_build(args)
    if args.stage == "build":
        return
    gt = stage_truth(args)
    if args.stage == "truth":
        return
    sw = stage_sweep(args, gt)
    if args.stage == "sweep":
        return
    t, r1 = stage_time(args, sw["epsilon"], gt)
    fn = args.fixture_nq
    ids = np.zeros((fn, 10), np.uint32)
    dists = np.zeros((fn, 10), np.float64)
    n = np.zeros(fn, np.uint32)
    for i in range(fn):
        m = len(r1[i]["ids"])
        ids[i, :m] = r1[i]["ids"]
        dists[i, :m] = r1[i]["dists"]
        n[i] = m
    np.savez_compressed(os.path.join(HERE, "c2_anng_ref.npz"), ids=ids, dists=dists, n=n,
                        truth=gt[:fn].astype(np.uint32))
    meta = {"command": "ngt create -d 128 -o f -D 2 -E 10 (defaults: -S 40 -b 200 -e 0.1 -p 24, ANNG + DVP tree)",
            "data": "splitmix64 U[0,1), seed 0x4E4754, 1,000,000 x 128 (bench.py splitmix_uniform)",
            "queries": "splitmix64 seed 0x4E4755, first %d rows" % args.nq,
            "build": b, "sweep": sw, "timing": t,
            "fixture": "c2_anng_ref.npz: ngt search -n 10 -e %g -i t -o e (read-only), first %d queries" % (
                sw["epsilon"], fn)}
    json.dump(meta, open(os.path.join(HERE, "c2_anng_ref.json"), "w"), indent=1)
    print("fixture written", flush=True)


if __name__ == "__main__":
    main()
