#!/usr/bin/env python3
"""Generate the committed golden fixtures from the reference NGT 1.13.8 CLI.

Run in the development container only (never on the GPU box):

    make -f oracle/ref.mk                      # the reference, built from its sources
    python3 tests/golden/make_goldens.py --out tests/golden

The `ngt` binary is the reference built from /root/reference by the committed
recipe oracle/ref.mk into oracle/_ref/; this script only *runs* it.
``--subset quick`` regenerates only the C1 ANNG, its tree-seeded searches at
epsilon 0.1 and two comparator fixtures (what tests/test_golden_regen.py
compares against the committed files).  It writes:

* ``c1_anng/``   -- the reference-built index for BASELINE config 1
  (``ngt create -d 128 -o f -D 2`` on data/sift-dataset-5k.tsv): prf/obj/grp/tre
  exactly as the reference wrote them.
* ``c1_onng/``   -- ANNG(E=100) + ``reconstruct-graph -m S -o 10 -i 120`` (ONNG).
* ``queries.npy`` -- 100 query rows (3 from data/sift-query-3.tsv + 97 seeded).
* ``search_<index>_<mode>_<eps>.npz`` -- reference search outputs (ids, 6-digit
  distances, distance-computation and visit counts) for ``ngt search -o e``.
* ``dist_<metric>_<otype>_d<D>.npz`` -- pairwise distances computed by the
  reference's comparators, harvested bit-exactly from the edge lists of small
  reference-built indexes (``grp`` stores each edge's float distance).
"""
import argparse
import os
import shutil
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ngt_files  # noqa: E402

EPSILONS = ["0.0", "0.02", "0.05", "0.1"]


def run(cmd, env, cwd, out=None):
    r = subprocess.run(cmd, env=env, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("%s failed:\n%s\n%s" % (cmd, r.stdout[-2000:], r.stderr[-2000:]))
    return r.stdout


def write_tsv(path, a, fmt):
    with open(path, "w") as f:
        for r in a:
            f.write("\t".join(fmt % v for v in r) + "\n")


def main():
    ap = argparse.ArgumentParser()
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap.add_argument("--ngt", default=os.path.join(root, "oracle", "_ref", "ngt"))
    ap.add_argument("--lib", default=os.path.join(root, "oracle", "_ref"))
    ap.add_argument("--subset", choices=["all", "quick"], default="all")
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--work", default="/tmp/ngt_goldens")
    args = ap.parse_args()

    env = dict(os.environ, LD_LIBRARY_PATH=args.lib)
    work = args.work
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    ngt = args.ngt

    # ---- data -------------------------------------------------------------
    sift = np.loadtxt(os.path.join(args.ref, "data/sift-dataset-5k.tsv"), delimiter="\t")[:, :128]
    q3 = np.loadtxt(os.path.join(args.ref, "data/sift-query-3.tsv"), delimiter="\t")[:, :128]
    rng = np.random.default_rng(0x4E4754)
    pick = rng.choice(sift.shape[0], 97, replace=False)
    noise = rng.integers(-12, 13, size=(97, 128))
    q97 = np.clip(sift[pick] + noise, 0, 255)
    queries = np.vstack([q3, q97]).astype(np.float32)
    np.save(os.path.join(args.out, "queries.npy"), queries.astype(np.uint8))
    np.save(os.path.join(args.out, "sift5k.npy"), sift.astype(np.uint8))
    write_tsv(os.path.join(work, "sift5k.tsv"), sift, "%d")
    write_tsv(os.path.join(work, "q100.tsv"), queries, "%d")

    quick = args.subset == "quick"
    # ---- C1: ANNG on sift-5k (BASELINE config 1) ---------------------------
    run([ngt, "create", "-d", "128", "-o", "f", "-D", "2", "c1_anng", "sift5k.tsv"], env, work)
    # ---- ONNG on sift-5k ---------------------------------------------------
    if not quick:
        run([ngt, "create", "-i", "t", "-g", "a", "-S", "0", "-e", "0.1", "-E", "100",
             "-d", "128", "-o", "f", "-D", "2", "anng100", "sift5k.tsv"], env, work)
        run([ngt, "reconstruct-graph", "-m", "S", "-o", "10", "-i", "120", "anng100", "c1_onng"], env, work)

    for name in (["c1_anng"] if quick else ["c1_anng", "c1_onng"]):
        dst = os.path.join(args.out, name)
        shutil.rmtree(dst, ignore_errors=True)
        shutil.copytree(os.path.join(work, name), dst)
        for mode in (["t"] if quick else ["t", "g", "s"]):
            for eps in (["0.1"] if quick else EPSILONS if mode != "s" else ["0.0"]):
                for om in (["r", "w"] if mode != "s" else ["r"]):
                    txt = run([ngt, "search", "-i", mode, "-n", "10", "-e", eps, "-m", om,
                               "-o", "e", name, "q100.tsv"], env, work)
                    res = ngt_files.parse_search_output(txt)
                    assert len(res) == queries.shape[0], (name, mode, eps, len(res))
                    ids = np.zeros((len(res), 10), np.int64) - 1
                    dists = np.full((len(res), 10), np.nan, np.float64)
                    for i, r in enumerate(res):
                        ids[i, :len(r["ids"])] = r["ids"]
                        dists[i, :len(r["dists"])] = r["dists"]
                    np.savez_compressed(
                        os.path.join(args.out, "search_%s_%s%s_%s.npz" % (name, mode, om, eps)),
                        ids=ids, dists=dists,
                        ndist=np.array([r["ndist"] for r in res]),
                        nvisit=np.array([r["nvisit"] for r in res]))
        if quick:
            continue
        # k=20 with a larger epsilon exercises a longer traversal.
        txt = run([ngt, "search", "-i", "t", "-n", "20", "-e", "0.2", "-o", "e", name, "q100.tsv"], env, work)
        res = ngt_files.parse_search_output(txt)
        ids = np.array([r["ids"] for r in res], dtype=np.int64)
        dists = np.array([r["dists"] for r in res], dtype=np.float64)
        np.savez_compressed(os.path.join(args.out, "search_%s_tr_k20_0.2.npz" % name),
                            ids=ids, dists=dists)

    # ---- per-metric pairwise distance goldens ------------------------------
    # (flag, name, object type, dims, source rows)
    sub = sift[:400]
    specs = [
        ("2", "l2", "f", 128), ("2", "l2", "f", 100), ("1", "l1", "f", 128), ("1", "l1", "f", 100),
        ("a", "angle", "f", 128), ("c", "cosine", "f", 100), ("A", "normalized_angle", "f", 128),
        ("C", "normalized_cosine", "f", 100), ("E", "normalized_l2", "f", 128),
        ("2", "l2", "c", 128), ("2", "l2", "c", 100), ("1", "l1", "c", 128),
        ("h", "hamming", "c", 128), ("h", "hamming", "c", 100), ("j", "jaccard", "c", 128),
        ("c", "cosine", "c", 128), ("a", "angle", "c", 100),
    ]
    if quick:
        specs = [("2", "l2", "f", 128), ("h", "hamming", "c", 128)]
    for flag, mname, ot, dim in specs:
        data = sub[:, :dim]
        if ot == "f":
            # non-integer floats exercise the rounding order of the reductions
            data = data * np.float32(0.37) + np.float32(0.013)
            fmt = "%.9g"
        else:
            fmt = "%d"
        tsv = os.path.join(work, "m_%s_%s_%d.tsv" % (mname, ot, dim))
        write_tsv(tsv, data, fmt)
        idx = "m_%s_%s_%d" % (mname, ot, dim)
        run([ngt, "create", "-d", str(dim), "-o", ot, "-D", flag, "-E", "12", idx, tsv], env, work)
        dtype = np.float32 if ot == "f" else np.uint8
        rows, valid = ngt_files.read_obj(os.path.join(work, idx, "obj"), dim, dtype)
        offs, ids, dists = ngt_files.read_grp(os.path.join(work, idx, "grp"))
        src = np.repeat(np.arange(len(offs) - 1, dtype=np.uint32), np.diff(offs).astype(np.int64))
        np.savez_compressed(os.path.join(args.out, "dist_%s_%s_d%d.npz" % (mname, ot, dim)),
                            rows=rows, src=src, dst=ids, dist=dists, dim=dim)
        print(mname, ot, dim, "pairs", len(ids))

    if quick:
        return
    # Poincare / Lorentz sets shipped with the reference (first 400 rows).
    for flag, mname, fn in [("p", "poincare", "poincare-input-5k.tsv"), ("l", "lorentz", "lorentz-input-5k.tsv")]:
        data = np.loadtxt(os.path.join(args.ref, "data", fn), delimiter="\t")[:400]
        dim = data.shape[1]
        tsv = os.path.join(work, "m_%s.tsv" % mname)
        write_tsv(tsv, data, "%.10f")
        idx = "m_%s" % mname
        run([ngt, "create", "-d", str(dim), "-o", "f", "-D", flag, "-E", "12", idx, tsv], env, work)
        rows, valid = ngt_files.read_obj(os.path.join(work, idx, "obj"), dim, np.float32)
        offs, ids, dists = ngt_files.read_grp(os.path.join(work, idx, "grp"))
        src = np.repeat(np.arange(len(offs) - 1, dtype=np.uint32), np.diff(offs).astype(np.int64))
        np.savez_compressed(os.path.join(args.out, "dist_%s_f_d%d.npz" % (mname, dim)),
                            rows=rows, src=src, dst=ids, dist=dists, dim=dim)
        print(mname, dim, "pairs", len(ids))


if __name__ == "__main__":
    main()
