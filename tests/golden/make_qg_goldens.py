#!/usr/bin/env python3
"""Generate the committed NGTQG golden fixtures from the reference NGT 1.13.8.

Development container only (never on the GPU box):

    make -f oracle/ref.mk                      # the reference, built from its sources
    python3 tests/golden/make_qg_goldens.py

Steps (all reference binaries come from oracle/_ref/, built from
/root/reference by the committed recipe oracle/ref.mk):

1. ``ngtqg quantize -E 128`` on a copy of ``c1_onng`` (ONNG over SIFT-5k,
   dsub=1 => M=128 subspaces), and on a small synthetic ANNG with D=20 and
   ``-Q 4`` (dsub=4 => M=5: odd subspace count + multi-element subvectors).
2. ``qg_harness.cpp`` (compiled by oracle/ref.mk with the reference's own flags
   and linked against oracle/_ref/libngt_ref.so) records per query the uint8 LUT / scale / totalOffset, ADC
   distances over a few nodes' packed code blocks, and NGTQG::Index::search
   results for several (k, epsilon, result_expansion) triples.
3. ``ngtqg search`` on the same queries cross-checks the harness's search path
   against the CLI's (identical ids and 6-digit distances).

Committed: ``<name>_qg/`` (qg/prf, qg/global/obj, qg/local-*/obj, qg/ivt -- the
quantizer state; qg/grp is *rebuilt* by our loader and checked against the
reference's sha256 in ``meta.json``), ``<name>_qg/goldens.npz``.
"""
import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ngt_files  # noqa: E402

PARAMS = ["10:0.0:1", "10:0.02:3", "10:0.05:3", "10:0.1:2", "20:0.03:3", "10:0.05:0.5", "5:0.08:1.5"]


def run(cmd, env, cwd=None):
    r = subprocess.run(cmd, env=env, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("%s failed:\n%s\n%s" % (cmd, r.stdout[-2000:], r.stderr[-2000:]))
    return r.stdout


def write_tsv(path, a, fmt):
    with open(path, "w") as f:
        for r in a:
            f.write("\t".join(fmt % v for v in r) + "\n")


def harness(args, env, index, queries, nodes, outdir):
    qf = os.path.join(outdir, "q.f32")
    queries.astype(np.float32).tofile(qf)
    nf = os.path.join(outdir, "nodes.u32")
    np.asarray(nodes, np.uint32).tofile(nf)
    run([args.harness_bin, index, qf, str(len(queries)), str(queries.shape[1]), outdir, nf] + PARAMS, env)


def collect(index, outdir, queries, nodes, M):
    me = ((M - 1) // 2 + 1) * 2
    nq = len(queries)
    g = {"queries": queries.astype(np.float32), "nodes": np.asarray(nodes, np.uint32)}
    g["lut"] = np.fromfile(os.path.join(outdir, "lut.bin"), np.uint8).reshape(nq, me * 16)
    sc = np.fromfile(os.path.join(outdir, "scale.bin"), np.float32).reshape(nq, 2)
    g["scale"], g["total_offset"] = sc[:, 0].copy(), sc[:, 1].copy()
    g["adc"] = np.fromfile(os.path.join(outdir, "adc.bin"), np.float32).reshape(nq, -1)
    for p in PARAMS:
        raw = np.fromfile(os.path.join(outdir, "search_%s.bin" % p), np.uint8)
        k = int(p.split(":")[0])
        rec = raw.reshape(nq, 4 + 8 * k)
        n = rec[:, :4].copy().view(np.uint32)[:, 0]
        body = rec[:, 4:].copy().view(np.uint32).reshape(nq, k, 2)
        key = p.replace(":", "_")
        g["n_" + key] = n
        g["ids_" + key] = body[:, :, 0].copy()
        g["dist_" + key] = body[:, :, 1].copy().view(np.float32)
    return g


def cli_crosscheck(args, env, index, queries, g, work):
    """ngtqg search -n 10 -e 0.05 -p 3 on the first queries == harness results."""
    qt = os.path.join(work, "q_cli.tsv")
    write_tsv(qt, queries[:8], "%.9g")
    out = run([args.ngtqg, "search", "-n", "10", "-e", "0.05", "-p", "3", "-o", "e", index, qt], env)
    res = ngt_files.parse_search_output(out)
    assert len(res) == 8
    for qi, r in enumerate(res):
        ids = r["ids"]
        assert ids == list(g["ids_10_0.05_3"][qi][: len(ids)]), (qi, ids, g["ids_10_0.05_3"][qi])
        for d, dg in zip(r["dists"], g["dist_10_0.05_3"][qi]):
            assert d == float("%g" % dg), (qi, d, dg)


def keep_state(index, dst):
    """Copy the quantizer state (not qg/grp, not qg/obj) into the fixture dir."""
    shutil.rmtree(dst, ignore_errors=True)
    os.makedirs(os.path.join(dst, "qg", "global"))
    src = os.path.join(index, "qg")
    for f in ("prf", "ivt"):
        shutil.copy(os.path.join(src, f), os.path.join(dst, "qg", f))
    for f in ("obj", "prf"):
        shutil.copy(os.path.join(src, "global", f), os.path.join(dst, "qg", "global", f))
    li = 0
    while os.path.isdir(os.path.join(src, "local-%d" % li)):
        os.makedirs(os.path.join(dst, "qg", "local-%d" % li))
        shutil.copy(os.path.join(src, "local-%d" % li, "obj"), os.path.join(dst, "qg", "local-%d" % li, "obj"))
        li += 1
    grp = open(os.path.join(src, "grp"), "rb").read()
    return {"grp_sha256": hashlib.sha256(grp).hexdigest(), "grp_size": len(grp), "local_codebooks": li}


def main():
    ap = argparse.ArgumentParser()
    ref_out = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "_ref")
    ap.add_argument("--ngt", default=os.path.join(ref_out, "ngt"))
    ap.add_argument("--ngtqg", default=os.path.join(ref_out, "ngtqg"))
    ap.add_argument("--lib", default=ref_out)
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--work", default="/tmp/ngt_qg_goldens")
    ap.add_argument("--harness-bin", default=os.path.join(ref_out, "qg_harness"))
    args = ap.parse_args()
    env = dict(os.environ, LD_LIBRARY_PATH=args.lib)
    work = args.work
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    if not os.path.exists(args.harness_bin):
        raise SystemExit("build the reference and harnesses first: make -f oracle/ref.mk")

    # ---- C1 ONNG, dsub=1 (M=128) -------------------------------------------
    idx = os.path.join(work, "c1")
    shutil.copytree(os.path.join(HERE, "c1_onng"), idx)
    run([args.ngtqg, "quantize", "-E", "128", idx], env)
    queries = np.load(os.path.join(HERE, "queries.npy")).astype(np.float32)
    nodes = [1, 2, 3, 17, 100, 1000, 2500, 4999, 5000]
    od = os.path.join(work, "c1_out")
    os.makedirs(od)
    harness(args, env, idx, queries, nodes, od)
    g = collect(idx, od, queries, nodes, 128)
    cli_crosscheck(args, env, idx, queries, g, work)
    dst = os.path.join(HERE, "c1_qg")
    meta = keep_state(idx, dst)
    meta.update({"source": "c1_onng", "quantize": "ngtqg quantize -E 128", "params": PARAMS})
    np.savez_compressed(os.path.join(dst, "goldens.npz"), **g)
    json.dump(meta, open(os.path.join(dst, "meta.json"), "w"), indent=1)

    # ---- synthetic D=20, -Q 4 (M=5, odd) ------------------------------------
    rng = np.random.default_rng(0x51475)
    base = np.round(rng.random((2000, 20)) * 100.0, 2).astype(np.float32)
    qs = np.round(rng.random((40, 20)) * 100.0, 2).astype(np.float32)
    write_tsv(os.path.join(work, "d20.tsv"), base, "%.2f")
    d20 = os.path.join(work, "d20")
    run([args.ngt, "create", "-i", "t", "-g", "a", "-S", "0", "-e", "0.1", "-E", "40", "-d", "20", "-o", "f", "-D", "2",
         d20, os.path.join(work, "d20.tsv")], env)
    run([args.ngtqg, "quantize", "-Q", "4", "-E", "64", d20], env)
    od = os.path.join(work, "d20_out")
    os.makedirs(od)
    nodes = [1, 2, 5, 700, 2000]
    harness(args, env, d20, qs, nodes, od)
    g = collect(d20, od, qs, nodes, 5)
    dst = os.path.join(HERE, "d20_qg")
    meta = keep_state(d20, dst)
    for f in ("prf", "obj", "grp", "tre"):
        shutil.copy(os.path.join(d20, f), os.path.join(dst, f))
    meta.update({"source": "synthetic 2000x20 (seed 0x51475)", "quantize": "ngtqg quantize -Q 4 -E 64",
                 "params": PARAMS})
    np.savez_compressed(os.path.join(dst, "goldens.npz"), **g)
    json.dump(meta, open(os.path.join(dst, "meta.json"), "w"), indent=1)
    print("ok")


if __name__ == "__main__":
    main()
