#!/usr/bin/env python3
"""Generate the committed NGTQ (IVF-ADC) golden fixtures from the reference
NGT 1.13.8.  Development container only (never on the GPU box):

    make -f oracle/ref.mk                  # the reference, built from its sources
    python3 tests/golden/make_ngtq_goldens.py

1. ``ngtq create -d 128 -C 64 -c 16 -N <n> -L k`` over data/sift-dataset-5k.tsv
   for N = 8, 16, 32 local divisions (dsub 16, 8, 4): a global codebook of up
   to 64 centroids, 16 k-means local centroids per subspace, the inverted
   lists and the object list.
2. ``ngtq_harness.cpp`` (oracle/ref.mk) runs NGTQ::Index::search for every
   aggregation mode (a, c, l, e, r) and a few (size, expansion, epsilon)
   settings, epsilon < 0 meaning the linear global-codebook search (``-e -``),
   and records ids and float distances, plus the float LUT of
   createDistanceLookup for global centroids 1..3.
3. ``ngtq search`` (the CLI) cross-checks one setting (6-digit distances).

Committed per index: ``ngtq_n<N>/`` = prf, global/{prf,obj,grp,tre},
local-*/obj, ivt (the object list ``obj`` is NOT committed: it holds the same
SIFT-5k rows as c1_anng/obj, ids 1..5000 in file order -- checked here --
and the tests rebuild it), and ``goldens.npz``.
"""
import os
import shutil
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import ngt_files as F  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref")
DATA = "/root/reference/data/sift-dataset-5k.tsv"
SPECS = ["%s:10:4:0.1" % m for m in "aclre"] + ["%s:20:8:0.05" % m for m in "aclre"] + \
        ["%s:10:16:-1" % m for m in "acl"] + ["l:5:2:0.2", "c:1:1:0.0"]
NQ = 40


def run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("%s failed:\n%s\n%s" % (cmd, r.stdout[-2000:], r.stderr[-2000:]))
    return r.stdout


def main():
    work = "/tmp/ngtq_goldens"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    rows = np.loadtxt(DATA, dtype=np.float32, delimiter="\t")[:, :128]
    np.savetxt(os.path.join(work, "data.tsv"), rows, delimiter="\t", fmt="%.9g")
    c1, _ = F.read_obj(os.path.join(HERE, "c1_anng", "obj"), 128, np.float32)
    assert np.array_equal(c1[1:, :128], rows), "c1_anng rows differ from the SIFT-5k file"
    qs = np.load(os.path.join(HERE, "queries.npy")).astype(np.float32)[:NQ, :128]
    qf = os.path.join(work, "q.f32")
    qs.tofile(qf)
    for n in (8, 16, 32):
        name = "ngtq_n%d" % n
        idx = os.path.join(work, name)
        run([os.path.join(REF, "ngtq"), "create", "-d", "128", "-C", "64", "-c", "16", "-N", str(n), "-L", "k",
             "-p", "8", idx, os.path.join(work, "data.tsv")])
        ol = F.read_array_file(os.path.join(idx, "obj"), 128)
        assert np.array_equal(ol[1:], rows), "object list differs from the data"
        out = os.path.join(work, name + "_out")
        os.makedirs(out)
        run([os.path.join(REF, "ngtq_harness"), idx, qf, str(NQ), "128", out] + SPECS)
        g = {"queries": qs}
        g["flut"] = np.fromfile(os.path.join(out, "flut.bin"), np.float32).reshape(NQ, 3, -1)
        for s in SPECS:
            size = int(s.split(":")[1])
            raw = np.fromfile(os.path.join(out, "search_%s.bin" % s), np.uint8).reshape(NQ, 4 + 8 * size)
            key = s.replace(":", "_").replace(".", "p").replace("-", "m")
            g["n_" + key] = raw[:, :4].copy().view(np.uint32)[:, 0]
            body = raw[:, 4:].copy().view(np.uint32).reshape(NQ, size, 2)
            g["ids_" + key] = body[:, :, 0].copy()
            g["d_" + key] = body[:, :, 1].copy().view(np.float32)
        # CLI cross-check of one setting (ngtq search prints 6 significant digits)
        np.savetxt(os.path.join(work, "q.tsv"), qs[:5], delimiter="\t", fmt="%.9g")
        cli = run([os.path.join(REF, "ngtq"), "search", "-n", "10", "-m", "l", "-e", "0.1", "-b", "4", idx,
                   os.path.join(work, "q.tsv")])
        got = [ln.split("\t") for ln in cli.splitlines() if ln[:1].isdigit() and ln.count("\t") == 2]
        key = "l_10_4_0p1"
        exp = [(str(int(g["ids_" + key][qi, r])), "%.6g" % g["d_" + key][qi, r]) for qi in range(5)
               for r in range(int(g["n_" + key][qi]))]
        assert [(a[1], a[2]) for a in got] == exp, "harness and CLI disagree"
        dst = os.path.join(HERE, name)
        shutil.rmtree(dst, ignore_errors=True)
        os.makedirs(dst)
        shutil.copy(os.path.join(idx, "prf"), dst)
        shutil.copy(os.path.join(idx, "ivt"), dst)
        shutil.copytree(os.path.join(idx, "global"), os.path.join(dst, "global"))
        for i in range(n):
            os.makedirs(os.path.join(dst, "local-%d" % i))
            for f in ("prf", "obj"):
                shutil.copy(os.path.join(idx, "local-%d" % i, f), os.path.join(dst, "local-%d" % i))
        np.savez_compressed(os.path.join(dst, "goldens.npz"), **g)
        print(name, "ok")


if __name__ == "__main__":
    main()
