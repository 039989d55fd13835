"""Pins the oracle's comparators and normalization against fixtures produced by
the reference's own code (tests/golden/make_comparator_goldens.py, running
tests/golden/comparator_harness.cpp compiled by oracle/ref.mk), and checks that
the committed fixtures regenerate from /root/reference (when it is present:
this container, never the GPU box).  CPU only.
"""
import ctypes
import glob
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import oracle_py as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
ROOT = os.path.dirname(HERE)
REF = "/root/reference"


def _pair_cases():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLD, "pair_*.npz"))):
        name = os.path.basename(f)[5:-4]
        metric, ot = name.rsplit("_", 2)[0], name.rsplit("_", 2)[1]
        out.append(pytest.param(f, metric, ot, id=name))
    return out


def oracle_pairs(metric, a, b):
    L = O.lib()
    ot = 2 if a.dtype == np.float32 else 1
    out = np.empty(a.shape[0], np.float32)
    for i in range(a.shape[0]):
        out[i] = L.ngto_distance(O.METRICS[metric], ot, a[i].ctypes.data, b[i].ctypes.data, a.shape[1])
    return out


@pytest.mark.parametrize("path,metric,ot", _pair_cases())
def test_oracle_pairs_bit_exact(path, metric, ot):
    """compareSparseJaccardDistance (PrimitiveComparator.h:399-418) incl. empty and
    full lists, and the uint8 dot-product family (:479-485, :226-234, :583-593, :644-648)."""
    z = np.load(path)
    a, b = np.ascontiguousarray(z["a"]), np.ascontiguousarray(z["b"])
    got = oracle_pairs(metric, a, b)
    assert np.array_equal(got.view(np.uint32), z["dist"].view(np.uint32))


@pytest.mark.parametrize("dim", [20, 100, 128, 960])
def test_oracle_normalize_within_2ulp(dim):
    """ObjectSpace::normalize (ObjectSpace.h:251-266): the sum order is the
    reference's; its -Ofast reciprocal square root is host-CPU dependent, so the
    stored vectors agree within 2 ulp (the tolerance the normalized-metric
    tests use)."""
    z = np.load(os.path.join(GOLD, "norm_f_d%d.npz" % dim))
    x, y = z["x"], z["y"]
    L = O.lib()
    for i in range(x.shape[0]):
        v = np.ascontiguousarray(x[i].copy())
        assert L.ngto_normalize_f32(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), dim) == 0
        ulp = np.spacing(np.abs(y[i])).astype(np.float32)
        assert np.all(np.abs(v - y[i]) <= 2 * ulp), (i, np.max(np.abs(v - y[i]) / ulp))


def _ref_ready():
    return os.path.isdir(REF) and shutil.which("cmake") and shutil.which("g++")


@pytest.mark.skipif(not _ref_ready(), reason="needs /root/reference (development container only)")
def test_fixtures_regenerate_from_reference(tmp_path):
    """oracle/ref.mk builds the reference from its sources; make_goldens.py
    --subset quick re-runs it and the C1 ANNG index files, its tree-seeded
    searches at epsilon 0.1 and two comparator fixtures equal the committed ones."""
    subprocess.check_call(["make", "-s", "-j8", "-f", "oracle/ref.mk"], cwd=ROOT, stdout=subprocess.DEVNULL)
    out = tmp_path / "gold"
    out.mkdir()
    subprocess.check_call([sys.executable, os.path.join(GOLD, "make_goldens.py"), "--subset", "quick",
                           "--out", str(out), "--work", str(tmp_path / "work")], cwd=ROOT,
                          stdout=subprocess.DEVNULL)
    for f in ("prf", "obj", "grp", "tre"):
        a = open(os.path.join(GOLD, "c1_anng", f), "rb").read()
        b = open(str(out / "c1_anng" / f), "rb").read()
        assert a == b, f
    for name in ("search_c1_anng_tr_0.1.npz", "search_c1_anng_tw_0.1.npz", "dist_l2_f_d128.npz",
                 "dist_hamming_c_d128.npz", "queries.npy", "sift5k.npy"):
        if name.endswith(".npy"):
            assert np.array_equal(np.load(os.path.join(GOLD, name)), np.load(str(out / name)))
            continue
        za, zb = np.load(os.path.join(GOLD, name)), np.load(str(out / name))
        assert sorted(za.files) == sorted(zb.files)
        for k in za.files:
            x, y = za[k], zb[k]
            assert x.dtype == y.dtype and x.shape == y.shape, (name, k)
            assert x.tobytes() == y.tobytes(), (name, k)


@pytest.mark.skipif(not _ref_ready(), reason="needs /root/reference (development container only)")
def test_batch_fixtures_regenerate_from_reference(tmp_path):
    """make_batch_goldens.py re-runs the reference CLI (`ngt create -b 1000 /
    5000`) and its grp/tre equal the committed c1_anng_b* fixtures."""
    subprocess.check_call(["make", "-s", "-j8", "-f", "oracle/ref.mk"], cwd=ROOT, stdout=subprocess.DEVNULL)
    out = tmp_path / "gold"
    out.mkdir()
    import shutil
    shutil.copy(os.path.join(GOLD, "sift5k.npy"), str(out / "sift5k.npy"))
    subprocess.check_call([sys.executable, os.path.join(GOLD, "make_batch_goldens.py"), "--out", str(out),
                           "--work", str(tmp_path / "work")], cwd=ROOT, stdout=subprocess.DEVNULL)
    for b in (1000, 5000):
        for f in ("prf", "grp", "tre"):
            a = open(os.path.join(GOLD, "c1_anng_b%d" % b, f), "rb").read()
            assert a == open(str(out / ("c1_anng_b%d" % b) / f), "rb").read(), (b, f)
    # a different batch size gives a different graph (the fixtures pin -b)
    assert open(os.path.join(GOLD, "c1_anng_b1000", "grp"), "rb").read() != \
        open(os.path.join(GOLD, "c1_anng", "grp"), "rb").read()


@pytest.mark.parametrize("isa", ["v3", "v4"])
def test_native_builds_agree(isa):
    """The vectorized OpenMP builds bench.py times as the CPU baseline
    (oracle/libngt_oracle_v{3,4}.so) give the checker's bits: tree-seeded
    searches on the reference-built C1 ONNG and linear search, 4 threads."""
    if isa == "v4" and O.host_isa() != "v4":
        pytest.skip("host has no AVX-512")
    import ngt_files as F
    d = os.path.join(GOLD, "c1_onng")
    rows, _ = F.read_obj(os.path.join(d, "obj"), 128, np.float32)
    offs, ids, _ = F.read_grp(os.path.join(d, "grp"))
    tree = F.read_tre(os.path.join(d, "tre"), 128, np.float32)
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    seeds = [O.tree_seeds("l2", tree, q, 10, 10)[0] for q in qs]
    L = O.native_lib(isa)
    bi, bd, bn, bc = O.search_batch("l2", rows, offs, ids, qs, seeds, 10, np.float32(0.05), edge_size=40,
                                    threads=4, L=L)
    for i, q in enumerate(qs):
        oid, od, ocnt = O.search("l2", rows, offs, ids, q, seeds[i], 10, np.float32(0.05), edge_size=40)
        assert list(bi[i, :bn[i]]) == list(oid)
        assert np.array_equal(bd[i, :bn[i]].view(np.uint32), od.view(np.uint32))
        assert int(bc[i, 0]) == int(ocnt[0])
    li, ld, ln = O.linear_search_batch("l2", rows, qs[:20], 10, threads=4, L=L)
    for i in range(20):
        oid, od = O.linear_search("l2", rows, qs[i], 10)
        assert list(li[i, :ln[i]]) == list(oid)
        assert np.array_equal(ld[i, :ln[i]].view(np.uint32), od.view(np.uint32))
