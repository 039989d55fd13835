"""GPU parity of the NGTQ IVF-ADC path (ivf_kernels.hip + the global-codebook
search kernels, through ngt_amd_ngtq_open / ngt_amd_ngtq_search) against the
reference's own outputs (tests/golden/ngtq_n*, made by make_ngtq_goldens.py
from the reference library) and against the CPU restatement (oracle/).

Bar: identical ids and float distance bits for every aggregation mode the
fixtures hold; the cached-distance modes at 4-float subvectors are refused
(the reference reads past the subvector there)."""
import os
import shutil

import numpy as np
import pytest

import ngt_files as F
import oracle_py as O
from ngt_amd import NativeError
from ngt_amd.ngtq import Index

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["ngtq_n8", "ngtq_n16", "ngtq_n32"]


def objects():
    rows, _ = F.read_obj(os.path.join(GOLD, "c1_anng", "obj"), 128, np.float32)
    return rows[:, :128]


def open_index(name, tmp_path):
    """The committed fixture plus its object list (the SIFT-5k rows of
    c1_anng, written as the reference's ArrayFile 'obj')."""
    d = os.path.join(str(tmp_path), name)
    shutil.copytree(os.path.join(GOLD, name), d)
    F.write_array_file(os.path.join(d, "obj"), objects())
    return Index(d)


def specs(z):
    for key in sorted(k for k in z if k.startswith("ids_")):
        s = key[4:]
        m, size, exp, eps = s.split("_")
        eps = float(eps.replace("p", ".").replace("m", "-"))
        yield s, m, int(size), float(exp), (None if eps < 0 else eps)


@pytest.mark.parametrize("name", NAMES)
def test_ngtq_search_matches_reference(name, tmp_path):
    z = dict(np.load(os.path.join(GOLD, name, "goldens.npz")))
    ix = open_index(name, tmp_path)
    dsub = 128 // int(name.split("_n")[1])
    checked = 0
    for s, m, size, exp, eps in specs(z):
        if dsub % 8 and m in "cr":
            with pytest.raises(NativeError):
                ix.search(z["queries"][:1], size=size, expansion=exp, mode=m, epsilon=eps)
            continue
        ids, ds, n = ix.search(z["queries"], size=size, expansion=exp, mode=m, epsilon=eps)
        assert np.array_equal(n, z["n_" + s]), (name, s)
        for qi in range(len(z["queries"])):
            k = int(n[qi])
            assert list(ids[qi, :k]) == list(z["ids_" + s][qi, :k]), (name, s, qi)
            assert np.array_equal(ds[qi, :k].view(np.uint32), z["d_" + s][qi, :k].view(np.uint32)), (name, s, qi)
        checked += 1
    assert checked >= 9
    ix.close()


@pytest.mark.parametrize("mode", ["a", "c", "l", "e", "r"])
def test_ngtq_search_matches_oracle_wide(mode, tmp_path):
    """Settings outside the fixtures (larger size and expansion, several global
    lists per query, epsilon 0 and 0.3) against the restatement."""
    name = "ngtq_n16"
    st = O.load_ngtq(os.path.join(GOLD, name), objects())
    ix = open_index(name, tmp_path)
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)[40:70, :128]
    for size, exp, eps in [(50, 30.0, 0.3), (7, 3.5, 0.0), (100, 12.0, None)]:
        ids, ds, n = ix.search(qs, size=size, expansion=exp, mode=mode, epsilon=eps)
        for qi, q in enumerate(qs):
            oi, od = O.ngtq_search(st, q, mode, size, exp, eps)
            assert int(n[qi]) == len(oi), (mode, size, qi)
            assert list(ids[qi, :n[qi]]) == list(oi), (mode, size, qi)
            assert np.array_equal(ds[qi, :n[qi]].view(np.uint32), od.view(np.uint32)), (mode, size, qi)
    ix.close()
