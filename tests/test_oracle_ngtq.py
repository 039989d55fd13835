"""The NGTQ IVF-ADC restatement (oracle/ngt_oracle.c ngto_ngtq_*) against the
reference's own outputs: tests/golden/ngtq_n{8,16,32} hold indexes built by
the reference's ``ngtq create`` over SIFT-5k (64 global centroids, 16 local
centroids per subspace, N = 8/16/32 subspaces) and NGTQ::Index::search results
for every aggregation mode (make_ngtq_goldens.py, ngtq_harness.cpp).

Bar: identical ids and float distance bits (the float-LUT entries too).  The
cached-distance modes ('c', 'r') are not pinned at N = 32: with 4-float
subvectors the reference's 8-float AVX loop reads past the subvector."""
import os

import numpy as np
import pytest

import ngt_files as F
import oracle_py as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["ngtq_n8", "ngtq_n16", "ngtq_n32"]
_CACHE = {}


def objects():
    rows, _ = F.read_obj(os.path.join(GOLD, "c1_anng", "obj"), 128, np.float32)
    return rows[:, :128]  # record 0 is the unused slot, ids 1..5000 = SIFT-5k in file order


def state(name):
    if name not in _CACHE:
        d = os.path.join(GOLD, name)
        _CACHE[name] = (O.load_ngtq(d, objects()), dict(np.load(os.path.join(d, "goldens.npz"))))
    return _CACHE[name]


def specs(z):
    for key in sorted(k for k in z if k.startswith("ids_")):
        s = key[4:]
        m, size, exp, eps = s.split("_")
        eps = float(eps.replace("p", ".").replace("m", "-"))
        yield s, m, int(size), float(exp), (None if eps < 0 else eps)


@pytest.mark.parametrize("name", NAMES)
def test_ngtq_float_lut_bit_exact(name):
    st, z = state(name)
    N, dsub = st["N"], st["dsub"]
    for qi in range(8):
        q = z["queries"][qi]
        for gi in range(3):
            ref = z["flut"][qi, gi].reshape(N, 17)[:, 1:]
            g = st["G"][gi + 1]
            got = np.array([[O.ngtq_term("l", q[li * dsub:(li + 1) * dsub], g[li * dsub:(li + 1) * dsub],
                                         st["local"][li, k]) for k in range(1, 17)] for li in range(N)], np.float32)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (name, qi, gi)


@pytest.mark.parametrize("name", NAMES)
def test_ngtq_search_matches_reference(name):
    st, z = state(name)
    checked = 0
    for s, m, size, exp, eps in specs(z):
        if st["dsub"] % 8 and m in "cr":
            continue
        for qi in range(len(z["queries"])):
            ids, ds = O.ngtq_search(st, z["queries"][qi], m, size, exp, eps)
            n = int(z["n_" + s][qi])
            assert list(ids) == list(z["ids_" + s][qi, :n]), (name, s, qi)
            assert np.array_equal(ds.view(np.uint32), z["d_" + s][qi, :n].view(np.uint32)), (name, s, qi)
            checked += 1
    assert checked >= 9 * 40
