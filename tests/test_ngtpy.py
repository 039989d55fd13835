"""ngtpy-compatible surface (ngt_amd/ngtpy.py): names and defaults on CPU
(python/src/ngtpy.cpp:505-560), results against the reference's own search
outputs on the C1 ONNG on the GPU."""
import inspect
import os

import numpy as np
import pytest

from ngt_amd import ngtpy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def defaults(fn):
    return {k: v.default for k, v in inspect.signature(fn).parameters.items() if k != "self"}


def test_ngtpy_names_and_defaults():
    assert defaults(ngtpy.create) == {"path": inspect._empty, "dimension": inspect._empty,
                                      "edge_size_for_creation": 10, "edge_size_for_search": 40,
                                      "distance_type": "L2", "object_type": "Float"}
    assert defaults(ngtpy.Index.__init__) == {"path": inspect._empty, "read_only": False,
                                              "zero_based_numbering": True, "tree_disabled": False,
                                              "log_disabled": False}
    s = defaults(ngtpy.Index.search)
    assert s["size"] == 0 and s["epsilon"] == -ngtpy.FLT_MAX and s["edge_size"] == -2 ** 31
    assert s["with_distance"] is True
    assert defaults(ngtpy.Index.linear_search) == {"query": inspect._empty, "size": 0, "with_distance": True}
    assert defaults(ngtpy.Index.batch_insert)["num_threads"] == 8
    for m in ("get_num_of_distance_computations", "save", "close", "remove", "build_index", "get_object",
              "insert", "set"):
        assert callable(getattr(ngtpy.Index, m))


def test_ngtpy_create_rejects_bad_types():
    with pytest.raises(Exception, match="invalid object type"):
        ngtpy.create("/tmp/unused", 4, object_type="Double")
    with pytest.raises(Exception, match="invalid distance type"):
        ngtpy.create("/tmp/unused", 4, distance_type="L3")


@pytest.mark.gpu
@pytest.mark.parametrize("eps", ["0.0", "0.05", "0.1"])
def test_ngtpy_search_matches_reference(eps):
    ix = ngtpy.Index(os.path.join(GOLD, "c1_onng"), read_only=True)
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    g = np.load(os.path.join(GOLD, "search_c1_onng_tr_%s.npz" % eps))
    for i in range(0, len(qs), 7):
        ref = g["ids"][i][g["ids"][i] >= 0][:10]
        res = ix.search(qs[i], size=10, epsilon=float(eps))
        assert [r[0] for r in res] == [int(x) - 1 for x in ref], i
        assert ["%g" % r[1] for r in res] == ["%g" % float(x) for x in g["dists"][i][:len(res)]], i
        assert list(ix.search(qs[i], size=10, epsilon=float(eps), with_distance=False)) == [r[0] for r in res]
    assert ix.get_num_of_distance_computations() > 0
    ix.close()


@pytest.mark.gpu
def test_ngtpy_linear_search_and_one_based_ids():
    ix0 = ngtpy.Index(os.path.join(GOLD, "c1_onng"), read_only=True)
    ix1 = ngtpy.Index(os.path.join(GOLD, "c1_onng"), read_only=True, zero_based_numbering=False)
    q = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)[3]
    a = ix0.linear_search(q, size=5)
    b = ix1.linear_search(q, size=5)
    assert [x[0] + 1 for x in a] == [x[0] for x in b]
    assert a[0][1] <= a[-1][1]
    assert ix0.get_object(a[0][0]) == ix1.get_object(b[0][0])
    ix0.close()
    ix1.close()
