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


def test_expected_accuracy_mapping_matches_reference():
    """ngtpy.search(expected_accuracy=a) searches at the epsilon the prf's
    AccuracyTable gives (Index::AccuracyTable::getEpsilon, Index.h:317-346):
    equal float bits to the reference's own function on the C1 ONNG's table
    for 209 accuracies (grid, table points and their neighbours, > 1 and
    below the first entry), tests/golden/accuracy_c1_onng.json."""
    import json
    table = ngtpy.accuracy_table(os.path.join(GOLD, "c1_onng"))
    assert len(table) == 31
    pairs = json.load(open(os.path.join(GOLD, "accuracy_c1_onng.json")))["pairs"]
    for ab, eb in pairs:
        a = float(np.array([ab], np.uint32).view(np.float32)[0])
        e = np.float32(ngtpy.epsilon_from_expected_accuracy(table, a))
        assert int(e.view(np.uint32)) == eb, a
    with pytest.raises(Exception, match="accuracy table is not set yet"):
        ngtpy.epsilon_from_expected_accuracy(table[:2], 0.9)


def test_expected_accuracy_without_table(tmp_path):
    """An index whose prf has no AccuracyTable (every `ngt create` index)
    raises the reference's error, as NGT::Index::search does."""
    import shutil
    d = tmp_path / "noacc"
    shutil.copytree(os.path.join(GOLD, "c1_anng"), str(d))
    assert ngtpy.accuracy_table(str(d)) == []
    with pytest.raises(Exception, match="table size=0"):
        ngtpy.epsilon_from_expected_accuracy(ngtpy.accuracy_table(str(d)), 0.9)


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs /root/reference (development container only)")
def test_accuracy_fixture_regenerates_from_reference(tmp_path):
    import json
    import subprocess
    import sys
    subprocess.check_call(["make", "-s", "-j8", "-f", "oracle/ref.mk"], cwd=ROOT, stdout=subprocess.DEVNULL)
    subprocess.check_call([sys.executable, os.path.join(GOLD, "make_accuracy_goldens.py"), "--out", str(tmp_path)])
    assert json.load(open(str(tmp_path / "accuracy_c1_onng.json"))) == json.load(
        open(os.path.join(GOLD, "accuracy_c1_onng.json")))


@pytest.mark.gpu
def test_ngtpy_expected_accuracy_search():
    """search(expected_accuracy=a) == search(epsilon=<the table's epsilon>);
    set(expected_accuracy=...) is kept like defaultExpectedAccuracy and, as in
    the reference (ngtpy.cpp:168-172, 333), changes no search."""
    ix = ngtpy.Index(os.path.join(GOLD, "c1_onng"), read_only=True)
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    for acc in (0.8, 0.9, 0.95):
        eps = ix.epsilon_for(acc)
        for i in range(0, len(qs), 11):
            a = ix.search(qs[i], size=10, epsilon=0.3, expected_accuracy=acc)
            b = ix.search(qs[i], size=10, epsilon=eps)
            assert [x[0] for x in a] == [x[0] for x in b], (acc, i)
            assert [np.float32(x[1]).view(np.uint32) for x in a] == [np.float32(x[1]).view(np.uint32) for x in b]
    ix.set(expected_accuracy=0.5)
    assert ix.expected_accuracy == 0.5
    assert ix.search(qs[0], size=10) == ix.search(qs[0], size=10, epsilon=0.1)
    ix.close()
