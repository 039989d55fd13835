"""ANNG construction on the GPU (build_kernels.hip + build.cpp) against the
reference: `ngt create -d 128 -o f -D 2` of data/sift-dataset-5k.tsv
(tests/golden/c1_anng, made by the reference CLI) must come out identical --
every edge list (ids and float distances, in order) and the DVP tree (node
ids, parents, leaf contents, pivots, borders), i.e. byte-identical grp/tre
files after ngt_save_index."""
import filecmp
import os

import numpy as np
import pytest

import ngt_files as F
from ngt_amd import base
from ngt_amd.device import DeviceIndex

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _first_diff(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return "shape %s vs %s" % (a.shape, b.shape)
    bad = np.flatnonzero(a.reshape(-1) != b.reshape(-1))
    return None if len(bad) == 0 else "first difference at flat index %d: %r vs %r" % (
        bad[0], a.reshape(-1)[bad[0]], b.reshape(-1)[bad[0]])


def test_device_anng_matches_reference_graph_and_tree():
    rows, valid = F.read_obj(os.path.join(GOLD, "c1_anng", "obj"), 128, np.float32)
    ix = DeviceIndex("l2", "float", 128)
    ix.set_objects(rows, valid)
    (offs, ids, ds), tree = ix.build_anng()
    goffs, gids, gds = F.read_grp(os.path.join(GOLD, "c1_anng", "grp"))
    n = min(len(offs), len(goffs)) - 1
    for v in range(1, n):
        a, b = int(offs[v]), int(offs[v + 1])
        c, d = int(goffs[v]), int(goffs[v + 1])
        assert list(ids[a:b]) == list(gids[c:d]), ("node", v, list(ids[a:b]), list(gids[c:d]))
        assert np.array_equal(ds[a:b].view(np.uint32), gds[c:d].view(np.uint32)), ("node", v)
    assert len(offs) == len(goffs)
    gt = F.read_tre(os.path.join(GOLD, "c1_anng", "tre"), 128, np.float32)
    nl = len(gt["leaf_off"]) - 1
    assert len(tree["leaf_off"]) - 1 == nl
    assert _first_diff(tree["leaf_off"], gt["leaf_off"]) is None, _first_diff(tree["leaf_off"], gt["leaf_off"])
    assert _first_diff(tree["leaf_ids"], gt["leaf_ids"]) is None, _first_diff(tree["leaf_ids"], gt["leaf_ids"])
    ni = len(gt["in_valid"])
    assert tree["in_child"].shape[0] == ni
    assert _first_diff(tree["in_child"][1:], gt["in_child"][1:]) is None
    assert np.array_equal(tree["in_border"][1:].view(np.uint32), gt["in_border"][1:].view(np.uint32))
    assert np.array_equal(tree["in_pivot"][1:, :128], gt["in_pivot"][1:, :128])
    ix.close()


@pytest.mark.parametrize("batch", [1000, 5000])
def test_device_anng_batch_size_matches_reference(batch):
    """`ngt create -d 128 -o f -D 2 -b <batch>` (batchSizeForCreation,
    Command.cpp:41, Index.cpp:1297): the same edge lists and DVP tree leaves as
    the reference CLI's build (tests/golden/make_batch_goldens.py).  At 5000
    the whole data set is one batch, so every edge comes from the batch's
    pairwise distances (Index.cpp:690-703)."""
    rows, valid = F.read_obj(os.path.join(GOLD, "c1_anng", "obj"), 128, np.float32)
    gold = os.path.join(GOLD, "c1_anng_b%d" % batch)
    ix = DeviceIndex("l2", "float", 128)
    ix.set_objects(rows, valid)
    (offs, ids, ds), tree = ix.build_anng(batch_size_for_creation=batch)
    goffs, gids, gds = F.read_grp(os.path.join(gold, "grp"))
    assert len(offs) == len(goffs)
    for v in range(1, len(offs) - 1):
        a, b = int(offs[v]), int(offs[v + 1])
        c, d = int(goffs[v]), int(goffs[v + 1])
        assert list(ids[a:b]) == list(gids[c:d]), ("node", v)
        assert np.array_equal(ds[a:b].view(np.uint32), gds[c:d].view(np.uint32)), ("node", v)
    gt = F.read_tre(os.path.join(gold, "tre"), 128, np.float32)
    assert _first_diff(tree["leaf_off"], gt["leaf_off"]) is None, _first_diff(tree["leaf_off"], gt["leaf_off"])
    assert _first_diff(tree["leaf_ids"], gt["leaf_ids"]) is None, _first_diff(tree["leaf_ids"], gt["leaf_ids"])
    assert _first_diff(tree["in_child"][1:], gt["in_child"][1:]) is None
    ix.close()


def test_capi_create_index_byte_identical(tmp_path):
    """ngt_create_graph_and_tree + ngt_insert_index_as_float x 5000 +
    ngt_create_index + ngt_save_index == the reference's files."""
    rows, valid = F.read_obj(os.path.join(GOLD, "c1_anng", "obj"), 128, np.float32)
    path = str(tmp_path / "anng")
    base.Index.create(path, 128, edge_size_for_creation=10, edge_size_for_search=40)
    ix = base.Index(path)
    for i in range(1, rows.shape[0]):
        ix.insert_object(rows[i, :128])
    ix.build_index(24)
    out = str(tmp_path / "saved")
    ix.save(out)
    for f in ["obj", "grp", "tre"]:
        assert filecmp.cmp(os.path.join(out, f), os.path.join(GOLD, "c1_anng", f), shallow=False), f
    # and the built index searches like the reference-built one
    q = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    g = np.load(os.path.join(GOLD, "search_c1_anng_tr_0.1.npz"))
    bi, bd, bn = ix.batch_search(q, 10, 0.1)
    for i in range(len(q)):
        ref = g["ids"][i][g["ids"][i] >= 0]
        assert list(bi[i, :bn[i]]) == list(ref), i
    ix.close()


def test_capi_incremental_create_index(tmp_path):
    """createIndex inserts only the objects without a graph node
    (Index.cpp:618-621): 2,400 objects built and saved, the index reopened,
    2,600 more appended and built -- at a batch boundary (200) this is the
    reference's one-shot build, so the files equal the golden ones."""
    rows, valid = F.read_obj(os.path.join(GOLD, "c1_anng", "obj"), 128, np.float32)
    a = str(tmp_path / "a")
    base.Index.create(a, 128, edge_size_for_creation=10, edge_size_for_search=40)
    ix = base.Index(a)
    for i in range(1, 2401):
        ix.insert_object(rows[i, :128])
    ix.build_index(8)
    ix.save(a)
    ix.close()
    ix = base.Index(a)
    for i in range(2401, rows.shape[0]):
        ix.insert_object(rows[i, :128])
    ix.build_index(8)
    out = str(tmp_path / "b")
    ix.save(out)
    ix.close()
    for f in ["obj", "grp", "tre"]:
        assert filecmp.cmp(os.path.join(out, f), os.path.join(GOLD, "c1_anng", f), shallow=False), f
