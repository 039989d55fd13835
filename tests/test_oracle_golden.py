"""Pins the CPU restatement (oracle/) against outputs of the reference itself.

The golden fixtures under tests/golden were produced by the reference NGT
1.13.8 CLI (tests/golden/make_goldens.py).  These tests run on CPU only.
"""
import ctypes
import glob
import os

import numpy as np
import pytest

import ngt_files as F
import oracle_py as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dist_cases():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLD, "dist_*.npz"))):
        name = os.path.basename(f)[5:-4]
        metric = name.rsplit("_", 2)[0]
        out.append(pytest.param(f, metric, id=name))
    return out


@pytest.mark.parametrize("path,metric", _dist_cases())
def test_comparators_bit_exact(path, metric):
    """Every edge distance the reference stored in its grp file is reproduced
    bit for bit (PrimitiveComparator.h:105-754 via ObjectSpaceRepository.h:33-283)."""
    z = np.load(path)
    got = O.pair_distances(metric, z["rows"], z["src"], z["dst"])
    ref = z["dist"].astype(np.float32)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def edge_size_for(prop, eps):
    """NeighborhoodGraph::getEdgeSize (lib/NGT/Graph.h:675-692) for sc.edgeSize = -1."""
    es = int(prop["EdgeSizeForSearch"])
    if es == 0:
        return 0
    if es > 0:
        return es
    coef = np.float32(np.float64(np.float32(eps)) + 1.0)
    add = 10 ** ((np.float64(coef) - 1.0) * float(np.float32(int(prop["DynamicEdgeSizeRate"]))))
    return 2 ** 31 - 1 if add >= 2 ** 31 - 1 else int(int(prop["DynamicEdgeSizeBase"]) + add)


def load_index(name):
    d = os.path.join(GOLD, name)
    prop = F.read_prf(os.path.join(d, "prf"))
    dim = int(prop["Dimension"])
    rows, valid = F.read_obj(os.path.join(d, "obj"), dim, np.float32)
    offs, ids, _ = F.read_grp(os.path.join(d, "grp"))
    tree = F.read_tre(os.path.join(d, "tre"), dim, np.float32)
    return prop, rows, valid, offs, ids, tree


def fmt(x):
    # `stream << objects[i].distance` (Command.cpp:349): default 6 significant digits
    return "%g" % float(x)


@pytest.mark.parametrize("name", ["c1_anng", "c1_onng"])
@pytest.mark.parametrize("eps", ["0.0", "0.02", "0.05", "0.1"])
@pytest.mark.parametrize("om", ["r", "w"])
def test_tree_seeded_search_matches_reference(name, eps, om):
    """`ngt search -i t` (GraphAndTreeIndex::search, Index.h:1570-1577)."""
    prop, rows, valid, offs, ids, tree = load_index(name)
    g = np.load(os.path.join(GOLD, "search_%s_t%s_%s.npz" % (name, om, eps)))
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    es = edge_size_for(prop, float(eps))
    for i, q in enumerate(qs):
        seeds, _, _ = O.tree_seeds("l2", tree, q, 10, int(prop["SeedSize"]))
        rid, rd, cnt = O.search("l2", rows, offs, ids, q, seeds, 10, np.float32(float(eps)),
                                edge_size=es)
        gi = g["ids"][i]
        assert list(rid) == list(gi[gi >= 0]), i
        assert [fmt(x) for x in rd] == [fmt(x) for x in g["dists"][i][:len(rd)]], i
        if om == "w":
            # Graph.cpp:604 counts every evaluated neighbour; seeds are only
            # counted under NGT_DISTANCE_COMPUTATION_COUNT (Graph.cpp:287).
            assert int(cnt[0]) - len(seeds) == int(g["ndist"][i]), i


@pytest.mark.parametrize("name", ["c1_anng", "c1_onng"])
def test_k20_search_matches_reference(name):
    prop, rows, valid, offs, ids, tree = load_index(name)
    g = np.load(os.path.join(GOLD, "search_%s_tr_k20_0.2.npz" % name))
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    es = edge_size_for(prop, 0.2)
    for i, q in enumerate(qs):
        seeds, _, _ = O.tree_seeds("l2", tree, q, 20, int(prop["SeedSize"]))
        rid, rd, _ = O.search("l2", rows, offs, ids, q, seeds, 20, np.float32(0.2), edge_size=es)
        assert list(rid) == list(g["ids"][i]), i


def random_seeds(rand, nrows, seed_size):
    """GraphIndex::getRandomSeeds (lib/NGT/Index.h:775-801) over the global rand()."""
    repo = nrows - 1
    seed_size = min(seed_size, repo)
    seeds = []
    while len(seeds) < seed_size:
        r = (float(rand()) + 1.0) / (2147483647.0 + 2.0)
        idx = int(np.floor(repo * r)) + 1
        if idx not in seeds:
            seeds.append(idx)
    return seeds


@pytest.mark.parametrize("name", ["c1_anng", "c1_onng"])
@pytest.mark.parametrize("eps", ["0.0", "0.1"])
def test_graph_only_search_matches_reference(name, eps):
    """`ngt search -i g` (Index::searchUsingOnlyGraph, Index.h:479-484): random seeds
    from the process-wide glibc rand() stream (default seed 1)."""
    prop, rows, valid, offs, ids, tree = load_index(name)
    g = np.load(os.path.join(GOLD, "search_%s_gr_%s.npz" % (name, eps)))
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    es = edge_size_for(prop, float(eps))
    st = O.lib()
    gen = O.ctypes.create_string_buffer(256)
    st.ngto_srand.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    st.ngto_rand.argtypes = [ctypes.c_void_p]
    st.ngto_srand(gen, 1)
    rand = lambda: st.ngto_rand(gen)  # noqa: E731
    for i, q in enumerate(qs):
        seeds = random_seeds(rand, rows.shape[0], int(prop["SeedSize"]))
        rid, rd, _ = O.search("l2", rows, offs, ids, q, np.array(seeds), 10,
                              np.float32(float(eps)), edge_size=es)
        assert list(rid) == list(g["ids"][i][g["ids"][i] >= 0]), i


@pytest.mark.parametrize("name", ["c1_anng", "c1_onng"])
def test_linear_search_matches_reference(name):
    """`ngt search -i s` (ObjectSpaceRepository::linearSearch, ObjectSpaceRepository.h:466-502)."""
    prop, rows, valid, offs, ids, tree = load_index(name)
    g = np.load(os.path.join(GOLD, "search_%s_sr_0.0.npz" % name))
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    for i, q in enumerate(qs):
        rid, rd = O.linear_search("l2", rows, q, 10, valid=valid, radius=3.402823466e38)
        assert list(rid) == list(g["ids"][i]), i
        assert [fmt(x) for x in rd] == [fmt(x) for x in g["dists"][i]], i


def test_glibc_rand_restatement():
    libc = ctypes.CDLL("libc.so.6")
    L = O.lib()
    gen = ctypes.create_string_buffer(256)
    L.ngto_srand.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    L.ngto_rand.argtypes = [ctypes.c_void_p]
    for seed in [1, 2, 7, 12345, 4000000000]:
        libc.srand(seed)
        L.ngto_srand(gen, seed)
        for _ in range(50):
            assert libc.rand() == L.ngto_rand(gen)


def test_tre_parser_consumes_file():
    for name in ["c1_anng", "c1_onng"]:
        t = F.read_tre(os.path.join(GOLD, name, "tre"), 128, np.float32)
        assert t["root"] == 1
        # every object appears in exactly one leaf
        assert len(t["leaf_ids"]) == 5000
        assert len(set(t["leaf_ids"].tolist())) == 5000
