"""The lookahead search kernel (ngt_amd/csrc/search_la.hip): one step expands
the node the reference pops next plus the next keys in line, and commits them
strictly in the reference's pop order (NeighborhoodGraph::searchReadOnlyGraph,
lib/NGT/Graph.cpp:398-495).  Bar: ids and float distance bits identical to
the oracle restatement; with the full visited set also the distance-computation
counts; with the accepted-only set (visited_hash_log2 = -2) counts >= the
reference's.  Both forms run: a wave per query (launches of >= 2 queries per
CU) and eight waves per query (smaller launches: single C-API calls,
construction batches)."""
import os

import numpy as np
import pytest

import oracle_py as O
from ngt_amd.device import SEED_GIVEN, SEED_TREE, DeviceIndex
from test_gpu_parity import _random_graph, device_index, queries

pytestmark = pytest.mark.gpu


def _graph(n, dim, deg, seed):
    if deg <= 64:
        return _random_graph(n, dim, deg, seed)
    # long lists: 16 near neighbours by index plus random far ones, sorted
    # so the lists are distinct per node
    rng = np.random.default_rng(seed)
    rows = np.zeros((n, dim), np.float32)
    rows[1:] = rng.random((n - 1, dim), dtype=np.float32)
    e = np.zeros((n - 1, deg), np.uint32)
    for v in range(1, n):
        cand = np.unique(rng.integers(1, n, deg * 2))
        cand = cand[cand != v]
        rng.shuffle(cand)
        e[v - 1] = cand[:deg]
    offs = np.zeros(n + 1, np.uint64)
    offs[2:] = np.arange(1, n, dtype=np.uint64) * deg
    return rows, offs, e.reshape(-1)


@pytest.mark.parametrize("nq", [24, 600])
@pytest.mark.parametrize("deg", [24, 100, 200])
@pytest.mark.parametrize("visited", [0, -2])
def test_lookahead_matches_oracle(monkeypatch, nq, deg, visited):
    n, dim = 4000, 128
    rows, offs, edges = _graph(n, dim, deg, 21 + deg)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(deg + nq)
    qs = rng.random((nq, dim), dtype=np.float32)
    seeds = [rng.choice(np.arange(1, n), 10, replace=False).astype(np.uint32) for _ in range(nq)]
    radius = float(np.sqrt(dim / 6.0))
    # force the form under test (the default routing sends long lists of
    # large launches to the one-expansion kernel)
    want_mode = 1 if nq < 2 * 256 else 0
    monkeypatch.setenv("NGT_AMD_LA", "2" if want_mode == 1 else "1")
    for eps, rad, cq, es in [(0.0, -1.0, "", 0), (0.2, -1.0, "", 0), (1.0, -1.0, "64", 0), (-0.05, -1.0, "", 0),
                             (0.2, radius, "", 0), (0.3, -1.0, "", 40)]:
        if cq:
            monkeypatch.setenv("NGT_AMD_CQ_CAP", cq)
        else:
            monkeypatch.delenv("NGT_AMD_CQ_CAP", raising=False)
        gi, gd, gn, cnt = ix.search(qs, k=20, epsilon=eps, radius=rad, edge_size=es, seed_mode=SEED_GIVEN,
                                    seeds=seeds, visited_hash_log2=visited)
        mode = ix.last_search_lookahead()
        assert mode == want_mode, (mode, want_mode)
        kw = {} if rad < 0 else {"radius": rad}
        oi, od, on, oc = O.search_batch("l2", rows, offs, edges, qs, seeds, 20, np.float32(eps), edge_size=es,
                                        threads=os.cpu_count() or 1, **kw)
        for i in range(nq):
            assert list(gi[i, :gn[i]]) == list(oi[i, :on[i]]), (eps, rad, i)
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od[i, :on[i]].view(np.uint32)), (eps, rad, i)
        if visited == 0:
            assert np.array_equal(cnt[:, 0], oc[:, 0].astype(np.uint64)), (eps, rad)
            assert np.array_equal(cnt[:, 2], oc[:, 2].astype(np.uint64))  # expansions
        else:
            assert (cnt[:, 0] >= oc[:, 0]).all()
    ix.close()


@pytest.mark.parametrize("lmax", ["256", "512"])
def test_lookahead_small_list_capacity(monkeypatch, lmax):
    """Target lists longer than the step's list capacity: the step keeps only
    the targets whose lists fit (the popped node's always does)."""
    monkeypatch.setenv("NGT_AMD_LA_LMAX", lmax)
    n, dim, deg = 3000, 128, 200
    rows, offs, edges = _graph(n, dim, deg, 5)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(6)
    qs = rng.random((16, dim), dtype=np.float32)
    seeds = [rng.choice(np.arange(1, n), 10, replace=False).astype(np.uint32) for _ in range(16)]
    gi, gd, gn, cnt = ix.search(qs, k=10, epsilon=0.3, edge_size=0, seed_mode=SEED_GIVEN, seeds=seeds)
    oi, od, on, oc = O.search_batch("l2", rows, offs, edges, qs, seeds, 10, np.float32(0.3), edge_size=0)
    assert np.array_equal(gn, on)
    for i in range(16):
        assert list(gi[i, :gn[i]]) == list(oi[i, :on[i]])
        assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od[i, :on[i]].view(np.uint32))
    assert np.array_equal(cnt[:, 0], oc[:, 0].astype(np.uint64))
    ix.close()


@pytest.mark.parametrize("name", ["c1_onng", "c1_anng"])
def test_lookahead_equals_single_expansion_kernel(monkeypatch, name):
    """On the reference-built C1 indexes with tree seeds, the lookahead kernel
    (both forms) and the one-expansion kernel return the same ids, distance
    bits and work counters (distances, expansions, edges read)."""
    ix = device_index(name)[0]
    qs = np.tile(queries(), (6, 1))  # 600 queries: the wave-per-query form
    out = {}
    for la in ["0", "1", "2"]:  # off, the wave-per-query form forced, the 8-wave form
        monkeypatch.setenv("NGT_AMD_LA", la)
        for nq in (40, 600):
            for eps in (0.0, 0.1):
                gi, gd, gn, cnt = ix.search(qs[:nq], k=10, epsilon=eps, seed_mode=SEED_TREE)
                out[(la, nq, eps)] = (gi, gd, gn, cnt, ix.last_search_lookahead())
    for nq in (40, 600):
        for eps in (0.0, 0.1):
            la = "2" if nq < 512 else "1"
            a, b = out[("0", nq, eps)], out[(la, nq, eps)]
            assert a[4] == -1 and b[4] == (1 if nq < 512 else 0)
            assert np.array_equal(a[2], b[2])
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
            for c in (0, 2, 4):
                assert np.array_equal(a[3][:, c], b[3][:, c]), (nq, eps, c)
    ix.close()


@pytest.mark.parametrize("knobs", [{"NGT_AMD_LAT_TAIL": "128"}, {"NGT_AMD_LAT_SLOTS": "2"},
                                   {"NGT_AMD_LAT_SLOTS": "3", "NGT_AMD_LAT_TAIL": "256"},
                                   {"NGT_AMD_LAT_SLOTS": "4"}, {"NGT_AMD_LAT_SLOTS": "6", "NGT_AMD_LAT_TAIL": "512"}])
@pytest.mark.parametrize("deg", [24, 150])
def test_latency_kernel_spill_and_slots(monkeypatch, knobs, deg):
    """The speculating latency kernel (search_lat.hip) with a tail small
    enough to push keys to the HBM spill and refill from it, with so few
    speculation slots that head entries lose theirs (orphaned slots reaped,
    and the deepest tagged head entry gives its slot up when every slot is
    held and the node to expand has none): ids, distance bits and the
    reference's distance/expansion counts."""
    for kv in knobs.items():
        monkeypatch.setenv(*kv)
    monkeypatch.setenv("NGT_AMD_LA", "2")
    n, dim = 5000, 128
    rows, offs, edges = _graph(n, dim, deg, 77 + deg)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(deg)
    qs = rng.random((12, dim), dtype=np.float32)
    seeds = [rng.choice(np.arange(1, n), 10, replace=False).astype(np.uint32) for _ in range(12)]
    for eps in (0.1, 0.5):
        gi, gd, gn, cnt = ix.search(qs, k=30, epsilon=eps, edge_size=0, seed_mode=SEED_GIVEN, seeds=seeds)
        assert ix.last_search_lookahead() == 1
        oi, od, on, oc = O.search_batch("l2", rows, offs, edges, qs, seeds, 30, np.float32(eps), edge_size=0,
                                        threads=os.cpu_count() or 1)
        assert np.array_equal(gn, on)
        for i in range(12):
            assert list(gi[i, :gn[i]]) == list(oi[i, :on[i]]), (eps, i)
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od[i, :on[i]].view(np.uint32)), (eps, i)
        assert np.array_equal(cnt[:, 0], oc[:, 0].astype(np.uint64)), eps
        assert np.array_equal(cnt[:, 2], oc[:, 2].astype(np.uint64)), eps
    ix.close()


@pytest.mark.parametrize("hop", ["0", "1"])
@pytest.mark.parametrize("deg", [24, 40, 150])
def test_latency_kernel_hop_forms(monkeypatch, hop, deg):
    """The latency kernel's hop prefetch -- each list part's nearest fresh
    neighbour read towards L2 by the speculation wave (1, the default) or not
    (0) -- leaves ids, distance bits and the reference's distance/expansion
    counts unchanged, also with two slots (issued, orphaned and re-issued
    head entries)."""
    monkeypatch.setenv("NGT_AMD_LA", "2")
    monkeypatch.setenv("NGT_AMD_LAT_HOP", hop)
    n, dim = 6000, 128
    rows, offs, edges = _graph(n, dim, deg, 91 + deg)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(deg + 3)
    qs = rng.random((12, dim), dtype=np.float32)
    seeds = [rng.choice(np.arange(1, n), 10, replace=False).astype(np.uint32) for _ in range(12)]
    for slots, eps in (("", 0.1), ("", 0.4), ("2", 0.2)):
        if slots:
            monkeypatch.setenv("NGT_AMD_LAT_SLOTS", slots)
        gi, gd, gn, cnt = ix.search(qs, k=20, epsilon=eps, edge_size=0, seed_mode=SEED_GIVEN, seeds=seeds)
        assert ix.last_search_lookahead() == 1
        oi, od, on, oc = O.search_batch("l2", rows, offs, edges, qs, seeds, 20, np.float32(eps), edge_size=0,
                                        threads=os.cpu_count() or 1)
        assert np.array_equal(gn, on)
        for i in range(12):
            assert list(gi[i, :gn[i]]) == list(oi[i, :on[i]]), (eps, i)
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od[i, :on[i]].view(np.uint32)), (eps, i)
        for c in (0, 2):
            assert np.array_equal(cnt[:, c], oc[:, c].astype(np.uint64)), (eps, c)
    ix.close()
