"""The resident serving grid (ngt_amd/csrc/serve.cpp, the SERVE form of
search_lat.hip): single queries posted to a ring in pinned host memory and
answered by a long-lived launch, the path concurrent ngt_search_index callers
take (lib/NGT/Capi.cpp:377-406).  Bar: every served answer equals the oracle's
restatement of NeighborhoodGraph::search (ids and float distance bits) and the
batch launch's counters, for tree seeds (GraphAndTreeIndex::getSeedsFromTree
on the device, Index.h:1524-1567) and random seeds (getRandomSeeds, the same
rand() stream as a launch), under concurrency, with the HBM spill and slot
reaping forced, and across a change of the index (the grid relaunches)."""
import ctypes
import os
import threading

import numpy as np
import pytest

import oracle_py as O
from ngt_amd import lib
from ngt_amd.device import SEED_RANDOM, SEED_TREE, DeviceIndex
from test_gpu_lookahead import _graph

pytestmark = pytest.mark.gpu


def _anng(n=4000, dim=128, seed=3):
    """A device-built ANNG + DVP tree over random float rows, loaded as a
    search index (edge size for search 40, seed size 10)."""
    rng = np.random.default_rng(seed)
    rows = np.zeros((n, dim), np.float32)
    rows[1:] = rng.random((n - 1, dim), dtype=np.float32)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    (offs, ids, _), tree = ix.build_anng(edge_size_for_creation=10, edge_size_for_search=40)
    ix.set_graph(offs, ids)
    ix.set_tree(tree)
    ix.set_search_property(edge_size_for_search=40, seed_size=10)
    return ix, rows, offs, ids, tree


def _oracle(rows, offs, ids, tree, q, k, eps, es):
    seeds, _, _ = O.tree_seeds("l2", tree, q, k, 10)
    return O.search("l2", rows, offs, ids, q, seeds, k, np.float32(eps), edge_size=es)


def test_served_equals_oracle_concurrent():
    ix, rows, offs, ids, tree = _anng()
    rng = np.random.default_rng(11)
    qs = rng.random((96, rows.shape[1]), dtype=np.float32)
    es = ix.resolve_edge_size(-1, 0.1)
    s0, _ = ix.serve_stats()
    got = [None] * len(qs)
    errors = []

    def worker(t):
        try:
            for i in range(t, len(qs), 8):
                got[i] = ix.search_served(qs[i], k=10, epsilon=0.1, seed_mode=SEED_TREE)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:3]
    s1, launches = ix.serve_stats()
    assert s1 - s0 == len(qs) and launches >= 1
    try:
        bi, bd, bn, bc = ix.search(qs, k=10, epsilon=0.1, seed_mode=SEED_TREE)
    except Exception as e:  # noqa: BLE001  (diagnostic: which form, and again?)
        form = ix.last_search_lookahead()
        try:
            ix.search(qs, k=10, epsilon=0.1, seed_mode=SEED_TREE)
            again = "ok"
        except Exception as e2:  # noqa: BLE001
            again = repr(e2)
        raise AssertionError("batch search failed (form %d): %r; again: %s" % (form, e, again))
    for i in range(len(qs)):
        assert got[i] is not None, "the grid does not serve this index"
        gi, gd, gc = got[i]
        oi, od, _ = _oracle(rows, offs, ids, tree, qs[i], 10, 0.1, es)
        assert list(gi) == list(oi), i
        assert np.array_equal(gd.view(np.uint32), od.view(np.uint32)), i
        for c in (0, 2, 4):  # distances, expansions, edges read: the launch's
            assert gc[c] == bc[i, c], (i, c)
    ix.close()


@pytest.mark.parametrize("knobs", [{"NGT_AMD_LAT_TAIL": "128"}, {"NGT_AMD_LAT_SLOTS": "2"}])
def test_served_spill_and_slots(monkeypatch, knobs):
    """Long searches (k 30, epsilon 0.5, lists of 150) with the tail forced
    small (HBM spill and refills) or two speculation slots (orphaned slots
    reaped): answers equal the oracle's and the launch's counters."""
    for kv in knobs.items():
        monkeypatch.setenv(*kv)
    n, dim, deg = 5000, 128, 150
    rows, offs, edges = _graph(n, dim, deg, 91)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(4)
    qs = rng.random((6, dim), dtype=np.float32)
    for i, q in enumerate(qs):
        lib().ngt_amd_srand(100 + i)
        r = ix.search_served(q, k=30, epsilon=0.5, edge_size=0, seed_mode=SEED_RANDOM)
        assert r is not None
        lib().ngt_amd_srand(100 + i)
        bi, bd, bn, bc = ix.search(q[None], k=30, epsilon=0.5, edge_size=0, seed_mode=SEED_RANDOM)
        gi, gd, gc = r
        assert list(gi) == list(bi[0, :bn[0]]), i
        assert np.array_equal(gd.view(np.uint32), bd[0, :bn[0]].view(np.uint32)), i
        assert gc[0] == bc[0, 0] and gc[2] == bc[0, 2], i
    ix.close()


def test_grid_stays_while_a_search_runs(monkeypatch):
    """The grid idles out only with nothing posted or in flight: with a 1 ms
    idle time, sequential calls whose searches take longer than that (epsilon
    1.0 over the whole 4k graph) are all answered by one grid -- the idle
    time runs from the last answer, not the last post (serve.cpp,
    search_lat.hip serve_dispatch) -- and equal the launch's answers."""
    import time
    monkeypatch.setenv("NGT_AMD_SERVE_IDLE_MS", "2")
    ix, rows, offs, ids, tree = _anng()
    rng = np.random.default_rng(23)
    qs = rng.random((12, rows.shape[1]), dtype=np.float32)
    ix.search_served(qs[0], k=10, epsilon=0.1, seed_mode=SEED_TREE)  # the grid is up
    _, l0 = ix.serve_stats()
    got, wall = [], []
    for q in qs:
        t = time.perf_counter()
        got.append(ix.search_served(q, k=10, epsilon=1.0, seed_mode=SEED_TREE))
        wall.append(time.perf_counter() - t)
    _, l1 = ix.serve_stats()
    assert all(g is not None for g in got)
    assert min(wall) > 0.003, wall  # every search outlasts the 2 ms idle time
    assert l1 == l0, "grid launches during %d sequential calls: %d (call ms %s)" % (
        len(qs), l1 - l0, [round(w * 1e3, 2) for w in wall])
    bi, bd, bn, bc = ix.search(qs, k=10, epsilon=1.0, seed_mode=SEED_TREE)
    for i, (gi, gd, gc) in enumerate(got):
        assert list(gi) == list(bi[i, :bn[i]]), i
        assert np.array_equal(gd.view(np.uint32), bd[i, :bn[i]].view(np.uint32)), i
        assert gc[2] == bc[i, 2] and gc[2] > 200, (i, gc[2])  # long searches: hundreds of expansions
    ix.close()


def test_served_random_seeds_follow_the_rand_stream():
    """getRandomSeeds draws the same rand() stream whether the query is served
    or launched: after the same ngt_amd_srand both answer identically."""
    n, dim, deg = 4000, 96, 24
    rows, offs, edges = _graph(n, dim, deg, 12)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(8)
    qs = rng.random((20, dim), dtype=np.float32)
    lib().ngt_amd_srand(7)
    served = [ix.search_served(q, k=10, epsilon=0.1, edge_size=0, seed_mode=SEED_RANDOM) for q in qs]
    lib().ngt_amd_srand(7)
    for i, q in enumerate(qs):
        bi, bd, bn, _ = ix.search(q[None], k=10, epsilon=0.1, edge_size=0, seed_mode=SEED_RANDOM)
        gi, gd, _ = served[i]
        assert list(gi) == list(bi[0, :bn[0]]), i
        assert np.array_equal(gd.view(np.uint32), bd[0, :bn[0]].view(np.uint32)), i
    ix.close()


def test_served_follows_index_changes():
    """New rows under a running grid: the next query relaunches it over the
    new index, and the grid stops on request and when idle."""
    ix, rows, offs, ids, tree = _anng(n=3000, seed=5)
    rng = np.random.default_rng(2)
    q = rng.random(rows.shape[1], dtype=np.float32)
    es = ix.resolve_edge_size(-1, 0.1)
    gi, gd, _ = ix.search_served(q, k=10, epsilon=0.1)
    oi, od, _ = _oracle(rows, offs, ids, tree, q, 10, 0.1, es)
    assert list(gi) == list(oi)
    _, l0 = ix.serve_stats()
    rows2 = rows.copy()
    rows2[1:] = rows2[1:] * np.float32(0.5) + np.float32(0.25)
    ix.set_objects(rows2)
    ix.set_graph(offs, ids)
    ix.set_tree(tree)
    gi, gd, _ = ix.search_served(q, k=10, epsilon=0.1)
    oi, od, _ = _oracle(rows2, offs, ids, tree, q, 10, 0.1, es)
    assert list(gi) == list(oi)
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    _, l1 = ix.serve_stats()
    assert l1 > l0
    ix.serve_stop()
    gi2, _, _ = ix.search_served(q, k=10, epsilon=0.1)  # relaunched after the stop
    assert list(gi2) == list(gi)
    ix.close()


def test_fresh_stream_error_word_zero_under_resident_grid():
    """GPUTEST_r03's "flag 36": a fresh call stream's launch context once read
    a stale error word because its zero-fill went to the null stream and sat
    behind the resident grid.  While served calls keep the grid resident,
    every new stream's word must read 0 before its first launch, and a batch
    search on it must succeed."""
    import torch
    ix, rows, offs, ids, tree = _anng(n=3000, seed=7)
    rng = np.random.default_rng(5)
    qs = rng.random((8, rows.shape[1]), dtype=np.float32)
    assert ix.search_served(qs[0], k=10, epsilon=0.1) is not None
    stop = threading.Event()
    errors = []

    def keep_resident():
        try:
            i = 0
            while not stop.is_set():
                ix.search_served(qs[i % len(qs)], k=10, epsilon=0.1)
                i += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = threading.Thread(target=keep_resident)
    th.start()
    try:
        dev = torch.device("cuda", 0)
        dq = torch.from_numpy(np.ascontiguousarray(qs)).to(dev)
        for _ in range(6):
            st = torch.cuda.Stream(dev)
            w = ctypes.c_int(-1)
            assert ix.L.ngt_amd_stream_error_word(ix.h, st.cuda_stream, ctypes.byref(w)) == 0
            assert w.value == 0
            oi = torch.zeros((len(qs), 10), dtype=torch.int32, device=dev)
            od = torch.zeros((len(qs), 10), dtype=torch.float32, device=dev)
            on = torch.zeros((len(qs),), dtype=torch.int32, device=dev)
            ix.search_device(dq.data_ptr(), dq.shape[1] * 4, len(qs), oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                             k=10, epsilon=0.1, seed_mode=SEED_TREE, stream=st.cuda_stream)
            st.synchronize()
    finally:
        stop.set()
        th.join()
    assert not errors, errors[:3]
    ix.close()


def test_index_changes_under_concurrent_served_calls():
    """a served call that read the index before a mutation began
    must not configure or relaunch the grid with the old buffers.  Four
    threads post served queries while the main thread replaces the graph
    (which releases and rebuilds the padded adjacency) and the tree, over and
    over, with identical contents: every answer, served or not, equals the
    oracle's."""
    ix, rows, offs, ids, tree = _anng(n=3000, seed=9)
    rng = np.random.default_rng(6)
    qs = rng.random((16, rows.shape[1]), dtype=np.float32)
    es = ix.resolve_edge_size(-1, 0.1)
    want = [_oracle(rows, offs, ids, tree, q, 10, 0.1, es) for q in qs]
    stop = threading.Event()
    errors, served = [], [0]

    def worker(t):
        try:
            i = t
            while not stop.is_set():
                r = ix.search_served(qs[i % len(qs)], k=10, epsilon=0.1)
                if r is not None:
                    oi, od, _ = want[i % len(qs)]
                    if list(r[0]) != list(oi) or not np.array_equal(r[1].view(np.uint32), od.view(np.uint32)):
                        errors.append("query %d differs" % (i % len(qs)))
                    served[0] += 1
                i += 4
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    try:
        for _ in range(12):
            ix.set_graph(offs, ids)
            ix.set_tree(tree)
    finally:
        stop.set()
        for t in th:
            t.join()
    assert not errors, errors[:3]
    assert served[0] > 0
    bi, bd, bn, _ = ix.search(qs, k=10, epsilon=0.1, seed_mode=SEED_TREE)
    for i in range(len(qs)):
        assert list(bi[i, :bn[i]]) == list(want[i][0]), i
    ix.close()

