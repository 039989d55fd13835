"""The launch schedule "probe and resume" (ngt_amd_api.cpp run_search,
search_kernels.hip): a probe launch runs every query for B expansions and
pauses the unfinished ones with their state saved (counters, results,
unchecked keys in LDS and spill, the popped ids); a counting sort orders them
by the unchecked keys within their exploration radius; a resume launch
rebuilds each one's accepted-only visited set and continues it.  The search
of every query is NeighborhoodGraph::searchReadOnlyGraph's (lib/NGT/Graph.cpp:
398-495) whatever the split: ids, distance bits, result counts, expansions
and edges read equal the one-launch search's and the oracle's."""
import numpy as np
import pytest

import oracle_py as O
from ngt_amd.device import SEED_GIVEN, DeviceIndex
from test_gpu_lookahead import _graph

pytestmark = pytest.mark.gpu


def _setup(n=6000, dim=128, deg=100, nq=600, seed=21):
    rows, offs, edges = _graph(n, dim, deg, seed)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(seed + 1)
    qs = rng.random((nq, dim), dtype=np.float32)
    seeds = [rng.choice(np.arange(1, n), 10, replace=False).astype(np.uint32) for _ in range(nq)]
    return ix, rows, offs, edges, qs, seeds


def _search(ix, qs, seeds, eps, k=10):
    # accepted-only visited set, 1-byte filter: the throughput path the schedule serves
    return ix.search(qs, k=k, epsilon=eps, edge_size=0, seed_mode=SEED_GIVEN, seeds=seeds, visited_hash_log2=-2,
                     distance_filter=1)


@pytest.mark.parametrize("budget,cq", [(1, None), (7, None), (40, None), (25, "64")])
def test_probe_and_resume_identical(monkeypatch, budget, cq):
    """Forced budgets: 1 (every query paused right after its first pop), 7
    and 40 (some queries end inside the probe; at epsilon 0.3 some spill more
    keys than a record holds and run to their end), and a 64-key LDS
    unchecked array (keys in the HBM spill are saved and restored too)."""
    monkeypatch.setenv("NGT_AMD_LA", "0")  # the one-expansion kernel
    ix, rows, offs, edges, qs, seeds = _setup()
    if cq:
        monkeypatch.setenv("NGT_AMD_CQ_CAP", cq)
    for eps in (0.1, 0.3):
        monkeypatch.setenv("NGT_AMD_SCHED", "0")
        ai, ad, an, ac = _search(ix, qs, seeds, eps)
        assert ix.last_search_budget() == 0
        monkeypatch.setenv("NGT_AMD_SCHED", "1")
        monkeypatch.setenv("NGT_AMD_SCHED_B", str(budget))
        bi, bd, bn, bc = _search(ix, qs, seeds, eps)
        monkeypatch.delenv("NGT_AMD_SCHED_B")
        assert ix.last_search_budget() == budget
        assert ix.last_search_lookahead() == -1
        assert np.array_equal(an, bn)
        assert np.array_equal(ai, bi)
        assert np.array_equal(ad.view(np.uint32), bd.view(np.uint32))
        for c in (2, 4):  # expansions, edges read: the same traversal
            assert np.array_equal(ac[:, c], bc[:, c]), (eps, c)
        # evaluations: never fewer; more only where a resume re-evaluated an
        # accepted id that compaction had dropped (ngt_kernels.h SearchArgs)
        assert (bc[:, 0] >= ac[:, 0]).all(), eps
        assert (bc[:, 2] > budget).any()  # some queries were paused and resumed
        for i in range(0, len(qs), 97):
            oi, od, _ = O.search("l2", rows, offs, edges, qs[i], seeds[i], 10, np.float32(eps))
            assert list(bi[i, :bn[i]]) == list(oi), (eps, i)
            assert np.array_equal(bd[i, :bn[i]].view(np.uint32), od.view(np.uint32)), (eps, i)
    ix.close()


def test_schedule_from_earlier_launches(monkeypatch):
    """Without a forced budget the second launch of a configuration takes a
    quarter of the first one's mean expansions per query (a launch with more
    queries than slots); results stay identical."""
    monkeypatch.setenv("NGT_AMD_LA", "0")
    monkeypatch.delenv("NGT_AMD_SCHED_B", raising=False)
    monkeypatch.setenv("NGT_AMD_SCHED", "1")
    ix, rows, offs, edges, qs, seeds = _setup(n=4000, deg=80, nq=6000, seed=33)
    ai, ad, an, ac = _search(ix, qs, seeds, 0.2)
    slots = ix.last_search_slots()
    bi, bd, bn, bc = _search(ix, qs, seeds, 0.2)
    if len(qs) * 4 >= slots * 5:
        mean = ac[:, 2].astype(np.float64).mean()
        assert ix.last_search_budget() == max(8, int(mean * 0.25))
    assert np.array_equal(ai, bi) and np.array_equal(an, bn)
    assert np.array_equal(ad.view(np.uint32), bd.view(np.uint32))
    assert np.array_equal(ac[:, 2], bc[:, 2])
    ix.close()
