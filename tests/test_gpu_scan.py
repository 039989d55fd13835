"""Parity of the batch exact scans (the batch form of
ObjectSpaceRepository::linearSearch, ObjectSpaceRepository.h:466-502) against
the oracle: identical ids and distance bits.  k <= 16 runs the matrix-core
filtered scan (scan_mfma.hip), k = 32 the query-tiled FMA scan
(scan_kernels.hip); cases cover padded widths Dp = 16..960, ragged query
blocks, tiny tables, removed objects, duplicate rows (ties ranked by id), a
finite radius, data far from the origin (wide filter margins) and Cosine."""
import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def _rows(n, dim, seed, dups=0):
    rng = np.random.default_rng(seed)
    rows = np.zeros((n, dim), np.float32)
    rows[1:] = rng.random((n - 1, dim), dtype=np.float32)
    for i in range(dups):  # exact duplicates: equal distances, rank by id
        rows[n - 1 - i] = rows[1 + i]
    return rows


@pytest.mark.parametrize("dim,k", [(8, 10), (20, 1), (100, 10), (128, 32), (200, 7), (256, 10)])
def test_scan_matches_oracle(dim, k):
    from ngt_amd.device import DeviceIndex
    n, nq = 12001, 200  # 200 queries: one full and one ragged 128-query block
    rows = _rows(n, dim, 11 + dim, dups=40)
    rng = np.random.default_rng(dim)
    qs = rng.random((nq, dim), dtype=np.float32)
    qs[:20] = rows[1:21]  # queries equal to objects: distance 0 ties
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    gi, gd, gn = ix.linear_search(qs, k=k)
    dp = ix.dp
    pad = np.zeros((n, dp), np.float32)
    pad[:, :dim] = rows
    qp = np.zeros((nq, dp), np.float32)
    qp[:, :dim] = qs
    oi, od, on = O.linear_search_batch("l2", pad, qp, k, threads=8)
    assert np.array_equal(gn, on)
    for q in range(nq):
        m = int(on[q])
        assert np.array_equal(gi[q, :m], oi[q, :m]), q
        assert np.array_equal(gd[q, :m].view(np.uint32), od[q, :m].view(np.uint32)), q


def test_scan_removed_objects_and_radius():
    from ngt_amd.device import DeviceIndex
    n, dim, nq, k = 9000, 64, 160, 10
    rows = _rows(n, dim, 5)
    valid = np.ones(n, np.uint8)
    valid[0] = 0
    valid[np.random.default_rng(2).choice(np.arange(1, n), 700, replace=False)] = 0
    qs = np.random.default_rng(3).random((nq, dim), dtype=np.float32)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows, valid=valid)
    for radius in (-1.0, 3.0):
        gi, gd, gn = ix.linear_search(qs, k=k, radius=radius)
        for q in range(nq):
            oi, od = O.linear_search("l2", rows, qs[q], k, valid=valid, radius=radius)
            assert gn[q] == len(oi), q
            assert np.array_equal(gi[q, :len(oi)], oi), q
            assert np.array_equal(gd[q, :len(oi)].view(np.uint32), od.view(np.uint32)), q


@pytest.mark.parametrize("metric,dim,n,nq,k,offset", [
    ("cosine", 100, 6001, 150, 10, 0.0),
    ("cosine", 960, 3001, 64, 10, 0.0),
    ("cosine", 40, 5001, 40, 16, -0.5),   # mixed signs: cosines spread over [-1, 1]
    ("l2", 128, 8001, 130, 16, 500.0),    # norms >> distances: the filter margin is wide
    ("l2", 24, 300, 33, 10, 0.0),         # one partial tile, one partial query block
])
def test_scan_metrics_and_shapes(metric, dim, n, nq, k, offset):
    from ngt_amd.device import DeviceIndex
    rng = np.random.default_rng(dim + n)
    rows = np.zeros((n, dim), np.float32)
    rows[1:] = rng.random((n - 1, dim), dtype=np.float32) + np.float32(offset)
    qs = rng.random((nq, dim), dtype=np.float32) + np.float32(offset)
    qs[:5] = rows[7:12]
    ix = DeviceIndex(metric, "float", dim)
    ix.set_objects(rows)
    gi, gd, gn = ix.linear_search(qs, k=k)
    dp = ix.dp
    pad = np.zeros((n, dp), np.float32)
    pad[:, :dim] = rows
    qp = np.zeros((nq, dp), np.float32)
    qp[:, :dim] = qs
    oi, od, on = O.linear_search_batch(metric, pad, qp, k, threads=8)
    assert np.array_equal(gn, on)
    for q in range(nq):
        m = int(on[q])
        assert np.array_equal(gi[q, :m], oi[q, :m]), q
        assert np.array_equal(gd[q, :m].view(np.uint32), od[q, :m].view(np.uint32)), q


def test_scan_cosine_radius_and_removed():
    from ngt_amd.device import DeviceIndex
    n, dim, nq, k = 7000, 64, 96, 10
    rows = _rows(n, dim, 21)
    valid = np.ones(n, np.uint8)
    valid[0] = 0
    valid[np.random.default_rng(5).choice(np.arange(1, n), 500, replace=False)] = 0
    qs = np.random.default_rng(6).random((nq, dim), dtype=np.float32)
    ix = DeviceIndex("cosine", "float", dim)
    ix.set_objects(rows, valid=valid)
    for radius in (-1.0, 0.12):
        gi, gd, gn = ix.linear_search(qs, k=k, radius=radius)
        for q in range(nq):
            oi, od = O.linear_search("cosine", rows, qs[q], k, valid=valid, radius=radius)
            assert gn[q] == len(oi), q
            assert np.array_equal(gi[q, :len(oi)], oi), q
            assert np.array_equal(gd[q, :len(oi)].view(np.uint32), od.view(np.uint32)), q
