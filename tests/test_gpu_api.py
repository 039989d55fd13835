"""GPU tests of the drop-in surface added in round 2: comparators against the
reference-harness fixtures (pair_*.npz), query normalization (norm_*.npz),
insertion into normalized-metric and SparseJaccard indexes through the C API,
concurrent single-query callers (coalesced launches), and the linear search
on concurrent streams.  Every result is compared with the oracle or the
reference's own outputs."""
import ctypes
import glob
import os
import tempfile
import threading

import numpy as np
import pytest

import ngt_files as F
import oracle_py as O
from ngt_amd import base, lib
from ngt_amd.device import DeviceIndex

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _pair_cases():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLD, "pair_*.npz"))):
        name = os.path.basename(f)[5:-4]
        out.append(pytest.param(f, name.rsplit("_", 2)[0], name.rsplit("_", 2)[1], id=name))
    return out


@pytest.mark.parametrize("path,metric,ot", _pair_cases())
def test_gpu_pairs_bit_exact_vs_reference(path, metric, ot):
    """compareSparseJaccardDistance (PrimitiveComparator.h:399-418) and the uint8
    dot-product metrics (:479-485) on the device: bit-exact vs the reference."""
    z = np.load(path)
    a, b, dim = z["a"], z["b"], int(z["dim"])
    odim = dim + 1 if metric == "sparse_jaccard" else dim  # Index.cpp:488-490
    ix = DeviceIndex(metric, "float" if ot == "f" else "uint8", odim)
    assert ix.dp == a.shape[1]
    rows = np.zeros((a.shape[0] + 1, a.shape[1]), a.dtype)
    rows[1:] = b
    ix.set_objects(rows)
    n = a.shape[0]
    got = ix.distances(a, np.arange(n, dtype=np.uint32), np.arange(1, n + 1, dtype=np.uint32))
    ref = z["dist"]
    bad = np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert len(bad) == 0, (bad[:10], got[bad[:5]], ref[bad[:5]])
    ix.close()


@pytest.mark.parametrize("dim", [20, 100, 128, 960])
def test_gpu_query_normalization(dim):
    """Index::allocateObject for the normalized metrics (ObjectSpace::normalize,
    ObjectSpace.h:251-266) on the device: bit-identical to the oracle's
    restatement (the stored form of inserted objects) and within 2 ulp of the
    reference's -Ofast build (whose rsqrt step is host-CPU dependent)."""
    import torch
    z = np.load(os.path.join(GOLD, "norm_f_d%d.npz" % dim))
    x, y = z["x"], z["y"]
    ix = DeviceIndex("normalized_cosine", "float", dim)
    dev = torch.device("cuda:0")
    d_in = torch.from_numpy(x).to(dev)
    d_out = torch.zeros((x.shape[0], ix.dp), dtype=torch.float32, device=dev)
    ix.prepare_queries_device(d_in.data_ptr(), x.shape[0], d_out.data_ptr())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    assert np.all(got[:, dim:] == 0)
    got = got[:, :dim]
    for i in range(x.shape[0]):
        v = np.ascontiguousarray(x[i].copy())
        O.lib().ngto_normalize_f32(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), dim)
        assert np.array_equal(got[i].view(np.uint32), v.view(np.uint32)), i
    ulp = np.spacing(np.abs(y)).astype(np.float32)
    assert np.all(np.abs(got - y) <= 2 * ulp)
    ix.close()


def _edge_size(prop, eps):
    es = int(prop["EdgeSizeForSearch"])
    return 0 if es == 0 else es


def _build_via_capi(tmp, dim, distance_type, rows, object_type="Float"):
    """ngt_create_graph_and_tree + ngt_insert_index_as_float (normalizing for the
    normalized metrics, ObjectSpaceRepository.h:560-566) + ngt_create_index on the
    device + ngt_save_index; returns the open index and its saved files."""
    path = os.path.join(tmp, "idx")
    base.Index.create(path, dim, edge_size_for_creation=10, edge_size_for_search=40, object_type=object_type,
                      distance_type=distance_type)
    ix = base.Index(path)
    for r in rows:
        ix.insert_object(r)
    ix.build_index()
    ix.save()
    prop = F.read_prf(os.path.join(path, "prf"))
    odim = ix.object_dim
    dt = np.float32 if object_type == "Float" else np.uint8
    srows, valid = F.read_obj(os.path.join(path, "obj"), odim, dt)
    offs, ids, _ = F.read_grp(os.path.join(path, "grp"))
    tree = F.read_tre(os.path.join(path, "tre"), odim, dt)
    return ix, prop, srows, offs, ids, tree


@pytest.mark.parametrize("metric,name", [("normalized_cosine", "Normalized Cosine"),
                                         ("normalized_angle", "Normalized Angle"),
                                         ("normalized_l2", "Normalized L2")])
def test_capi_normalized_insert_and_search(metric, name):
    """Objects inserted into a normalized-metric index are stored normalized
    (ObjectSpaceRepository.h:560-566); the device-built ANNG is searched with
    tree seeds and equals the oracle's search over the saved files bit for bit."""
    rng = np.random.default_rng(0x4E)
    dim, n = 48, 1500
    X = rng.random((n, dim), dtype=np.float32) - np.float32(0.3)
    with tempfile.TemporaryDirectory() as tmp:
        ix, prop, srows, offs, ids, tree = _build_via_capi(tmp, dim, name, X)
        for i in range(0, n, 37):
            v = np.ascontiguousarray(X[i].copy())
            O.lib().ngto_normalize_f32(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), dim)
            assert np.array_equal(srows[i + 1, :dim].view(np.uint32), v.view(np.uint32)), i
            assert np.array_equal(np.asarray(ix.get_object(i + 1), np.float32).view(np.uint32), v.view(np.uint32))
        qs = rng.random((32, dim), dtype=np.float32) - np.float32(0.3)
        gi, gd, gn = ix.batch_search(qs, 10, 0.1)
        es = _edge_size(prop, 0.1)
        dp = srows.shape[1]
        for i in range(len(qs)):
            q = np.zeros(dp, np.float32)
            v = np.ascontiguousarray(qs[i].copy())
            O.lib().ngto_normalize_f32(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), dim)
            q[:dim] = v
            seeds, _, _ = O.tree_seeds(metric, tree, q, 10, int(prop["SeedSize"]))
            oid, od, _ = O.search(metric, srows, offs, ids, q, seeds, 10, np.float32(0.1), edge_size=es)
            assert list(gi[i, :gn[i]]) == list(oid), i
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32)), i
        ix.close()


def _sparse_rows(rng, n, dim, universe):
    odim = dim + 1
    out = np.zeros((n, odim), np.uint32)
    for i in range(n):
        m = int(rng.integers(1, dim + 1))
        out[i, :m] = np.sort(rng.choice(np.arange(1, universe + 1), size=m, replace=False))
    return out.view(np.float32)


def test_capi_sparse_jaccard_index():
    """SparseJaccard (0-terminated id lists in dimension+1 float slots,
    Index::makeSparseObject, Index.cpp:304-320): insertion, device ANNG build and
    tree-seeded search equal the oracle over the saved files."""
    rng = np.random.default_rng(0x5A)
    dim, n = 24, 1200
    X = _sparse_rows(rng, n, dim, 60)
    with tempfile.TemporaryDirectory() as tmp:
        ix, prop, srows, offs, ids, tree = _build_via_capi(tmp, dim, "Sparse Jaccard", X)
        assert ix.object_dim == dim + 1
        assert np.array_equal(srows[1:, :dim + 1].view(np.uint32), X.view(np.uint32))
        qs = _sparse_rows(rng, 24, dim, 60)
        gi, gd, gn = ix.batch_search(qs, 10, 0.1)
        es = _edge_size(prop, 0.1)
        for i in range(len(qs)):
            q = np.zeros(srows.shape[1], np.float32)
            q[:dim + 1] = qs[i]
            seeds, _, _ = O.tree_seeds("sparse_jaccard", tree, q, 10, int(prop["SeedSize"]))
            oid, od, _ = O.search("sparse_jaccard", srows, offs, ids, q, seeds, 10, np.float32(0.1), edge_size=es)
            assert list(gi[i, :gn[i]]) == list(oid), i
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32)), i
        ix.close()


def test_concurrent_capi_callers_coalesced():
    """16 threads x single-query ngt_search_index / ngt_linear_search_index on
    one handle (the reference allows concurrent read-only searches,
    Capi.cpp:377-406): every answer equals the reference's, and the calls are
    served by fewer device launches than calls (coalesce.h)."""
    ix = base.Index(os.path.join(GOLD, "c1_anng"))
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    g = np.load(os.path.join(GOLD, "search_c1_anng_tw_0.1.npz"))
    gs = np.load(os.path.join(GOLD, "search_c1_anng_sr_0.0.npz"))
    ix.search(qs[0].astype(np.float64), 10, 0.1)  # warm: device index built
    errors = []
    barrier = threading.Barrier(16)

    def worker(t):
        try:
            barrier.wait()
            for rep in range(4):
                for i in range(t, len(qs), 16):
                    r = ix.search(qs[i].astype(np.float64), 10, 0.1)
                    if [x.id for x in r] != list(g["ids"][i]):
                        errors.append(("search", t, i))
                    if rep == 0:
                        r = ix.linear_search(qs[i].astype(np.float64), 10)
                        if [x.id for x in r] != list(gs["ids"][i]):
                            errors.append(("linear", t, i))
        except Exception as e:  # noqa: BLE001
            errors.append(("exc", t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    L = lib()
    b, s = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.ngt_get_coalesce_stats(ix.index, ctypes.byref(b), ctypes.byref(s), ix.err)
    assert s.value == 1 + 4 * len(qs) + len(qs)
    assert b.value < s.value, (b.value, s.value)
    ix.close()


def test_linear_search_two_streams():
    """The slice buffer of the linear search belongs to (index, stream): two
    streams searching at once give the single-stream results."""
    import torch
    rng = np.random.default_rng(3)
    n, dim, nq, k = 40000, 64, 96, 10
    rows = np.zeros((n, dim), np.float32)
    rows[1:] = rng.random((n - 1, dim), dtype=np.float32)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    dev = torch.device("cuda:0")
    qs = [torch.from_numpy(rng.random((nq, dim), dtype=np.float32)).to(dev) for _ in range(2)]
    outs = [(torch.zeros((nq, k), dtype=torch.int32, device=dev), torch.zeros((nq, k), device=dev),
             torch.zeros((nq,), dtype=torch.int32, device=dev)) for _ in range(2)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    torch.cuda.synchronize()
    for rep in range(3):
        for b in range(2):
            oi, od, on = outs[b]
            ix.linear_search_device(qs[b].data_ptr(), dim * 4, nq, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                                    stream=streams[b].cuda_stream)
    torch.cuda.synchronize()
    for b in range(2):
        ri, rd, rn = ix.linear_search(qs[b].cpu().numpy(), k)
        oi, od, on = outs[b]
        assert np.array_equal(oi.cpu().numpy().view(np.uint32), ri)
        assert np.array_equal(od.cpu().numpy().view(np.uint32), rd.view(np.uint32))
    ix.close()
