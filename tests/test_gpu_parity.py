"""GPU parity: the HIP path (through the C ABI) against the reference's own
outputs (tests/golden) and against the CPU restatement (oracle/).

Bar: bit-exact float distances for the comparators whose reduction order the
oracle pins (all float/uint8 metrics except the query-normalization step);
identical result ids and distances for every search."""
import ctypes
import glob
import os

import numpy as np
import pytest

import ngt_files as F
import oracle_py as O
from ngt_amd import base
from ngt_amd.device import SEED_GIVEN, SEED_RANDOM, SEED_TREE, DeviceIndex

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
QUERIES = None


def queries():
    global QUERIES
    if QUERIES is None:
        QUERIES = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    return QUERIES


def fmt(x):
    return "%g" % float(x)


def load(name):
    d = os.path.join(GOLD, name)
    prop = F.read_prf(os.path.join(d, "prf"))
    rows, valid = F.read_obj(os.path.join(d, "obj"), 128, np.float32)
    offs, ids, _ = F.read_grp(os.path.join(d, "grp"))
    tree = F.read_tre(os.path.join(d, "tre"), 128, np.float32)
    return prop, rows, valid, offs, ids, tree


def device_index(name):
    prop, rows, valid, offs, ids, tree = load(name)
    ix = DeviceIndex("l2", "float", 128)
    ix.set_objects(rows, valid)
    ix.set_graph(offs, ids)
    ix.set_tree(tree)
    ix.set_search_property(int(prop["EdgeSizeForSearch"]), int(prop["DynamicEdgeSizeBase"]),
                           int(prop["DynamicEdgeSizeRate"]), int(prop["SeedSize"]), 0)
    return ix, prop, rows, offs, ids, tree


# ---------------------------------------------------------------------------
# comparators
# ---------------------------------------------------------------------------
def _dist_cases():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLD, "dist_*.npz"))):
        name = os.path.basename(f)[5:-4]
        out.append(pytest.param(f, name.rsplit("_", 2)[0], name.rsplit("_", 2)[1], id=name))
    return out


@pytest.mark.parametrize("path,metric,ot", _dist_cases())
def test_gpu_comparators_bit_exact_vs_reference(path, metric, ot):
    z = np.load(path)
    rows = z["rows"]
    dim = int(z["dim"])
    ix = DeviceIndex(metric, "float" if ot == "f" else "uint8", dim)
    ix.set_objects(rows)
    got = ix.distances(rows, z["src"], z["dst"])
    ref = z["dist"].astype(np.float32)
    if metric in ("poincare", "lorentz"):
        # double sums in an order the reference's -Ofast build chose; tolerance per north_star
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
    else:
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
            np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))[:10]
    ix.close()


# ---------------------------------------------------------------------------
# graph search on the reference-built C1 indexes
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["c1_anng", "c1_onng"])
@pytest.mark.parametrize("eps", ["0.0", "0.02", "0.05", "0.1"])
def test_tree_seeded_search_matches_reference(name, eps):
    ix, prop, rows, offs, ids, tree = device_index(name)
    qs = queries()
    gi, gd, gn, cnt = ix.search(qs, k=10, epsilon=float(eps), seed_mode=SEED_TREE)
    g = np.load(os.path.join(GOLD, "search_%s_tr_%s.npz" % (name, eps)))
    gw = np.load(os.path.join(GOLD, "search_%s_tw_%s.npz" % (name, eps)))
    es = ix.resolve_edge_size(-1, float(eps))
    for i, q in enumerate(qs):
        ref = g["ids"][i][g["ids"][i] >= 0]
        assert list(gi[i, :gn[i]]) == list(ref), i
        assert [fmt(x) for x in gd[i, :gn[i]]] == [fmt(x) for x in g["dists"][i][:gn[i]]], i
        # bit-exact against the restatement, and the same work
        seeds, _, _ = O.tree_seeds("l2", tree, q, 10, int(prop["SeedSize"]))
        oid, od, ocnt = O.search("l2", rows, offs, ids, q, seeds, 10, np.float32(float(eps)), edge_size=es)
        assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32)), i
        assert int(cnt[i, 0]) == int(ocnt[0]), i
        # reference rw-mode distance count excludes the seeds (Graph.cpp:287, :604)
        assert int(cnt[i, 0]) - len(seeds) == int(gw["ndist"][i]), i
    ix.close()


@pytest.mark.parametrize("name", ["c1_anng", "c1_onng"])
def test_k20_search_matches_reference(name):
    ix, *_ = device_index(name)
    gi, gd, gn, _ = ix.search(queries(), k=20, epsilon=0.2, seed_mode=SEED_TREE)
    g = np.load(os.path.join(GOLD, "search_%s_tr_k20_0.2.npz" % name))
    for i in range(len(queries())):
        assert list(gi[i, :gn[i]]) == list(g["ids"][i]), i
    ix.close()


@pytest.mark.parametrize("name", ["c1_anng", "c1_onng"])
@pytest.mark.parametrize("eps", ["0.0", "0.1"])
def test_graph_only_search_matches_reference(name, eps):
    """`ngt search -i g`: random seeds from a fresh process's rand() stream
    (seed 1), one query after another -- in one batch and query by query."""
    from ngt_amd import lib
    ix, *_ = device_index(name)
    lib().ngt_amd_srand(1)
    gi, gd, gn, _ = ix.search(queries(), k=10, epsilon=float(eps), seed_mode=SEED_RANDOM)
    g = np.load(os.path.join(GOLD, "search_%s_gr_%s.npz" % (name, eps)))
    for i in range(len(queries())):
        assert list(gi[i, :gn[i]]) == list(g["ids"][i][g["ids"][i] >= 0]), i
    lib().ngt_amd_srand(1)
    for i in range(len(queries())):
        si, sd, sn, _ = ix.search(queries()[i:i + 1], k=10, epsilon=float(eps), seed_mode=SEED_RANDOM)
        assert list(si[0, :sn[0]]) == list(g["ids"][i][g["ids"][i] >= 0]), i
    ix.close()


@pytest.mark.parametrize("name", ["c1_anng", "c1_onng"])
def test_linear_search_matches_reference(name):
    ix, prop, rows, *_ = device_index(name)
    gi, gd, gn = ix.linear_search(queries(), k=10)
    g = np.load(os.path.join(GOLD, "search_%s_sr_0.0.npz" % name))
    for i in range(len(queries())):
        assert list(gi[i, :gn[i]]) == list(g["ids"][i]), i
        assert [fmt(x) for x in gd[i]] == [fmt(x) for x in g["dists"][i]], i
    ix.close()


def test_capi_single_query_matches_reference():
    """The drop-in ngt_search_index / ngt_linear_search_index path (Capi.cpp:346-483)."""
    ix = base.Index(os.path.join(GOLD, "c1_anng"))
    g = np.load(os.path.join(GOLD, "search_c1_anng_tw_0.1.npz"))
    gs = np.load(os.path.join(GOLD, "search_c1_anng_sr_0.0.npz"))
    for i, q in enumerate(queries()[:20]):
        r = ix.search(q.astype(np.float64), 10, 0.1)
        assert [x.id for x in r] == list(g["ids"][i]), i
        r = ix.linear_search(q.astype(np.float64), 10)
        assert [x.id for x in r] == list(gs["ids"][i]), i
    bi, bd, bn = ix.batch_search(queries(), 10, 0.1)
    for i in range(len(queries())):
        assert list(bi[i, :bn[i]]) == list(g["ids"][i]), i
    ix.close()


# ---------------------------------------------------------------------------
# every metric x object type: GPU search vs the restatement on the small
# reference-built graphs (graph = the grp edge lists stored in dist_*.npz)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("path,metric,ot", _dist_cases())
def test_search_all_metrics_vs_oracle(path, metric, ot):
    z = np.load(path)
    rows = z["rows"]
    dim = int(z["dim"])
    n = rows.shape[0]
    src, dst = z["src"].astype(np.int64), z["dst"]
    offs = np.zeros(n + 1, np.uint64)
    np.add.at(offs, src + 1, 1)
    offs = np.cumsum(offs).astype(np.uint64)
    ix = DeviceIndex(metric, "float" if ot == "f" else "uint8", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, dst)
    rng = np.random.default_rng(7)
    qrows = rows[rng.integers(1, n, 16)].astype(np.float32)[:, :dim]
    if ot == "f" and metric not in ("normalized_angle", "normalized_cosine", "normalized_l2"):
        qrows = qrows * np.float32(1.01)
    seeds = [rng.choice(np.arange(1, n), 5, replace=False).astype(np.uint32) for _ in range(16)]
    gi, gd, gn, cnt = ix.search(qrows, k=10, epsilon=0.1, edge_size=0, seed_mode=SEED_GIVEN, seeds=seeds)
    for i in range(16):
        # the oracle sees the query exactly as the device prepared it
        q = np.zeros(rows.shape[1], rows.dtype)
        q[:dim] = qrows[i] if ot == "f" else qrows[i].astype(np.int64).astype(np.uint8)
        if metric.startswith("normalized") and ot == "f":
            # ObjectSpace::normalize of the query, restated in the device's
            # (and the reference's) 16-lane order: the same prepared row
            qv = np.ascontiguousarray(q[:dim])
            assert O.lib().ngto_normalize_f32(qv.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), dim) == 0
            q[:dim] = qv
        oid, od, ocnt = O.search(metric, rows, offs, dst, q, seeds[i], 10, np.float32(0.1))
        assert list(gi[i, :gn[i]]) == list(oid), (i, metric)
        if metric in ("poincare", "lorentz"):
            np.testing.assert_allclose(gd[i, :gn[i]], od, rtol=1e-5)
        else:
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32)), i
        assert int(cnt[i, 0]) == int(ocnt[0])
    ix.close()


# ---------------------------------------------------------------------------
# exactness of the LDS overflow paths (visited hash -> HBM bitmap, unchecked
# array -> HBM spill) on a synthetic graph, forced with tiny LDS capacities.
# ---------------------------------------------------------------------------
def _random_graph(n, dim, deg, seed):
    rng = np.random.default_rng(seed)
    rows = np.zeros((n, dim), np.float32)
    rows[1:] = rng.random((n - 1, dim), dtype=np.float32)
    # node 0 is the dummy slot with no edges; nodes 1..n-1 have `deg` edges each
    offs = np.zeros(n + 1, np.uint64)
    offs[2:] = np.arange(1, n, dtype=np.uint64) * deg
    edges = rng.integers(1, n, size=(n - 1) * deg).astype(np.uint32)
    # no self loops / duplicates within a list
    e = edges.reshape(n - 1, deg)
    for v in range(1, n):
        row = np.unique(e[v - 1][e[v - 1] != v])
        while len(row) < deg:
            extra = rng.integers(1, n, deg)
            row = np.unique(np.concatenate([row, extra[extra != v]]))[:deg]
        e[v - 1] = row[:deg]
    return rows, offs, e.reshape(-1)


@pytest.mark.parametrize("ht,cq,adj,vf", [("12", "1024", "1", ""), ("8", "64", "1", ""), ("9", "128", "0", ""),
                                          ("bitmap", "1024", "1", ""), ("bitmap", "64", "0", ""),
                                          ("bitmap", "512", "1", "0"), ("bitmap", "512", "1", "11"),
                                          ("8", "64", "1", "11")])
@pytest.mark.parametrize("dim", [32, 128])
def test_overflow_paths_exact(monkeypatch, ht, cq, adj, vf, dim):
    """LDS-overflow forms of the visited and unchecked sets, forced small:
    visited hash -> HBM epochs, the LDS visited filter (default 32 Kbit in the
    epoch mode; vf "0" off, "11" a 2 Kbit filter that saturates, so both its
    proven-fresh and fall-through paths run), unchecked array -> HBM spill."""
    if ht != "bitmap":
        monkeypatch.setenv("NGT_AMD_HT_LOG2", ht)
    if vf:
        monkeypatch.setenv("NGT_AMD_VFILTER", vf)
    monkeypatch.setenv("NGT_AMD_CQ_CAP", cq)
    monkeypatch.setenv("NGT_AMD_ADJ", adj)
    vh = -1 if ht == "bitmap" else 0
    n, deg = 3000, 24
    rows, offs, edges = _random_graph(n, dim, deg, 11)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(3)
    qs = rng.random((24, dim), dtype=np.float32)
    seeds = [rng.choice(np.arange(1, n), 10, replace=False).astype(np.uint32) for _ in range(24)]
    for eps in [0.0, 0.3, 1.0]:  # noqa: B007
        gi, gd, gn, cnt = ix.search(qs, k=20, epsilon=eps, edge_size=0, seed_mode=SEED_GIVEN, seeds=seeds,
                                    visited_hash_log2=vh)
        for i in range(24):
            oid, od, ocnt = O.search("l2", rows, offs, edges, qs[i], seeds[i], 20, np.float32(eps))
            assert list(gi[i, :gn[i]]) == list(oid), (eps, i)
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32))
            assert int(cnt[i, 0]) == int(ocnt[0])
        if ht == "8" and eps == 1.0:
            assert cnt[:, 3].sum() > 0  # the bitmap path really ran
    ix.close()


@pytest.mark.parametrize("cq,vf", [("512", ""), ("64", ""), ("512", "11"), ("64", "11")])
@pytest.mark.parametrize("dim", [32, 128])
def test_accepted_only_visited_exact(monkeypatch, cq, vf, dim):
    """visited_hash_log2 = -2: the HBM epochs and the LDS filter hold only
    accepted ids (seeds and neighbours within the exploration radius); rejected
    neighbours met again are re-evaluated.  Ids and distances must equal the
    restatement's exactly, including negative epsilon (exploration radius
    below the result radius), a finite search radius, HBM spill of the
    unchecked set (cq 64) and a saturated filter (vf 11); evaluations can
    only exceed the reference's distinct distance count."""
    if vf:
        monkeypatch.setenv("NGT_AMD_VFILTER", vf)
    monkeypatch.setenv("NGT_AMD_CQ_CAP", cq)
    n, deg = 3000, 24
    rows, offs, edges = _random_graph(n, dim, deg, 12)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(4)
    qs = rng.random((24, dim), dtype=np.float32)
    seeds = [rng.choice(np.arange(1, n), 10, replace=False).astype(np.uint32) for _ in range(24)]
    radius = float(np.sqrt(dim / 6.0))  # about the median distance of U[0,1) rows
    for eps, rad in [(0.0, -1.0), (0.3, -1.0), (1.0, -1.0), (-0.05, -1.0), (0.2, radius)]:
        gi, gd, gn, cnt = ix.search(qs, k=20, epsilon=eps, radius=rad, edge_size=0, seed_mode=SEED_GIVEN,
                                    seeds=seeds, visited_hash_log2=-2)
        for i in range(24):
            kw = {} if rad < 0 else {"radius": rad}
            oid, od, ocnt = O.search("l2", rows, offs, edges, qs[i], seeds[i], 20, np.float32(eps), **kw)
            assert list(gi[i, :gn[i]]) == list(oid), (eps, rad, i)
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32)), (eps, rad, i)
            assert int(cnt[i, 0]) >= int(ocnt[0])
    ix.close()


def test_accepted_only_visited_reference_index():
    """visited_hash_log2 = -2 on the reference-built C1 ONNG with tree seeds:
    identical to the default visited set, whose results the tests above pin to
    the reference's own (tests/golden/c1_onng)."""
    ix = device_index("c1_onng")[0]
    qs = queries()[:64]
    for eps in [0.0, 0.1]:
        gi, gd, gn, _ = ix.search(qs, k=10, epsilon=eps, seed_mode=SEED_TREE, visited_hash_log2=-2)
        ri, rd, rn, _ = ix.search(qs, k=10, epsilon=eps, seed_mode=SEED_TREE, visited_hash_log2=0)
        assert np.array_equal(gn, rn)
        for i in range(len(qs)):
            assert list(gi[i, :gn[i]]) == list(ri[i, :rn[i]]), (eps, i)
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), rd[i, :rn[i]].view(np.uint32))
    ix.close()


def test_edge_cases():
    rows, offs, edges = _random_graph(500, 16, 8, 5)
    ix = DeviceIndex("l2", "float", 16)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    qs = np.random.default_rng(1).random((4, 16), dtype=np.float32)
    # k larger than the reachable set, empty seed list, tiny radius
    seeds = [np.array([1, 2, 3], np.uint32), np.array([], np.uint32), np.array([5], np.uint32),
             np.array([7, 8], np.uint32)]
    gi, gd, gn, cnt = ix.search(qs, k=600, epsilon=0.1, edge_size=0, seed_mode=SEED_GIVEN, seeds=seeds)
    for i in range(4):
        oid, od, _ = O.search("l2", rows, offs, edges, qs[i], seeds[i], 600, np.float32(0.1))
        assert list(gi[i, :gn[i]]) == list(oid)
    assert gn[1] == 0
    gi, gd, gn, cnt = ix.search(qs, k=5, epsilon=0.1, radius=0.5, edge_size=3, seed_mode=SEED_GIVEN,
                                seeds=seeds)
    for i in range(4):
        oid, od, _ = O.search("l2", rows, offs, edges, qs[i], seeds[i], 5, np.float32(0.1), radius=0.5,
                              edge_size=3)
        assert list(gi[i, :gn[i]]) == list(oid)
    ix.close()


def test_device_api_first_launch_exact():
    """The *_device entry points on the default (NULL) stream: the very first
    launch (which allocates and zeroes the per-slot visited arrays) must already
    be exact, and repeated launches must agree bit for bit."""
    import torch
    n, dim, deg, nq = 60000, 32, 24, 256
    rows, offs, edges = _random_graph(n, dim, deg, 21)
    dev = torch.device("cuda:0")
    d_rows = torch.from_numpy(rows).to(dev)
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_edges = torch.from_numpy(edges.astype(np.int32)).to(dev)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects_device(d_rows.data_ptr(), n)
    ix.set_graph_device(d_offs.data_ptr(), d_edges.data_ptr(), len(edges))
    rng = np.random.default_rng(8)
    qs = rng.random((nq, dim), dtype=np.float32)
    seeds = np.stack([rng.choice(np.arange(1, n), 10, replace=False) for _ in range(nq)]).astype(np.uint32)
    d_q = torch.from_numpy(qs).to(dev)
    d_seeds = torch.from_numpy(seeds.reshape(-1).astype(np.int32)).to(dev)
    d_soff = torch.arange(0, nq + 1, dtype=torch.int64, device=dev) * 10
    outs = []
    for _ in range(3):
        oi = torch.zeros((nq, 10), dtype=torch.int32, device=dev)
        od = torch.zeros((nq, 10), dtype=torch.float32, device=dev)
        on = torch.zeros((nq,), dtype=torch.int32, device=dev)
        cnt = torch.zeros((nq, 8), dtype=torch.int64, device=dev)
        ix.search_device(d_q.data_ptr(), dim * 4, nq, oi.data_ptr(), od.data_ptr(), on.data_ptr(), cnt.data_ptr(),
                         k=10, epsilon=0.3, edge_size=0, seed_mode=SEED_GIVEN, d_seeds=d_seeds.data_ptr(),
                         d_seed_off=d_soff.data_ptr(), stream=None, visited_hash_log2=-1)
        torch.cuda.synchronize()
        outs.append((oi.cpu().numpy().view(np.uint32), od.cpu().numpy(), on.cpu().numpy(), cnt.cpu().numpy()))
    for o in outs[1:]:
        assert np.array_equal(o[0], outs[0][0]) and np.array_equal(o[1].view(np.uint32), outs[0][1].view(np.uint32))
        assert np.array_equal(o[3][:, :3], outs[0][3][:, :3])
    gi, gd, gn, cnt = outs[0]
    for i in range(0, nq, 4):
        oid, od_, ocnt = O.search("l2", rows, offs, edges, qs[i], seeds[i], 10, np.float32(0.3))
        assert list(gi[i, :gn[i]]) == list(oid), i
        assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od_.view(np.uint32))
        assert int(cnt[i, 0]) == int(ocnt[0])
    ix.close()


def test_concurrent_streams_exact():
    """Searches on two HIP streams run concurrently, each with its own launch
    scratch (visited epochs, work counter): results equal the sequential run
    and the oracle."""
    import torch
    n, dim, deg, nq = 30000, 32, 24, 512
    rows, offs, edges = _random_graph(n, dim, deg, 33)
    dev = torch.device("cuda:0")
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(12)
    qs = rng.random((2, nq, dim), dtype=np.float32)
    seeds = np.stack([rng.choice(np.arange(1, n), 10, replace=False) for _ in range(nq)]).astype(np.uint32)
    d_s = torch.from_numpy(seeds.reshape(-1).view(np.int32)).to(dev)
    d_o = torch.arange(0, nq + 1, dtype=torch.int64, device=dev) * 10
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    outs = []
    for b in range(2):
        d_q = torch.from_numpy(qs[b]).to(dev)
        oi = torch.zeros((nq, 10), dtype=torch.int32, device=dev)
        od = torch.zeros((nq, 10), dtype=torch.float32, device=dev)
        on = torch.zeros((nq,), dtype=torch.int32, device=dev)
        outs.append((d_q, oi, od, on))
    torch.cuda.synchronize()
    for rep in range(3):
        for b in range(2):
            d_q, oi, od, on = outs[b]
            ix.search_device(d_q.data_ptr(), dim * 4, nq, oi.data_ptr(), od.data_ptr(), on.data_ptr(), None, k=10,
                             epsilon=0.3, edge_size=0, seed_mode=SEED_GIVEN, d_seeds=d_s.data_ptr(),
                             d_seed_off=d_o.data_ptr(), stream=streams[b].cuda_stream, visited_hash_log2=-1)
    torch.cuda.synchronize()
    for b in range(2):
        _, oi, od, on = outs[b]
        gi, gd, gn = oi.cpu().numpy().view(np.uint32), od.cpu().numpy(), on.cpu().numpy()
        for i in range(0, nq, 8):
            oid, od_, _ = O.search("l2", rows, offs, edges, qs[b][i], seeds[i], 10, np.float32(0.3))
            assert list(gi[i, :gn[i]]) == list(oid), (b, i)
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od_.view(np.uint32))
    ix.close()


@pytest.mark.parametrize("metric", ["l2", "cosine", "angle"])
@pytest.mark.parametrize("dim", [256, 960, 200])
def test_long_rows_stream_exact(metric, dim):
    """Long float rows take the streamed comparator (Dp/16 a multiple of 4:
    256, 960; 200 -> Dp 208 stays on the generic one): same ids, bit-exact
    distances and the same work as the restatement."""
    n, deg, nq = 2500, 16, 24
    rows, offs, edges = _random_graph(n, dim, deg, 17)
    ix = DeviceIndex(metric, "float", dim)
    ix.set_objects(rows)
    ix.set_graph(offs, edges)
    rng = np.random.default_rng(6)
    qs = rng.random((nq, dim), dtype=np.float32)
    seeds = [rng.choice(np.arange(1, n), 10, replace=False).astype(np.uint32) for _ in range(nq)]
    gi, gd, gn, cnt = ix.search(qs, k=10, epsilon=0.2, edge_size=0, seed_mode=SEED_GIVEN, seeds=seeds,
                                visited_hash_log2=-1)
    dp = ((dim - 1) // 16 + 1) * 16
    rp = np.zeros((n, dp), np.float32)
    rp[:, :dim] = rows
    for i in range(nq):
        q = np.zeros(dp, np.float32)
        q[:dim] = qs[i]
        oid, od, ocnt = O.search(metric, rp, offs, edges, q, seeds[i], 10, np.float32(0.2))
        assert list(gi[i, :gn[i]]) == list(oid), (metric, dim, i)
        assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32)), (metric, dim, i)
        assert int(cnt[i, 0]) == int(ocnt[0])
    ix.close()
