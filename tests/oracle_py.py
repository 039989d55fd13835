"""ctypes binding of the CPU restatement in oracle/ (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = None

METRICS = {
    "l1": 0, "l2": 1, "hamming": 2, "angle": 3, "cosine": 4, "normalized_angle": 5,
    "normalized_cosine": 6, "jaccard": 7, "sparse_jaccard": 8, "normalized_l2": 9,
    "poincare": 100, "lorentz": 101,
}
OTYPES = {"c": 1, "u8": 1, "f": 2, "f32": 2}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ROOT, "oracle", "libngt_oracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(path)
        vp, sz, u32p, f32p, u64p = (ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_uint32),
                                    ctypes.POINTER(ctypes.c_float),
                                    ctypes.POINTER(ctypes.c_uint64))
        L.ngto_distance.restype = ctypes.c_float
        L.ngto_distance.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz]
        L.ngto_distances.restype = None
        L.ngto_distances.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz, u32p, sz, sz, f32p]
        L.ngto_search.restype = ctypes.c_int
        L.ngto_search.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, sz, sz, u64p, u32p, vp,
                                  u32p, sz, sz, ctypes.c_float, ctypes.c_float, sz, u32p, f32p, u64p]
        L.ngto_linear_search.restype = ctypes.c_int
        L.ngto_linear_search.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, sz, sz, vp, vp, sz,
                                         ctypes.c_double, u32p, f32p]
        L.ngto_thin_seeds.restype = sz
        L.ngto_thin_seeds.argtypes = [u32p, sz, ctypes.c_uint, sz, sz]
        L.ngto_tree_leaf.restype = ctypes.c_uint32
        L.ngto_tree_leaf.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, ctypes.c_uint32, vp, sz,
                                     u32p, f32p, sz, u64p]
        L.ngto_normalize_f32.restype = ctypes.c_int
        L.ngto_normalize_f32.argtypes = [f32p, sz]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def distances(metric, rows, query, ids):
    """Reference comparator distances between `query` and rows[ids]."""
    rows = np.ascontiguousarray(rows)
    query = np.ascontiguousarray(query, dtype=rows.dtype)
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    out = np.zeros(len(ids), np.float32)
    ot = 2 if rows.dtype == np.float32 else 1
    lib().ngto_distances(METRICS[metric], ot, query.ctypes.data, rows.ctypes.data,
                         rows.strides[0], _p(ids, ctypes.c_uint32), len(ids), rows.shape[1],
                         _p(out, ctypes.c_float))
    return out


def pair_distances(metric, rows, src, dst):
    rows = np.ascontiguousarray(rows)
    ot = 2 if rows.dtype == np.float32 else 1
    L = lib()
    out = np.empty(len(src), np.float32)
    rb = rows.strides[0]
    base = rows.ctypes.data
    m = METRICS[metric]
    for i, (s, d) in enumerate(zip(src, dst)):
        out[i] = L.ngto_distance(m, ot, base + int(s) * rb, base + int(d) * rb, rows.shape[1])
    return out


def search(metric, rows, offsets, edges, query, seeds, k, epsilon, radius=3.402823466e38,
           edge_size=0):
    rows = np.ascontiguousarray(rows)
    ot = 2 if rows.dtype == np.float32 else 1
    query = np.ascontiguousarray(query, dtype=rows.dtype)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    edges = np.ascontiguousarray(edges, dtype=np.uint32)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
    ids = np.zeros(max(k, 1), np.uint32)
    ds = np.zeros(max(k, 1), np.float32)
    cnt = np.zeros(3, np.uint64)
    n = lib().ngto_search(METRICS[metric], ot, rows.ctypes.data, rows.strides[0], rows.shape[0],
                          rows.shape[1], _p(offsets, ctypes.c_uint64), _p(edges, ctypes.c_uint32),
                          query.ctypes.data, _p(seeds, ctypes.c_uint32), len(seeds), k,
                          epsilon, radius, edge_size, _p(ids, ctypes.c_uint32),
                          _p(ds, ctypes.c_float), _p(cnt, ctypes.c_uint64))
    return ids[:n].copy(), ds[:n].copy(), cnt


def linear_search(metric, rows, query, k, valid=None, radius=-1.0):
    rows = np.ascontiguousarray(rows)
    ot = 2 if rows.dtype == np.float32 else 1
    query = np.ascontiguousarray(query, dtype=rows.dtype)
    ids = np.zeros(max(k, 1), np.uint32)
    ds = np.zeros(max(k, 1), np.float32)
    vptr = None
    if valid is not None:
        valid = np.ascontiguousarray(valid, dtype=np.uint8)
        vptr = valid.ctypes.data
    n = lib().ngto_linear_search(METRICS[metric], ot, rows.ctypes.data, rows.strides[0],
                                 rows.shape[0], rows.shape[1], vptr, query.ctypes.data, k, radius,
                                 _p(ids, ctypes.c_uint32), _p(ds, ctypes.c_float))
    return ids[:n].copy(), ds[:n].copy()


def tree_seeds(metric, tree, query, k, seed_size=10, dtype=np.float32):
    """getSeedsFromTree (lib/NGT/Index.h:1524-1567) on a parsed tre dict."""
    query = np.ascontiguousarray(query, dtype=dtype)
    piv = np.ascontiguousarray(tree["in_pivot"])
    child = np.ascontiguousarray(tree["in_child"], dtype=np.uint32)
    border = np.ascontiguousarray(tree["in_border"], dtype=np.float32)
    nd = np.zeros(1, np.uint64)
    ot = 2 if piv.dtype == np.float32 else 1
    leaf = lib().ngto_tree_leaf(METRICS[metric], ot, query.ctypes.data, piv.shape[1], tree["root"],
                                piv.ctypes.data, piv.strides[0], _p(child, ctypes.c_uint32),
                                _p(border, ctypes.c_float), 5, _p(nd, ctypes.c_uint64))
    lid = leaf & 0x7FFFFFFF
    b, e = int(tree["leaf_off"][lid]), int(tree["leaf_off"][lid + 1])
    seeds = np.ascontiguousarray(tree["leaf_ids"][b:e], dtype=np.uint32).copy()
    n = lib().ngto_thin_seeds(_p(seeds, ctypes.c_uint32), len(seeds), lid, seed_size, k)
    return seeds[:n].copy(), int(nd[0]), lid


def _qg_sigs(L):
    if getattr(L, "_qg", False):
        return
    vp, sz, u8p, u32p, f32p, u64p = (ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint8),
                                     ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_float),
                                     ctypes.POINTER(ctypes.c_uint64))
    L.ngto_qg_lut.restype = None
    L.ngto_qg_lut.argtypes = [f32p, f32p, f32p, sz, sz, u8p, f32p, f32p]
    L.ngto_qg_adc.restype = None
    L.ngto_qg_adc.argtypes = [u8p, sz, u8p, sz, ctypes.c_float, ctypes.c_float, f32p]
    L.ngto_qg_search.restype = ctypes.c_int
    L.ngto_qg_search.argtypes = [f32p, sz, sz, u64p, u32p, u64p, u8p, sz, u8p, ctypes.c_float, ctypes.c_float,
                                 f32p, u32p, sz, sz, ctypes.c_float, ctypes.c_float, ctypes.c_float, u32p, f32p,
                                 u64p]
    L._qg = True


def qg_lut(qg, query):
    """createDistanceLookup (NGTQ/Quantizer.h:709-760) -> (lut, scale, totalOffset)."""
    L = lib()
    _qg_sigs(L)
    M = qg["M"]
    me = (M + 1) // 2 * 2
    q = np.ascontiguousarray(query[:qg["dim"]], dtype=np.float32)
    g = np.ascontiguousarray(qg["global"][:qg["dim"]], dtype=np.float32)
    loc = np.ascontiguousarray(qg["local"], dtype=np.float32)
    lut = np.zeros(me * 16, np.uint8)
    sc = np.zeros(1, np.float32)
    to = np.zeros(1, np.float32)
    L.ngto_qg_lut(_p(q, ctypes.c_float), _p(g, ctypes.c_float), _p(loc, ctypes.c_float), M, qg["dsub"],
                  _p(lut, ctypes.c_uint8), _p(sc, ctypes.c_float), _p(to, ctypes.c_float))
    return lut, sc[0], to[0]


def qg_adc(qg, node, lut, scale, total):
    L = lib()
    _qg_sigs(L)
    a, b = int(qg["qoff"][node]), int(qg["qoff"][node + 1])
    codes = np.ascontiguousarray(qg["codes"][int(qg["code_off"][node]):int(qg["code_off"][node + 1])])
    out = np.zeros(max(b - a, 1), np.float32)
    L.ngto_qg_adc(_p(codes, ctypes.c_uint8), b - a, _p(np.ascontiguousarray(lut), ctypes.c_uint8), qg["M"],
                  scale, total, _p(out, ctypes.c_float))
    return out[:b - a]


def qg_search(qg, rows, query, seeds, k, epsilon, expansion, radius=3.402823466e38):
    """NGTQG::Index::searchQuantizedGraph (QuantizedGraph.h:192-320)."""
    L = lib()
    _qg_sigs(L)
    rows = np.ascontiguousarray(rows, dtype=np.float32)
    dp = rows.shape[1]
    q = np.zeros(dp, np.float32)
    q[:len(query)] = query
    lut, sc, to = qg_lut(qg, q)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
    cap = max(k, int(k * expansion) + 1, 1)
    ids = np.zeros(cap, np.uint32)
    ds = np.zeros(cap, np.float32)
    cnt = np.zeros(4, np.uint64)
    n = L.ngto_qg_search(_p(rows, ctypes.c_float), dp, rows.shape[0], _p(qg["qoff"], ctypes.c_uint64),
                         _p(qg["qids"], ctypes.c_uint32), _p(qg["code_off"], ctypes.c_uint64),
                         _p(qg["codes"], ctypes.c_uint8), qg["M"], _p(lut, ctypes.c_uint8), sc, to,
                         _p(q, ctypes.c_float), _p(seeds, ctypes.c_uint32), len(seeds), k, epsilon, expansion,
                         radius, _p(ids, ctypes.c_uint32), _p(ds, ctypes.c_float), _p(cnt, ctypes.c_uint64))
    return ids[:n].copy(), ds[:n].copy(), cnt


# ---------------------------------------------------------------------------
# Native (vectorized, OpenMP) builds of the same restatement: bench.py's
# cpu_baseline and parity sample.  x86-64-v4 (AVX-512) when the host has it,
# else v3 (AVX2).
# ---------------------------------------------------------------------------
_NATIVE = {}


def host_isa():
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return "v3"
    return "v4" if (" avx512f" in flags and " avx512bw" in flags and " avx512vl" in flags
                    and " avx512dq" in flags) else "v3"


def native_lib(isa=None):
    isa = isa or host_isa()
    if isa not in _NATIVE:
        path = os.path.join(ROOT, "oracle", "libngt_oracle_%s.so" % isa)
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(path)
        vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        f32 = ctypes.c_float
        L.ngto_search_batch.restype = None
        L.ngto_search_batch.argtypes = [i32, i32, vp, sz, sz, sz, vp, vp, vp, sz, sz, vp, vp, sz, f32, f32, sz,
                                        vp, vp, vp, vp, i32]
        L.ngto_linear_search_batch.restype = None
        L.ngto_linear_search_batch.argtypes = [i32, i32, vp, sz, sz, sz, vp, sz, sz, sz, ctypes.c_double, vp, vp,
                                               vp, i32]
        L.ngto_qg_search_batch.restype = None
        L.ngto_qg_search_batch.argtypes = [vp, sz, sz, vp, vp, vp, vp, sz, vp, sz, vp, vp, vp, sz, vp, vp, sz, f32,
                                           f32, f32, sz, vp, vp, vp, vp, i32]
        _NATIVE[isa] = L
    return _NATIVE[isa]


def search_batch(metric, rows, offsets, edges, queries, seeds, k, epsilon, radius=3.402823466e38, edge_size=0,
                 threads=1, L=None):
    """ngto_search over a batch: queries [nq, dp] (rows' dtype), seeds [nq, s]
    or a list.  Returns ids [nq, k], dists [nq, k], n [nq], counters [nq, 3]."""
    L = L or native_lib()
    rows = np.ascontiguousarray(rows)
    queries = np.ascontiguousarray(queries, dtype=rows.dtype)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    edges = np.ascontiguousarray(edges, dtype=np.uint32)
    nq = queries.shape[0]
    if isinstance(seeds, np.ndarray) and seeds.ndim == 2:
        so = np.arange(nq + 1, dtype=np.uint64) * np.uint64(seeds.shape[1])
        sp = np.ascontiguousarray(seeds, dtype=np.uint32).reshape(-1)
    else:
        so = np.zeros(nq + 1, np.uint64)
        so[1:] = np.cumsum([len(s) for s in seeds])
        sp = np.ascontiguousarray(np.concatenate([np.asarray(s, np.uint32) for s in seeds]), dtype=np.uint32)
    ids = np.zeros((nq, k), np.uint32)
    ds = np.zeros((nq, k), np.float32)
    n = np.zeros(nq, np.uint32)
    cnt = np.zeros((nq, 3), np.uint64)
    ot = 2 if rows.dtype == np.float32 else 1
    L.ngto_search_batch(METRICS[metric], ot, rows.ctypes.data, rows.strides[0], rows.shape[0], rows.shape[1],
                        offsets.ctypes.data, edges.ctypes.data, queries.ctypes.data, queries.strides[0], nq,
                        sp.ctypes.data, so.ctypes.data, k, epsilon, radius, edge_size, ids.ctypes.data,
                        ds.ctypes.data, n.ctypes.data, cnt.ctypes.data, threads)
    return ids, ds, n, cnt


def linear_search_batch(metric, rows, queries, k, radius=-1.0, threads=1, L=None):
    L = L or native_lib()
    rows = np.ascontiguousarray(rows)
    queries = np.ascontiguousarray(queries, dtype=rows.dtype)
    nq = queries.shape[0]
    ids = np.zeros((nq, k), np.uint32)
    ds = np.zeros((nq, k), np.float32)
    n = np.zeros(nq, np.uint32)
    ot = 2 if rows.dtype == np.float32 else 1
    L.ngto_linear_search_batch(METRICS[metric], ot, rows.ctypes.data, rows.strides[0], rows.shape[0],
                               rows.shape[1], queries.ctypes.data, queries.strides[0], nq, k, radius,
                               ids.ctypes.data, ds.ctypes.data, n.ctypes.data, threads)
    return ids, ds, n


def qg_search_batch(qg, rows, queries, seeds, k, epsilon, expansion, luts, scales, offsets,
                    radius=3.402823466e38, threads=1, L=None):
    """ngto_qg_search over a batch (qg: dict of qoff/qids/code_off/codes/M as in
    qg_search).  Returns ids/dists [nq, stride], n [nq], counters [nq, 4]."""
    L = L or native_lib()
    rows = np.ascontiguousarray(rows, dtype=np.float32)
    queries = np.ascontiguousarray(queries, dtype=np.float32)
    nq = queries.shape[0]
    if isinstance(seeds, np.ndarray) and seeds.ndim == 2:
        so = np.arange(nq + 1, dtype=np.uint64) * np.uint64(seeds.shape[1])
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32).reshape(-1)
    else:  # ragged lists (tree seeds)
        so = np.zeros(nq + 1, np.uint64)
        so[1:] = np.cumsum([len(s) for s in seeds])
        seeds = np.ascontiguousarray(np.concatenate([np.asarray(s, np.uint32) for s in seeds]), dtype=np.uint32)
    stride = max(k, int(k * expansion) + 1)
    ids = np.zeros((nq, stride), np.uint32)
    ds = np.zeros((nq, stride), np.float32)
    n = np.zeros(nq, np.uint32)
    cnt = np.zeros((nq, 4), np.uint64)
    luts = np.ascontiguousarray(luts, dtype=np.uint8)
    scales = np.ascontiguousarray(scales, dtype=np.float32)
    offsets = np.ascontiguousarray(offsets, dtype=np.float32)
    L.ngto_qg_search_batch(rows.ctypes.data, rows.shape[1], rows.shape[0], qg["qoff"].ctypes.data,
                           qg["qids"].ctypes.data, qg["code_off"].ctypes.data, qg["codes"].ctypes.data, qg["M"],
                           luts.ctypes.data, luts.shape[1], scales.ctypes.data, offsets.ctypes.data,
                           queries.ctypes.data, nq, seeds.ctypes.data, so.ctypes.data, k, epsilon, expansion,
                           radius, stride, ids.ctypes.data, ds.ctypes.data, n.ctypes.data, cnt.ctypes.data, threads)
    return ids, ds, n, cnt


# ---------------------------------------------------------------------------
# NGTQ IVF-ADC (lib/NGT/NGTQ/Quantizer.h:2471-2549)
# ---------------------------------------------------------------------------
NGTQ_MODES = {"a": 0, "l": 1, "c": 2, "r": 3, "e": 4}


def load_ngtq(index_dir, objects):
    """An NGTQ index directory (ngtq create) as arrays: global codebook rows /
    graph / tree / property, local [N, 17, dsub], inverted lists in CSR
    (list_off by global id, eids, elids [E, N]) and the object list
    `objects` [records, dim] (record 0 unused)."""
    import ngt_files as F
    prop = F.read_prf(os.path.join(index_dir, "prf"))
    dim, N = int(prop["Dimension"]), int(prop["LocalDivisionNo"])
    dsub = dim // N
    G, _ = F.read_obj(os.path.join(index_dir, "global", "obj"), dim, np.float32)
    goffs, gids, _ = F.read_grp(os.path.join(index_dir, "global", "grp"))
    gtree = F.read_tre(os.path.join(index_dir, "global", "tre"), dim, np.float32)
    gprop = F.read_prf(os.path.join(index_dir, "global", "prf"))
    local = np.stack([F.read_obj(os.path.join(index_dir, "local-%d" % i, "obj"), dsub, np.float32)[0][:17, :dsub]
                      for i in range(N)])
    ents = F.read_ivt(os.path.join(index_dir, "ivt"))
    nlists = min(max(ents) + 1, G.shape[0]) if ents else 1
    list_off = np.zeros(nlists + 1, np.uint64)
    eids, elids = [], []
    for gid in range(nlists):
        if gid in ents:
            eids.append(ents[gid][0])
            elids.append(ents[gid][1][:, :N])
        list_off[gid + 1] = list_off[gid] + (len(ents[gid][0]) if gid in ents else 0)
    dp = G.shape[1]
    orows = np.zeros((objects.shape[0], dp), np.float32)
    orows[:, :dim] = objects[:, :dim]
    return {"dim": dim, "N": N, "dsub": dsub, "G": G, "goffs": goffs, "gids": gids, "gtree": gtree,
            "gprop": gprop, "local": np.ascontiguousarray(local, np.float32), "list_off": list_off,
            "eids": np.concatenate(eids).astype(np.uint32) if eids else np.zeros(0, np.uint32),
            "elids": np.ascontiguousarray(np.concatenate(elids), np.uint16) if elids else np.zeros((0, N), np.uint16),
            "orows": orows}


def ngtq_search(st, query, mode, size, expansion, epsilon):
    """NGTQ::Index::search(object, objs, size, expansion, mode, epsilon)
    (Quantizer.h:2877-2883 -> :2471-2549); epsilon None = linear
    global-codebook search (the CLI's '-e -')."""
    L = lib()
    if not getattr(L, "_ngtq", False):
        L.ngto_ngtq_aggregate.restype = ctypes.c_size_t
        L.ngto_ngtq_aggregate.argtypes = [ctypes.c_int] + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                          ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        L._ngtq = True
    G = st["G"]
    dp = G.shape[1]
    q = np.zeros(dp, np.float32)
    q[:len(query)] = query
    ass = int(np.float32(size) * np.float32(expansion))
    cbs = ass // (st["orows"].shape[0] // G.shape[0]) + 1
    if epsilon is None:
        cids, cds = linear_search("l2", G, q, cbs)
    else:
        seeds, _, _ = tree_seeds("l2", st["gtree"], q, cbs, int(st["gprop"]["SeedSize"]))
        cids, cds, _ = search("l2", G, st["goffs"], st["gids"], q, seeds, cbs, np.float32(epsilon),
                              edge_size=int(st["gprop"]["EdgeSizeForSearch"]))
    cids = np.ascontiguousarray(cids, np.uint32)
    cds = np.ascontiguousarray(cds, np.float32)
    out_i = np.zeros(size, np.uint32)
    out_d = np.zeros(size, np.float32)
    c = lambda a: a.ctypes.data
    n = L.ngto_ngtq_aggregate(NGTQ_MODES[mode], c(q), dp, c(cids), c(cds), len(cids), c(G), c(st["local"]), st["N"],
                              st["dsub"], c(st["list_off"]), len(st["list_off"]) - 1, c(st["eids"]), c(st["elids"]),
                              c(st["orows"]), size, ass, c(out_i), c(out_d))
    return out_i[:n].copy(), out_d[:n].copy()


def ngtq_term(mode, o, g, l):
    """One residual term (ngto_ngtq_term): mode 'l' float LUT entry, 'a' / 'c'
    per-subspace double."""
    L = lib()
    L.ngto_ngtq_term.restype = ctypes.c_double
    L.ngto_ngtq_term.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    a = [np.ascontiguousarray(x, np.float32) for x in (o, g, l)]
    return L.ngto_ngtq_term(NGTQ_MODES[mode], a[0].ctypes.data, a[1].ctypes.data, a[2].ctypes.data, len(a[0]))
