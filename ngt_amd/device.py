"""Thin wrapper over the batched C ABI of include/ngt_amd.h.

``DeviceIndex`` holds an index resident in HBM (padded row-major object slab,
CSR adjacency, optional DVP tree) and exposes the batched hot path:
``search`` (best-first graph search), ``linear_search`` and ``distances``.
Host arrays are numpy; the ``*_device`` forms take raw device pointers (e.g.
``torch.Tensor.data_ptr()`` of tensors on ``cuda:N``) and a HIP stream handle.
"""
import ctypes
from ctypes import byref, c_void_p

import numpy as np

from . import NativeError, lib
from ._sigs import QgSearchParams, SearchParams

DISTANCE = {
    "l1": 0, "l2": 1, "hamming": 2, "angle": 3, "cosine": 4, "normalized_angle": 5,
    "normalized_cosine": 6, "jaccard": 7, "sparse_jaccard": 8, "normalized_l2": 9,
    "poincare": 100, "lorentz": 101,
}
SEED_TREE, SEED_GIVEN, SEED_RANDOM = 0, 1, 2
COUNTERS = 8


def padded_dim(dim):
    return ((dim - 1) // 16 + 1) * 16


def _chk(rc):
    if rc != 0:
        raise NativeError(lib().ngt_amd_last_error().decode())


def _ptr(a):
    return a.ctypes.data if a is not None else None


class DeviceIndex(object):
    def __init__(self, distance="l2", object_type="float", dim=128, device=0):
        self.L = lib()
        self.metric = DISTANCE[distance] if isinstance(distance, str) else int(distance)
        self.otype = 2 if object_type in ("float", "f", 2) else 1
        self.dtype = np.float32 if self.otype == 2 else np.uint8
        self.dim = dim
        self.dp = padded_dim(dim)
        h = c_void_p()
        _chk(self.L.ngt_amd_index_create(byref(h), device, self.metric, self.otype, dim))
        self.h = h
        self.nrows = 0

    @classmethod
    def wrap(cls, handle, distance="l2", object_type="float", dim=128, nrows=0):
        """A non-owning view of an existing ngt_amd_index (e.g. the one a C-API
        handle serves its searches from, ngt_get_device_index)."""
        self = cls.__new__(cls)
        self.L = lib()
        self.metric = DISTANCE[distance] if isinstance(distance, str) else int(distance)
        self.otype = 2 if object_type in ("float", "f", 2) else 1
        self.dtype = np.float32 if self.otype == 2 else np.uint8
        self.dim = dim
        self.dp = padded_dim(dim)
        self.h = c_void_p(handle)
        self.nrows = nrows
        self._borrowed = True
        return self

    # ---- data -------------------------------------------------------------
    def set_objects(self, rows, valid=None):
        """rows: [nrows, dim or padded dim] with row 0 the dummy slot."""
        rows = np.asarray(rows, dtype=self.dtype)
        if rows.shape[1] != self.dp:
            p = np.zeros((rows.shape[0], self.dp), self.dtype)
            p[:, :rows.shape[1]] = rows
            rows = p
        rows = np.ascontiguousarray(rows)
        v = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
        _chk(self.L.ngt_amd_index_set_objects(self.h, rows.ctypes.data, rows.shape[0], _ptr(v)))
        self.nrows = rows.shape[0]

    def set_objects_device(self, d_rows, nrows):
        _chk(self.L.ngt_amd_index_set_objects_device(self.h, d_rows, nrows))
        self.nrows = nrows

    def set_graph(self, offsets, edges):
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        edges = np.ascontiguousarray(edges, dtype=np.uint32)
        _chk(self.L.ngt_amd_index_set_graph(self.h, offsets.ctypes.data, edges.ctypes.data, len(edges)))

    def set_graph_device(self, d_offsets, d_edges, nedges):
        _chk(self.L.ngt_amd_index_set_graph_device(self.h, d_offsets, d_edges, nedges))

    def set_tree(self, tree):
        piv = np.ascontiguousarray(tree["in_pivot"], dtype=self.dtype)
        if piv.shape[1] != self.dp:
            p = np.zeros((piv.shape[0], self.dp), self.dtype)
            p[:, :piv.shape[1]] = piv
            piv = p
        child = np.ascontiguousarray(tree["in_child"], dtype=np.uint32)
        border = np.ascontiguousarray(tree["in_border"], dtype=np.float32)
        loff = np.ascontiguousarray(tree["leaf_off"], dtype=np.uint64)
        lids = np.ascontiguousarray(tree["leaf_ids"], dtype=np.uint32)
        _chk(self.L.ngt_amd_index_set_tree(self.h, piv.ctypes.data, piv.shape[0], child.ctypes.data,
                                           border.ctypes.data, child.shape[1], int(tree["root"]),
                                           loff.ctypes.data, len(loff) - 1, lids.ctypes.data, len(lids)))

    def set_search_property(self, edge_size_for_search=0, dynamic_edge_size_base=30,
                            dynamic_edge_size_rate=20, seed_size=10, seed_type=0):
        _chk(self.L.ngt_amd_index_set_search_property(self.h, edge_size_for_search, dynamic_edge_size_base,
                                                      dynamic_edge_size_rate, seed_size, seed_type))

    def resolve_edge_size(self, edge_size, epsilon):
        return int(self.L.ngt_amd_resolve_edge_size(self.h, edge_size, epsilon))

    # ---- hot path -----------------------------------------------------------
    def search(self, queries, k=10, epsilon=0.1, radius=-1.0, edge_size=-1, seed_mode=SEED_TREE,
               seeds=None, counters=True, visited_hash_log2=0, distance_filter=0):
        """queries: [nq, dim] float.  seeds: list of arrays for SEED_GIVEN."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        nq = q.shape[0]
        prm = SearchParams(k, epsilon, radius, edge_size, seed_mode, 0, visited_hash_log2, distance_filter)
        ids = np.zeros((nq, k), np.uint32)
        ds = np.zeros((nq, k), np.float32)
        n = np.zeros(nq, np.uint32)
        cnt = np.zeros((nq, COUNTERS), np.uint64) if counters else None
        sp = so = None
        if seed_mode == SEED_GIVEN:
            so = np.zeros(nq + 1, np.uint64)
            so[1:] = np.cumsum([len(s) for s in seeds])
            sp = np.ascontiguousarray(np.concatenate([np.asarray(s, np.uint32) for s in seeds])
                                      if so[-1] else np.zeros(1, np.uint32))
        _chk(self.L.ngt_amd_search(self.h, byref(prm), q.ctypes.data, nq, _ptr(sp), _ptr(so), ids.ctypes.data,
                                   ds.ctypes.data, n.ctypes.data, _ptr(cnt)))
        return ids, ds, n, cnt

    def search_served(self, query, k=10, epsilon=0.1, radius=-1.0, edge_size=-1, seed_mode=SEED_TREE):
        """One query through the resident serving grid (serve.cpp); None when
        the grid does not serve this index/request (ngt_amd_search_served = 1)."""
        q = np.ascontiguousarray(query, dtype=np.float32).reshape(-1)
        prm = SearchParams(k, epsilon, radius, edge_size, seed_mode, 0, 0, 0)
        ids = np.zeros(k, np.uint32)
        ds = np.zeros(k, np.float32)
        n = ctypes.c_uint32()
        cnt = np.zeros(COUNTERS, np.uint64)
        rc = self.L.ngt_amd_search_served(self.h, byref(prm), q.ctypes.data, ids.ctypes.data, ds.ctypes.data,
                                          byref(n), cnt.ctypes.data)
        if rc == 1:
            return None
        _chk(rc)
        return ids[:n.value], ds[:n.value], cnt

    def serve_stop(self):
        _chk(self.L.ngt_amd_serve_stop(self.h))

    def serve_stats(self):
        """(queries the serving grid answered, grids launched)."""
        s, l = ctypes.c_uint64(), ctypes.c_uint64()
        _chk(self.L.ngt_amd_serve_stats(self.h, byref(s), byref(l)))
        return s.value, l.value

    def search_device(self, d_queries, query_bytes, nq, d_ids, d_dists, d_n, d_counters=None, k=10,
                      epsilon=0.1, radius=-1.0, edge_size=-1, seed_mode=SEED_TREE, d_seeds=None,
                      d_seed_off=None, stream=None, visited_hash_log2=0, distance_filter=0):
        prm = SearchParams(k, epsilon, radius, edge_size, seed_mode, 0, visited_hash_log2, distance_filter)
        _chk(self.L.ngt_amd_search_device(self.h, byref(prm), d_queries, query_bytes, nq, d_seeds, d_seed_off,
                                          d_ids, d_dists, d_n, d_counters, stream))

    def last_search_kernel_ms(self):
        return float(self.L.ngt_amd_last_search_kernel_ms(self.h))

    def last_search_filtered(self):
        """True if the last graph search read the 1-byte filter copy (counters
        [6]: exact neighbour distances, [7]: seed distances)."""
        return bool(self.L.ngt_amd_last_search_filtered(self.h))

    def last_search_lookahead(self):
        """Form of the latest graph-search launch: -1 one expansion per pop,
        0 lookahead with a wave per query, 1 lookahead with eight waves per query."""
        return int(self.L.ngt_amd_last_search_lookahead(self.h))

    def last_search_budget(self):
        """0: the last search ran as one launch in query order; B > 0: probe
        launch (every query paused after B expansions) + resume launch,
        longest predicted first (ngt_amd_last_search_budget)."""
        return int(self.L.ngt_amd_last_search_budget(self.h))

    def last_search_slots(self):
        """Workgroups (resident query slots) of the last search launch."""
        return int(self.L.ngt_amd_last_search_slots(self.h))

    def prepare_queries_device(self, d_in, nq, d_out, stream=None):
        _chk(self.L.ngt_amd_prepare_queries_device(self.h, d_in, nq, d_out, stream))

    def linear_search(self, queries, k=10, radius=-1.0):
        q = np.ascontiguousarray(queries, dtype=np.float32)
        nq = q.shape[0]
        ids = np.zeros((nq, k), np.uint32)
        ds = np.zeros((nq, k), np.float32)
        n = np.zeros(nq, np.uint32)
        _chk(self.L.ngt_amd_linear_search(self.h, q.ctypes.data, nq, k, radius, ids.ctypes.data, ds.ctypes.data,
                                          n.ctypes.data))
        return ids, ds, n

    def linear_search_device(self, d_queries, query_bytes, nq, k, d_ids, d_dists, d_n, radius=-1.0,
                             stream=None):
        _chk(self.L.ngt_amd_linear_search_device(self.h, d_queries, query_bytes, nq, k, radius, d_ids, d_dists,
                                                 d_n, stream))

    def distances(self, queries, qidx, oid):
        """queries: prepared rows [nq, dim or dp] of the object type."""
        q = np.asarray(queries, dtype=self.dtype)
        if q.shape[1] != self.dp:
            p = np.zeros((q.shape[0], self.dp), self.dtype)
            p[:, :q.shape[1]] = q
            q = p
        q = np.ascontiguousarray(q)
        qidx = np.ascontiguousarray(qidx, dtype=np.uint32)
        oid = np.ascontiguousarray(oid, dtype=np.uint32)
        out = np.zeros(len(oid), np.float32)
        _chk(self.L.ngt_amd_distances(self.h, q.ctypes.data, q.shape[0], qidx.ctypes.data, oid.ctypes.data,
                                      len(oid), out.ctypes.data))
        return out

    # ---- ANNG construction (GraphAndTreeIndex::createIndex) -----------------
    def build_anng(self, first_id=1, end_id=None, edge_size_for_creation=10, edge_size_for_search=40,
                   batch_size_for_creation=200, seed_size=10, epsilon_for_creation=0.1, begin=True):
        """Build the ANNG + DVP tree of the objects on the device; returns
        (offsets, ids, dists) of the graph and the tree dict (read_tre layout)."""
        from ._sigs import BuildParams
        if begin:
            prm = BuildParams(edge_size_for_creation, edge_size_for_search, batch_size_for_creation, seed_size,
                              epsilon_for_creation, 0)
            _chk(self.L.ngt_amd_build_begin(self.h, byref(prm)))
        _chk(self.L.ngt_amd_build_insert(self.h, first_id, self.nrows if end_id is None else end_id))
        return self.build_graph(), self.build_tree()

    def build_graph(self):
        gs, ne = ctypes.c_uint64(), ctypes.c_uint64()
        _chk(self.L.ngt_amd_build_graph_size(self.h, byref(gs), byref(ne)))
        offs = np.zeros(gs.value + 1, np.uint64)
        ids = np.zeros(max(ne.value, 1), np.uint32)
        ds = np.zeros(max(ne.value, 1), np.float32)
        _chk(self.L.ngt_amd_build_get_graph(self.h, offs.ctypes.data, ids.ctypes.data, ds.ctypes.data))
        return offs, ids[:ne.value], ds[:ne.value]

    def build_tree(self):
        nl, ni, nli = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
        _chk(self.L.ngt_amd_build_tree_size(self.h, byref(nl), byref(ni), byref(nli)))
        nl, ni, nli = nl.value, ni.value, nli.value
        t = {"leaf_parent": np.zeros(nl, np.uint32), "leaf_off": np.zeros(nl + 1, np.uint64),
             "leaf_ids": np.zeros(max(nli, 1), np.uint32), "leaf_dists": np.zeros(max(nli, 1), np.float32),
             "leaf_has_pivot": np.zeros(nl, np.uint8), "leaf_pivot": np.zeros((nl, self.dp), self.dtype),
             "in_parent": np.zeros(ni, np.uint32), "in_pivot": np.zeros((ni, self.dp), self.dtype),
             "in_child": np.zeros((ni, 5), np.uint32), "in_border": np.zeros((ni, 4), np.float32)}
        _chk(self.L.ngt_amd_build_get_tree(self.h, *[t[k].ctypes.data for k in (
            "leaf_parent", "leaf_off", "leaf_ids", "leaf_dists", "leaf_has_pivot", "leaf_pivot", "in_parent",
            "in_pivot", "in_child", "in_border")]))
        t["leaf_ids"], t["leaf_dists"] = t["leaf_ids"][:nli], t["leaf_dists"][:nli]
        # DVPTree::getRootNode (lib/NGT/Tree.h:219-235): internal 1 once the root leaf has split
        t["root"] = 1 if ni > 1 else 0x80000001
        return t

    # ---- NGTQG quantized graph (L2 float) ---------------------------------
    def qg_set_quantizer(self, global_centroid, local):
        """global_centroid: [dim]; local: [M, 16, dsub] (local ids 1..16)."""
        g = np.ascontiguousarray(np.asarray(global_centroid, np.float32)[:self.dim])
        loc = np.ascontiguousarray(local, dtype=np.float32)
        M, _, dsub = loc.shape
        _chk(self.L.ngt_amd_qg_set_quantizer(self.h, g.ctypes.data, loc.ctypes.data, M, dsub))
        self.qg_M = M
        self.qg_Me = (M + 1) // 2 * 2

    def qg_build_graph(self, local_codes=None, max_edges=128):
        """local_codes: [nrows, M] localID - 1 (0..15) of every object, or
        None for the codes of the last qg_encode (kept in HBM)."""
        if local_codes is None:
            _chk(self.L.ngt_amd_qg_build_graph(self.h, None, max_edges))
            return
        c = np.ascontiguousarray(local_codes, dtype=np.uint8)
        _chk(self.L.ngt_amd_qg_build_graph(self.h, c.ctypes.data, max_edges))

    def qg_encode(self, return_codes=True):
        """Nearest local centroid of every object's residual subvectors (the
        encoder of Quantizer::insert); codes stay on the device for
        qg_build_graph(None).  Returns [nrows, M] localID - 1, or None."""
        if not return_codes:
            _chk(self.L.ngt_amd_qg_encode(self.h, None))
            return None
        out = np.zeros((self.nrows, self.qg_M), np.uint8)
        _chk(self.L.ngt_amd_qg_encode(self.h, out.ctypes.data))
        return out

    def qg_train(self, M, nsample=1600, max_iter=20):
        """Train and install NGTQG local codebooks (global = zero vector) from
        objects 1..nsample.  Returns (local [M, 16, dim/M], iterations [M])."""
        dsub = self.dim // M
        loc = np.zeros((M, 16, dsub), np.float32)
        its = np.zeros(M, np.uint32)
        _chk(self.L.ngt_amd_qg_train(self.h, M, nsample, max_iter, loc.ctypes.data, its.ctypes.data))
        self.qg_M = M
        self.qg_Me = (M + 1) // 2 * 2
        return loc, its

    def qg_train_ngt(self, rows, dsub=1):
        """The codebooks ngtqg_quantize would train (kmeansWithNGT restatement,
        ngt_amd_qg_train_local_ngt) from host rows [nrows][>= dim] (row 0 the
        dummy slot), set as this index's quantizer (zero global centroid,
        QuantizedGraph.h:397-399); returns local [M][16][dsub]."""
        r = np.ascontiguousarray(np.asarray(rows, np.float32)[:1601, :self.dim])
        M = self.dim // dsub
        local = np.zeros((M, 16, dsub), np.float32)
        _chk(self.L.ngt_amd_qg_train_local_ngt(r.ctypes.data, r.shape[0], self.dim, dsub, local.ctypes.data))
        self.qg_set_quantizer(np.zeros(self.dim, np.float32), local)
        return local

    def qg_set_graph(self, qoff, qids, code_off, codes):
        qoff = np.ascontiguousarray(qoff, dtype=np.uint64)
        qids = np.ascontiguousarray(qids if len(qids) else np.zeros(1), dtype=np.uint32)
        code_off = np.ascontiguousarray(code_off, dtype=np.uint64)
        codes = np.ascontiguousarray(codes if len(codes) else np.zeros(1), dtype=np.uint8)
        _chk(self.L.ngt_amd_qg_set_graph(self.h, qoff.ctypes.data, qids.ctypes.data, code_off.ctypes.data,
                                         codes.ctypes.data))

    def qg_max_degree(self):
        return int(self.L.ngt_amd_qg_max_degree(self.h))

    def qg_get_graph(self):
        """(ids [nrows, max_degree] 0-terminated, codes [nrows, code_stride])."""
        if self.nrows <= 0:
            raise NativeError("qg_get_graph: the view does not know the index's row count")
        md = self.qg_max_degree()
        cs = int(self.L.ngt_amd_qg_code_stride(self.h))
        ids = np.zeros((self.nrows, md), np.uint32)
        codes = np.zeros((self.nrows, cs), np.uint8)
        _chk(self.L.ngt_amd_qg_get_graph(self.h, ids.ctypes.data, codes.ctypes.data))
        return ids, codes

    def qg_lut(self, queries):
        q = np.ascontiguousarray(queries, dtype=np.float32)
        nq = q.shape[0]
        lut = np.zeros((nq, self.qg_Me * 16), np.uint8)
        sc = np.zeros(nq, np.float32)
        to = np.zeros(nq, np.float32)
        _chk(self.L.ngt_amd_qg_lut(self.h, q.ctypes.data, nq, lut.ctypes.data, sc.ctypes.data, to.ctypes.data))
        return lut, sc, to

    def qg_adc(self, lut, scale, total_offset, qidx, nodes):
        lut = np.ascontiguousarray(lut, dtype=np.uint8)
        sc = np.ascontiguousarray(scale, dtype=np.float32)
        to = np.ascontiguousarray(total_offset, dtype=np.float32)
        qidx = np.ascontiguousarray(qidx, dtype=np.uint32)
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        md = self.qg_max_degree()
        out = np.zeros((len(nodes), md), np.float32)
        n = np.zeros(len(nodes), np.uint32)
        _chk(self.L.ngt_amd_qg_adc(self.h, lut.ctypes.data, sc.ctypes.data, to.ctypes.data, lut.shape[0],
                                   qidx.ctypes.data, nodes.ctypes.data, len(nodes), out.ctypes.data, n.ctypes.data))
        return out, n

    def qg_search(self, queries, k=20, epsilon=0.03, result_expansion=3.0, radius=-1.0, seed_mode=SEED_TREE,
                  seeds=None, counters=True, visited_hash_log2=0):
        """NGTQG::Index::search for a batch; defaults of ngtqg_initialize_query."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        nq = q.shape[0]
        prm = QgSearchParams(k, epsilon, result_expansion, radius, seed_mode, visited_hash_log2)
        ids = np.zeros((nq, k), np.uint32)
        ds = np.zeros((nq, k), np.float32)
        n = np.zeros(nq, np.uint32)
        cnt = np.zeros((nq, COUNTERS), np.uint64) if counters else None
        sp = so = None
        if seed_mode == SEED_GIVEN:
            so = np.zeros(nq + 1, np.uint64)
            so[1:] = np.cumsum([len(s) for s in seeds])
            sp = np.ascontiguousarray(np.concatenate([np.asarray(s, np.uint32) for s in seeds])
                                      if so[-1] else np.zeros(1, np.uint32))
        _chk(self.L.ngt_amd_qg_search(self.h, byref(prm), q.ctypes.data, nq, _ptr(sp), _ptr(so), ids.ctypes.data,
                                      ds.ctypes.data, n.ctypes.data, _ptr(cnt)))
        return ids, ds, n, cnt

    def qg_search_device(self, d_queries, query_bytes, nq, d_ids, d_dists, d_n, d_counters=None, k=20,
                         epsilon=0.03, result_expansion=3.0, radius=-1.0, seed_mode=SEED_TREE, d_seeds=None,
                         d_seed_off=None, stream=None, visited_hash_log2=0):
        prm = QgSearchParams(k, epsilon, result_expansion, radius, seed_mode, visited_hash_log2)
        _chk(self.L.ngt_amd_qg_search_device(self.h, byref(prm), d_queries, query_bytes, nq, d_seeds, d_seed_off,
                                             d_ids, d_dists, d_n, d_counters, stream))

    def close(self):
        if getattr(self, "h", None):
            if not getattr(self, "_borrowed", False):
                self.L.ngt_amd_index_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
