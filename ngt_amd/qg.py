"""NGTQG quantized-graph index over the drop-in ``ngtqg_*`` C API
(include/NGT/NGTQ/Capi.h), shaped like the reference's ``ngtpy.QuantizedIndex``
(python/src/ngtpy.cpp:383-473, 613-640): ``search`` returns a list of
(id, distance) tuples, ids zero-based by default.  Every search runs on the
MI355X (qg_kernels.hip); without a device opening the index fails.
"""
import ctypes

import numpy as np

from . import NativeError, lib
from ._sigs import NGTQGQuery, NGTQGQuantizationParameters


def quantize(path, dimension_of_subvector=0, max_number_of_edges=128):
    """``ngtqg quantize`` / ngtqg_quantize (NGTQ/Capi.cpp:120-131): writes
    <path>/qg (codebooks, codes, quantized graph) on the device; a no-op when
    <path>/qg exists (QuantizedGraph.h:456-475)."""
    L = lib()
    err = L.ngt_create_error_object()
    try:
        p = NGTQGQuantizationParameters()
        L.ngtqg_initialize_quantization_parameters(ctypes.byref(p))
        p.dimension_of_subvector = float(dimension_of_subvector)
        p.max_number_of_edges = int(max_number_of_edges)
        if not L.ngtqg_quantize(path.encode(), p, err):
            raise NativeError(L.ngt_get_error_string(err).decode())
    finally:
        L.ngt_destroy_error_object(err)


class QuantizedIndex(object):
    def __init__(self, path, max_no_of_edges=128, zero_based_numbering=True, tree_disabled=False,
                 log_disabled=False):
        if max_no_of_edges != 128:
            raise NativeError("QuantizedIndex: max_no_of_edges other than 128 needs a saved qg/grp")
        if tree_disabled:
            raise NativeError("QuantizedIndex: tree_disabled is not supported (seeds come from the DVP tree)")
        self.L = lib()
        self.err = self.L.ngt_create_error_object()
        self.h = self.L.ngtqg_open_index(path.encode(), self.err)
        if not self.h:
            raise NativeError(self._error())
        self.zero = zero_based_numbering
        q = NGTQGQuery()
        self.L.ngtqg_initialize_query(ctypes.byref(q))
        self.dim = None
        # ngtpy.QuantizedIndex defaults (ngtpy.cpp:396-399)
        self.default_size, self.default_epsilon, self.default_expansion = 20, 0.02, 3.0

    def _error(self):
        s = self.L.ngt_get_error_string(self.err).decode()
        self.L.ngt_clear_error_string(self.err)
        return s

    def set(self, num_of_search_objects=0, epsilon=-3.4e38, result_expansion=-1.0, edge_size=-3):
        if num_of_search_objects > 0:
            self.default_size = num_of_search_objects
        if epsilon > -1.0:
            self.default_epsilon = epsilon
        if result_expansion >= 0.0:
            self.default_expansion = result_expansion

    def _params(self, size, epsilon, result_expansion):
        size = size if size > 0 else self.default_size
        epsilon = epsilon if epsilon > -1.0 else self.default_epsilon
        result_expansion = result_expansion if result_expansion >= 0.0 else self.default_expansion
        return size, epsilon, result_expansion

    def search(self, query, size=0, epsilon=-3.4e38, result_expansion=-1.0, edge_size=-3):
        size, epsilon, result_expansion = self._params(size, epsilon, result_expansion)
        q = np.ascontiguousarray(query, dtype=np.float32)
        sq = NGTQGQuery()
        self.L.ngtqg_initialize_query(ctypes.byref(sq))
        sq.query = q.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        sq.size = size
        sq.epsilon = epsilon
        sq.result_expansion = result_expansion
        res = self.L.ngt_create_empty_results(self.err)
        try:
            if not self.L.ngtqg_search_index(self.h, sq, res, self.err):
                raise NativeError(self._error())
            n = self.L.ngt_get_result_size(res, self.err)
            out = []
            for i in range(n):
                r = self.L.ngt_get_result(res, i, self.err)
                out.append((r.id - 1 if self.zero else r.id, r.distance))
            return out
        finally:
            self.L.ngt_destroy_results(res)

    def batch_search(self, queries, size=0, epsilon=-3.4e38, result_expansion=-1.0, radius=-1.0):
        """All queries in one device batch: (ids [nq, size], dists, n [nq]); ids
        keep the index's 1-based numbering."""
        size, epsilon, result_expansion = self._params(size, epsilon, result_expansion)
        q = np.ascontiguousarray(queries, dtype=np.float32)
        nq, dim = q.shape
        ids = np.zeros((nq, size), np.uint32)
        ds = np.zeros((nq, size), np.float32)
        n = np.zeros(nq, np.uint32)
        f32p, u32p = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint32)
        ok = self.L.ngtqg_batch_search_index(self.h, q.ctypes.data_as(f32p), nq, dim, size, epsilon,
                                             result_expansion, radius, ids.ctypes.data_as(u32p),
                                             ds.ctypes.data_as(f32p), n.ctypes.data_as(u32p), self.err)
        if not ok:
            raise NativeError(self._error())
        return ids, ds, n

    def close(self):
        if getattr(self, "h", None):
            self.L.ngtqg_close_index(self.h)
            self.h = None
        if getattr(self, "err", None):
            self.L.ngt_destroy_error_object(self.err)
            self.err = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
