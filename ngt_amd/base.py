"""ctypes binding of the drop-in ``ngt_*`` C API, mirroring the reference's
``ngt.base.Index`` (python/ngt/base.py:42-501): same method names, arguments
and error behaviour (``NativeError`` carries the C API's error string).
Every search runs on the MI355X through libngt_amd.so.
"""
import ctypes
from ctypes import POINTER, c_double, c_float, c_uint32, c_uint64

import numpy as np

from . import NativeError, lib
from ._sigs import NGTQuery, ObjectDistance  # noqa: F401  (re-exported)


class APIError(Exception):
    pass


def _err_string(L, err):
    s = L.ngt_get_error_string(err)
    return s.decode() if s else ""


class Index(object):
    """An NGT index opened from its directory (prf/obj/grp/tre)."""

    def __init__(self, path):
        self.path = path
        L = self._L = lib()
        self.err = L.ngt_create_error_object()
        self.index = L.ngt_open_index(path.encode(), self.err)
        if not self.index:
            raise NativeError(_err_string(L, self.err))
        self.prop = L.ngt_create_property(self.err)
        if not L.ngt_get_property(self.index, self.prop, self.err):
            raise NativeError(_err_string(L, self.err))
        self.dim = L.ngt_get_property_dimension(self.prop, self.err)
        self.otype = L.ngt_get_property_object_type(self.prop, self.err)
        self.is_float = bool(L.ngt_is_property_object_type_float(self.otype))
        self.distance_type = L.ngt_get_property_distance_type(self.prop, self.err)
        # SparseJaccard objects keep one more slot (Index.cpp:488-490)
        self.object_dim = self.dim + (1 if self.distance_type == 8 else 0)
        self.ospace = L.ngt_get_object_space(self.index, self.err)

    def _check(self, ok, err):
        if not ok:
            raise NativeError(_err_string(self._L, err))

    @staticmethod
    def create(path, dimension, edge_size_for_creation=10, edge_size_for_search=40, object_type="Float",
               distance_type="L2"):
        """Create an empty index directory (python/ngt/base.py:199-279 ->
        ngt_create_graph_and_tree)."""
        L = lib()
        err = L.ngt_create_error_object()
        prop = L.ngt_create_property(err)
        ok = L.ngt_set_property_dimension(prop, dimension, err) and \
            L.ngt_set_property_edge_size_for_creation(prop, edge_size_for_creation, err) and \
            L.ngt_set_property_edge_size_for_search(prop, edge_size_for_search, err)
        ok = ok and (L.ngt_set_property_object_type_float(prop, err) if object_type == "Float"
                     else L.ngt_set_property_object_type_integer(prop, err))
        setters = {"L1": L.ngt_set_property_distance_type_l1, "L2": L.ngt_set_property_distance_type_l2,
                   "Angle": L.ngt_set_property_distance_type_angle,
                   "Hamming": L.ngt_set_property_distance_type_hamming,
                   "Jaccard": L.ngt_set_property_distance_type_jaccard,
                   "Cosine": L.ngt_set_property_distance_type_cosine,
                   "Normalized Angle": L.ngt_set_property_distance_type_normalized_angle,
                   "Normalized Cosine": L.ngt_set_property_distance_type_normalized_cosine,
                   "Normalized L2": L.ngt_set_property_distance_type_normalized_l2,
                   "Sparse Jaccard": L.ngt_set_property_distance_type_sparse_jaccard}
        ok = ok and setters[distance_type](prop, err)
        index = L.ngt_create_graph_and_tree(path.encode(), prop, err) if ok else None
        msg = _err_string(L, err)
        if index:
            L.ngt_close_index(index)
        L.ngt_destroy_property(prop)
        L.ngt_destroy_error_object(err)
        if not ok or not index:
            raise NativeError(msg)

    def insert_object(self, obj):
        """Append one object (ngt_insert_index_as_float); returns its id."""
        o = np.ascontiguousarray(obj, dtype=np.float32)
        oid = self._L.ngt_insert_index_as_float(self.index, o.ctypes.data_as(POINTER(c_float)), len(o), self.err)
        if oid == 0:
            raise NativeError(_err_string(self._L, self.err))
        return oid

    def insert(self, objects, num_threads=8):
        """Append objects and build the index (python/ngt/base.py:378-389)."""
        for o in objects:
            self.insert_object(o)
        self.build_index(num_threads)

    def build_index(self, num_threads=8):
        """ngt_create_index: ANNG + DVP tree of the appended objects, built on the GPU."""
        self._check(self._L.ngt_create_index(self.index, num_threads, self.err), self.err)

    def search(self, query, k=20, epsilon=0.1, radius=-1.0):
        """k nearest neighbours of `query` (ngt_search_index, Capi.cpp:346-375).
        Returns a list of ObjectDistance (id, distance) ascending."""
        L = self._L
        err = L.ngt_create_error_object()
        results = L.ngt_create_empty_results(err)
        try:
            q = np.ascontiguousarray(query, dtype=np.float64)
            ok = L.ngt_search_index(self.index, q.ctypes.data_as(POINTER(c_double)), len(q), k, epsilon, radius,
                                    results, err)
            self._check(ok, err)
            n = L.ngt_get_size(results, err)
            return [L.ngt_get_result(results, i, err) for i in range(n)]
        finally:
            L.ngt_destroy_results(results)
            L.ngt_destroy_error_object(err)

    def search_with_query(self, query, k=20, epsilon=0.1, radius=-1.0, edge_size=-1):
        """ngt_search_index_with_query (Capi.cpp:408-439)."""
        L = self._L
        err = L.ngt_create_error_object()
        results = L.ngt_create_empty_results(err)
        try:
            q = np.ascontiguousarray(query, dtype=np.float32)
            nq = NGTQuery(q.ctypes.data_as(POINTER(c_float)), k, epsilon, 0.0, radius,
                          ctypes.c_size_t(edge_size & 0xFFFFFFFFFFFFFFFF).value)
            self._check(L.ngt_search_index_with_query(self.index, nq, results, err), err)
            n = L.ngt_get_result_size(results, err)
            return [L.ngt_get_result(results, i, err) for i in range(n)]
        finally:
            L.ngt_destroy_results(results)
            L.ngt_destroy_error_object(err)

    def linear_search(self, query, k=20):
        """Exact k-NN (ngt_linear_search_index, Capi.cpp:458-483)."""
        L = self._L
        err = L.ngt_create_error_object()
        results = L.ngt_create_empty_results(err)
        try:
            q = np.ascontiguousarray(query, dtype=np.float64)
            ok = L.ngt_linear_search_index(self.index, q.ctypes.data_as(POINTER(c_double)), len(q), k, results,
                                           err)
            self._check(ok, err)
            n = L.ngt_get_size(results, err)
            return [L.ngt_get_result(results, i, err) for i in range(n)]
        finally:
            L.ngt_destroy_results(results)
            L.ngt_destroy_error_object(err)

    def _batch(self, queries):
        """[nq][object dimension] float32 queries; a wrong length is an error,
        as allocateObject's dimension check makes it (ObjectRepository.h:228-233)."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim != 2:
            raise NativeError("queries must be a 2-d array")
        if q.shape[1] != self.object_dim:
            if self.distance_type == 8 and q.shape[1] < self.object_dim:
                q = np.ascontiguousarray(np.pad(q, ((0, 0), (0, self.object_dim - q.shape[1]))))
            else:
                raise NativeError("The dimensionality is invalid. The indexed objects=%d The specified object=%d"
                                  % (self.dim, q.shape[1]))
        return q

    def batch_search(self, queries, k=20, epsilon=0.1, radius=-1.0, edge_size=-1, graph_only=False):
        """Batched search on the device: returns (ids[nq,k], dists[nq,k], n[nq])."""
        L = self._L
        q = self._batch(queries)
        nq = q.shape[0]
        ids = np.zeros((nq, k), np.uint32)
        ds = np.zeros((nq, k), np.float32)
        n = np.zeros(nq, np.uint32)
        fn = L.ngt_batch_search_index_using_only_graph if graph_only else L.ngt_batch_search_index
        ok = fn(self.index, q.ctypes.data_as(POINTER(c_float)), nq, q.shape[1], k, epsilon, radius, edge_size,
                ids.ctypes.data_as(POINTER(c_uint32)), ds.ctypes.data_as(POINTER(c_float)),
                n.ctypes.data_as(POINTER(c_uint32)), self.err)
        self._check(ok, self.err)
        return ids, ds, n

    def batch_linear_search(self, queries, k=20, radius=-1.0):
        """Exact k-NN of a batch (linearSearch with SearchContainer::radius;
        radius < 0 is unbounded)."""
        L = self._L
        q = self._batch(queries)
        nq = q.shape[0]
        ids = np.zeros((nq, k), np.uint32)
        ds = np.zeros((nq, k), np.float32)
        n = np.zeros(nq, np.uint32)
        ok = L.ngt_batch_linear_search_index_with_radius(self.index, q.ctypes.data_as(POINTER(c_float)), nq,
                                                         q.shape[1], k, radius,
                                                         ids.ctypes.data_as(POINTER(c_uint32)),
                                                         ds.ctypes.data_as(POINTER(c_float)),
                                                         n.ctypes.data_as(POINTER(c_uint32)), self.err)
        self._check(ok, self.err)
        return ids, ds, n

    def last_search_counters(self):
        c = np.zeros(3, np.uint64)
        self._check(self._L.ngt_get_last_search_counters(self.index, c.ctypes.data_as(POINTER(c_uint64)),
                                                         self.err), self.err)
        return c

    def get_object(self, id):
        """ngt_get_object_as_float / _as_integer (Capi.cpp:750-781)."""
        L = self._L
        if self.is_float:
            p = L.ngt_get_object_as_float(self.ospace, id, self.err)
        else:
            p = L.ngt_get_object_as_integer(self.ospace, id, self.err)
        if not p:
            raise NativeError(_err_string(L, self.err))
        return [p[i] for i in range(self.dim)]

    def get_edges(self, id):
        L = self._L
        err = L.ngt_create_error_object()
        results = L.ngt_create_empty_results(err)
        try:
            self._check(L.ngt_get_edges(self.index, id, results, err), err)
            n = L.ngt_get_result_size(results, err)
            return [L.ngt_get_result(results, i, err) for i in range(n)]
        finally:
            L.ngt_destroy_results(results)
            L.ngt_destroy_error_object(err)

    def batch_append(self, objects):
        """Append objects without building (ngt_batch_append_index); ids continue
        from the repository size."""
        o = np.ascontiguousarray(objects, dtype=np.float32)
        self._check(self._L.ngt_batch_append_index(self.index, o.ctypes.data_as(POINTER(c_float)), o.shape[0],
                                                   self.err), self.err)

    def device_index(self):
        """The DeviceIndex view of the ngt_amd_index this handle searches on
        (ngt_get_device_index); valid until the next write or close."""
        from .device import DeviceIndex
        h = self._L.ngt_get_device_index(self.index, self.err)
        if not h:
            raise NativeError(_err_string(self._L, self.err))
        # nrows: the repository's slots, dummy slot 0 included (the device rows)
        return DeviceIndex.wrap(h, int(self.distance_type), "float" if self.is_float else "uint8", self.dim,
                                nrows=int(self._L.ngt_get_object_repository_size(self.index, self.err)))

    def save(self, path=None):
        if path is None:
            path = self.path
        self._check(self._L.ngt_save_index(self.index, path.encode(), self.err), self.err)

    def close(self):
        if getattr(self, "index", None):
            self._L.ngt_close_index(self.index)
            self.index = None
        if getattr(self, "prop", None):
            self._L.ngt_destroy_property(self.prop)
            self.prop = None
        if getattr(self, "err", None):
            self._L.ngt_destroy_error_object(self.err)
            self.err = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
