"""NGTQ (IVF-ADC) search over the C ABI: the Python mirror of ``NGTQ::Index``
(lib/NGT/NGTQ/Quantizer.h:2819-2930) and the ``ngtq search`` command
(lib/NGT/NGTQ/NGTQCommand.h:272-420).

``Index(path)`` opens an NGTQ index directory made by ``ngtq create`` (prf,
global/, local-<i>/, ivt, obj) into HBM; ``search`` is
``NGTQ::Index::search(object, objs, size, expansion, aggregationMode, epsilon)``
for a batch of queries.  Modes are the CLI's letters (``-m``):

    'a' AggregationModeApproximateDistance                 (residual distances)
    'c' AggregationModeApproximateDistanceWithCache        (AVX residual distances)
    'l' AggregationModeApproximateDistanceWithLookupTable  (float LUT ADC)
    'e' AggregationModeExactDistance                       (object list, L2 comparator)
    'r' AggregationModeExactDistanceThroughApproximateDistance ('c', then exact refinement)

``epsilon=None`` (the CLI's ``-e -``) searches the global codebook linearly.
Every distance is computed on the device; there is no CPU path.
"""
from ctypes import byref, c_void_p

import numpy as np

from . import NativeError, lib
from ._sigs import NgtqSearchParams

MODES = {"a": 0, "l": 1, "c": 2, "r": 3, "e": 4}


def _chk(L, rc):
    if rc != 0:
        raise NativeError(L.ngt_amd_last_error().decode())


class Index(object):
    """NGTQ::Index(path) on device `device`."""

    def __init__(self, path, device=0):
        self.L = lib()
        h = c_void_p()
        _chk(self.L, self.L.ngt_amd_ngtq_open(path.encode(), device, byref(h)))
        self.h = h
        self.dim = int(self.L.ngt_amd_index_padded_dimension(self.h))
        self.path = path

    @classmethod
    def from_arrays(cls, index, local, list_off, eids, elids, objects):
        """The quantizer state from host arrays on an existing DeviceIndex
        `index` holding the global codebook (rows, graph, tree): local
        [N, 16, dsub], list_off [nlists + 1], eids [E], elids [E, N] uint16,
        objects [records, dim] (record 0 unused).  The DeviceIndex keeps the
        device memory; this object borrows it."""
        self = cls.__new__(cls)
        self.L = lib()
        local = np.ascontiguousarray(local, np.float32)
        N, _, dsub = local.shape
        lo = np.ascontiguousarray(list_off, np.uint64)
        ei = np.ascontiguousarray(eids, np.uint32)
        el = np.ascontiguousarray(elids, np.uint16)
        ob = np.ascontiguousarray(objects, np.float32)
        _chk(self.L, self.L.ngt_amd_ngtq_set(index.h, local.ctypes.data, N, dsub, lo.ctypes.data, len(lo) - 1,
                                             ei.ctypes.data, el.ctypes.data, len(ei), ob.ctypes.data, ob.shape[0]))
        self.h = index.h
        self.dim = index.dp
        self.path = None
        self._borrowed = index
        return self

    def search(self, queries, size=20, expansion=16.0, mode="a", epsilon=0.1):
        """Batch of NGTQ::Index::search; returns (ids [nq, size], dists, n [nq])."""
        q = np.ascontiguousarray(np.atleast_2d(queries), dtype=np.float32)
        nq = q.shape[0]
        prm = NgtqSearchParams(size, expansion, -1.0 if epsilon is None else epsilon, MODES[mode])
        ids = np.zeros((nq, size), np.uint32)
        ds = np.zeros((nq, size), np.float32)
        n = np.zeros(nq, np.uint32)
        _chk(self.L, self.L.ngt_amd_ngtq_search(self.h, byref(prm), q.ctypes.data, nq, ids.ctypes.data,
                                                ds.ctypes.data, n.ctypes.data))
        return ids, ds, n

    def search_device(self, d_queries, query_bytes, nq, d_ids, d_dists, d_n, size=20, expansion=16.0, mode="a",
                      epsilon=0.1, stream=None):
        prm = NgtqSearchParams(size, expansion, -1.0 if epsilon is None else epsilon, MODES[mode])
        _chk(self.L, self.L.ngt_amd_ngtq_search_device(self.h, byref(prm), d_queries, query_bytes, nq, d_ids,
                                                       d_dists, d_n, stream))

    def close(self):
        if getattr(self, "h", None) and getattr(self, "_borrowed", None) is None:
            self.L.ngt_amd_index_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
