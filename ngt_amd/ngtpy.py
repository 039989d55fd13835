"""``ngtpy``-compatible surface over the drop-in C API (python/src/ngtpy.cpp:30-330
for the behaviour, :505-560 for the names and defaults).

Same module-level ``create`` and ``Index`` class, same argument names and
defaults, same result shapes: a list of ``(id, distance)`` tuples, or an int32
id array with ``with_distance=False``, ids zero-based unless
``zero_based_numbering=False``.  Every search runs on the MI355X through
libngt_amd.so (``ngt_batch_search_index`` / ``_using_only_graph`` /
``ngt_batch_linear_search_index``); there is no host fallback.
"""
import os

import numpy as np

from . import NativeError
from . import base

FLT_MAX = 3.4028234663852886e38
INT_MIN = -(2 ** 31)


def create(path, dimension, edge_size_for_creation=10, edge_size_for_search=40, distance_type="L2",
           object_type="Float"):
    """ngtpy.create (ngtpy.cpp:52-101): an empty index directory."""
    ot = {"Float": "Float", "float": "Float", "Byte": "Integer", "byte": "Integer"}.get(object_type)
    if ot is None:
        raise NativeError("ngtpy::create: invalid object type. " + object_type)
    if distance_type not in ("L1", "L2", "Normalized L2", "Hamming", "Jaccard", "Sparse Jaccard", "Angle",
                             "Normalized Angle", "Cosine", "Normalized Cosine"):
        raise NativeError("ngtpy::create: invalid distance type. " + distance_type)
    base.Index.create(path, dimension, edge_size_for_creation, edge_size_for_search, ot, distance_type)


def accuracy_table(path):
    """The prf's AccuracyTable (Index.h:255, written by the optimizer) as
    Index::AccuracyTable::set parses it (Index.h:299-315): comma-separated
    ``epsilon:accuracy`` pairs, epsilon stored as float, accuracy as double;
    fewer than two tokens leave the table empty."""
    text = ""
    with open(os.path.join(path, "prf")) as f:
        for line in f:
            key, _, val = line.rstrip("\n").partition("\t")
            if key == "AccuracyTable":
                text = val
    toks = [t for t in text.split(",") if t]
    if len(toks) < 2:
        return []
    table = []
    for t in toks:
        ts = [x for x in t.split(":") if x]
        if len(ts) != 2:
            raise NativeError("AccuracyTable: Invalid accuracy table string %s:%s" % (t, text))
        table.append((np.float32(float(ts[0])), float(ts[1])))
    return table


def epsilon_from_expected_accuracy(table, accuracy):
    """Index::AccuracyTable::getEpsilon (Index.h:317-346): linear
    interpolation between the entries that bracket `accuracy`, in the
    reference's mixed float/double arithmetic, clamped below at -0.9."""
    if len(table) <= 2:
        raise NativeError("AccuracyTable: The accuracy table is not set yet. The table size=%d" % len(table))
    accuracy = min(float(accuracy), 1.0)
    i = 0
    while i < len(table) and table[i][1] < accuracy:
        i += 1
    if i == len(table):
        i -= 2
    elif i != 0:
        i -= 1
    (lf, ls), (uf, us) = table[i], table[i + 1]
    e = np.float32(float(lf) + float(np.float32(uf - lf)) * (accuracy - ls) / (us - ls))
    return float(max(e, np.float32(-0.9)))


class Index(object):
    """ngtpy.Index (ngtpy.cpp:30-50): defaults k=20, epsilon=0.1,
    radius=FLT_MAX, edge size from the property."""

    def __init__(self, path, read_only=False, zero_based_numbering=True, tree_disabled=False,
                 log_disabled=False):
        self._ix = base.Index(path)
        self.read_only = read_only
        self.zero = zero_based_numbering
        self.tree = not tree_disabled
        self.num_of_search_objects = 20
        self.epsilon = 0.1
        self.radius = FLT_MAX
        self.edge_size = -1
        self.expected_accuracy = -1.0  # defaultExpectedAccuracy (ngtpy.cpp:49)
        self.distance_computations = 0
        self._table = None

    def _id_out(self, ids):
        return ids.astype(np.int64) - 1 if self.zero else ids.astype(np.int64)

    def _id_in(self, oid):
        return oid + 1 if self.zero else oid

    def _results(self, ids, ds, n, with_distance):
        ids = self._id_out(ids[0, :n[0]])
        if not with_distance:
            return ids.astype(np.int32)
        return [(int(i), float(d)) for i, d in zip(ids, ds[0, :n[0]])]

    def search(self, query, size=0, epsilon=-FLT_MAX, edge_size=INT_MIN, expected_accuracy=-FLT_MAX,
               with_distance=True):
        """ngtpy.cpp:141-214: tree-seeded search unless tree_disabled.  A
        positive expected_accuracy replaces epsilon with the one the prf's
        AccuracyTable maps it to (sc.setExpectedAccuracy, then
        GraphIndex::search's getEpsilonFromExpectedAccuracy, Index.h:1156-1158)."""
        q = np.ascontiguousarray(query, dtype=np.float32).reshape(1, -1)
        k = size if size > 0 else self.num_of_search_objects
        eps = self.epsilon if epsilon <= -1.0 else epsilon
        if expected_accuracy > 0.0:
            eps = self.epsilon_for(expected_accuracy)
        es = self.edge_size if edge_size < -2 else edge_size
        ids, ds, n = self._ix.batch_search(q, k, eps, self.radius, es, graph_only=not self.tree)
        self.distance_computations += int(self._ix.last_search_counters()[0])
        return self._results(ids, ds, n, with_distance)

    def epsilon_for(self, expected_accuracy):
        """The epsilon a search with this expected accuracy uses (the pybind
        argument is a float, widened to double for getEpsilon)."""
        if self._table is None:
            self._table = accuracy_table(self._ix.path)
        return epsilon_from_expected_accuracy(self._table, float(np.float32(expected_accuracy)))

    def linear_search(self, query, size=0, with_distance=True):
        """ngtpy.cpp:216-268: exact k-NN by full scan within the index's search
        radius (sc.setRadius(defaultRadius)).  The reference adds
        sc.distanceComputationCount, which ObjectSpaceRepository::linearSearch
        (ObjectSpaceRepository.h:466-502) never increments: the count is unchanged."""
        q = np.ascontiguousarray(query, dtype=np.float32).reshape(1, -1)
        k = size if size > 0 else self.num_of_search_objects
        ids, ds, n = self._ix.batch_linear_search(q, k, radius=self.radius)
        return self._results(ids, ds, n, with_distance)

    def get_num_of_distance_computations(self):
        return self.distance_computations

    def set(self, num_of_search_objects=0, search_radius=-FLT_MAX, epsilon=-FLT_MAX, edge_size=INT_MIN,
            expected_accuracy=-FLT_MAX):
        """ngtpy.cpp:322-333: a non-positive / out-of-range value keeps the
        default.  expected_accuracy is kept as defaultExpectedAccuracy, which
        the reference's search never reads (it takes only its own argument,
        ngtpy.cpp:168-172): a set() value changes no search there or here."""
        if num_of_search_objects > 0:
            self.num_of_search_objects = num_of_search_objects
        if epsilon > -1.0:
            self.epsilon = epsilon
        if search_radius >= 0.0:
            self.radius = search_radius
        if edge_size >= -2:
            self.edge_size = edge_size
        if expected_accuracy > 0.0:
            self.expected_accuracy = expected_accuracy

    def insert(self, object, debug=False):
        """ngtpy.cpp:119-139: append one object (no graph update until build_index)."""
        return self._id_out(np.array([self._ix.insert_object(object)]))[0].item()

    def batch_insert(self, objects, num_threads=8, debug=False):
        """ngtpy.cpp:98-117: append all rows, then build the index on the GPU."""
        objs = np.asarray(objects, dtype=np.float32)
        if objs.ndim != 2 or objs.shape[1] != self._ix.dim:
            raise NativeError("ngtpy::insert: Error! dimensions are inconsitency. %d:%d"
                              % (self._ix.dim, objs.shape[-1]))
        self._ix.insert(objs, num_threads)
        self.distance_computations = 0

    def build_index(self, num_threads=8, target_size_of_graph=0):
        self._ix.build_index(num_threads)

    def get_object(self, object_id):
        return [float(x) for x in self._ix.get_object(self._id_in(object_id))]

    def remove(self, object_id):
        """Not supported: GraphAndTreeIndex::remove re-links the graph around the
        removed node (graph maintenance, out of this build's scope); raises
        NativeError with the C API's message."""
        L = self._ix._L
        self._ix._check(L.ngt_remove_index(self._ix.index, self._id_in(object_id), self._ix.err), self._ix.err)

    def save(self):
        if self.read_only:
            raise NativeError("ngtpy::save: the index is read only")
        self._ix.save()

    def close(self):
        self._ix.close()
