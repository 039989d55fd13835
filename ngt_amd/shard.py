"""Object repository sharded across GPUs (BASELINE configs C4
and C5).

One process per GPU.  Rank r holds shard r -- objects with global ids
``offset_r + 1 .. offset_r + n_r`` as its own index (rows, graph, and for
NGTQG its quantized graph) in HBM -- and every rank searches every query on
its shard: the exact best-first search (NeighborhoodGraph::searchReadOnlyGraph,
Graph.cpp:398-495) or the quantized-graph search (NGTQG::Index::search,
QuantizedGraph.h:354-372).  The one exchange step is ONE all-gather per batch
of the packed per-shard result lists: ``k`` 8-byte words per query, each the
``{uint32 id, float distance}`` pair of NGT::ObjectDistance (Common.h:1937-1992)
packed as ``distance bits << 32 | local id`` by ``ngt_amd_pack_results_device``
(0 = empty slot) -- RCCL over xGMI when the process group is ``nccl``, Q*k*8 B
per rank (800 KB at 10k queries, k = 10).  Every rank then merges the gathered
words on its device with ``ngt_amd_merge_packed_device``: the k best by
(distance, global id), the result one index over the union would rank.

The exchange is backend-agnostic (torch.distributed collectives on tensors of
the merge's device); the CPU tests run it over ``gloo`` with numpy stand-ins
for the two device kernels (``pack=`` / ``merge=``).
"""
import contextlib

import numpy as np

from . import NativeError, lib


def shard_bounds(n_total, world, rank):
    """Contiguous global-id range of shard `rank`: (offset, count), ids
    offset+1 .. offset+count (shard s owns [s*N/W+1, (s+1)*N/W])."""
    base, extra = divmod(n_total, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def gather_offsets(torch, dist, offset, device):
    """All ranks' shard offsets, in rank order; `offset` is this rank's offset
    or the list of its local shards' offsets (the same count on every rank),
    and the result lists every shard rank-major."""
    world = dist.get_world_size()
    local = list(offset) if isinstance(offset, (list, tuple)) else [offset]
    t = torch.tensor(local, dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [int(v) for x in out for v in x.tolist()]


def pack_device(torch, ids, dists, n, k, stream=None):
    """[nq, k] ids/dists + [nq] counts -> [nq, k] int64 words (ngt_amd_pack_results_device)."""
    L = lib()
    nq = int(n.shape[0])
    out = torch.empty((nq, k), dtype=torch.int64, device=ids.device)
    rc = L.ngt_amd_pack_results_device(ids.device.index or 0, ids.data_ptr(), dists.data_ptr(), n.data_ptr(), nq, k,
                                       out.data_ptr(), stream)
    if rc != 0:
        raise NativeError(L.ngt_amd_last_error().decode())
    return out


def exchange_packed(torch, dist, packed):
    """The one collective: all-gather of every rank's packed words, [nq, k]
    (one shard per rank) or [S, nq, k] (S local shards) -> [world * S, nq, k]
    on every rank, shards rank-major."""
    world = dist.get_world_size()
    shape = tuple(packed.shape) if packed.dim() == 3 else (1,) + tuple(packed.shape)
    g = torch.empty((world * shape[0] * shape[1], shape[2]), dtype=packed.dtype, device=packed.device)
    dist.all_gather_into_tensor(g, packed.contiguous().view(shape[0] * shape[1], shape[2]))
    return g.view((world * shape[0],) + shape[1:])


def merge_packed_device(torch, g_packed, offsets, k, stream=None):
    """Device merge of gathered packed words (ngt_amd_merge_packed_device)."""
    L = lib()
    world, nq = int(g_packed.shape[0]), int(g_packed.shape[1])
    dev = g_packed.device
    out_i = torch.zeros((nq, k), dtype=torch.int32, device=dev)
    out_d = torch.zeros((nq, k), dtype=torch.float32, device=dev)
    out_n = torch.zeros((nq,), dtype=torch.int32, device=dev)
    off = np.ascontiguousarray(offsets, dtype=np.uint32)
    rc = L.ngt_amd_merge_packed_device(dev.index or 0, g_packed.data_ptr(), world, nq, k, off.ctypes.data,
                                       out_i.data_ptr(), out_d.data_ptr(), out_n.data_ptr(), stream)
    if rc != 0:
        raise NativeError(L.ngt_amd_last_error().decode())
    return out_i, out_d, out_n


def merge_device(torch, g_ids, g_d, g_n, offsets, k, stream=None):
    """Device merge of gathered unpacked lists (ngt_amd_merge_results_device):
    [world, nq, k] ids/dists and [world, nq] counts."""
    L = lib()
    world, nq = int(g_n.shape[0]), int(g_n.shape[1])
    dev = g_ids.device
    out_i = torch.zeros((nq, k), dtype=torch.int32, device=dev)
    out_d = torch.zeros((nq, k), dtype=torch.float32, device=dev)
    out_n = torch.zeros((nq,), dtype=torch.int32, device=dev)
    off = np.ascontiguousarray(offsets, dtype=np.uint32)
    rc = L.ngt_amd_merge_results_device(dev.index or 0, g_ids.data_ptr(), g_d.data_ptr(), g_n.data_ptr(), world, nq,
                                        k, off.ctypes.data, out_i.data_ptr(), out_d.data_ptr(), out_n.data_ptr(),
                                        stream)
    if rc != 0:
        raise NativeError(L.ngt_amd_last_error().decode())
    return out_i, out_d, out_n


class ShardedIndex(object):
    """Search front end of one rank's shard.  `index` is the rank's
    DeviceIndex (ids 1..n_r local); `offset` its global id offset.  A rank may
    also hold S shards (lists of S indexes and S offsets, the same S on every
    rank): an index larger than one graph a run can build is served as S
    shards per GPU -- each searched on its own stream, all S packed into the
    rank's one all-gather message, and the merge ranks world * S lists."""

    def __init__(self, torch, dist, index, offset, device, pack=pack_device, merge=merge_packed_device):
        self.torch, self.dist = torch, dist
        self.indexes = list(index) if isinstance(index, (list, tuple)) else [index]
        self.index = self.indexes[0]
        self.device = device
        self.offsets = gather_offsets(torch, dist, offset, device)
        self.pack = pack
        self.merge = merge

    @contextlib.contextmanager
    def _on(self, stream):
        """Context in which torch's current stream is `stream` (a raw HIP
        stream handle), so every allocation, fill and collective below is
        ordered with the library's launches on it; yields that torch stream
        (None on CPU tensors or without a stream)."""
        if stream is None or getattr(self.device, "type", "cpu") != "cuda":
            yield None
            return
        if int(stream) == self.torch.cuda.current_stream(self.device).cuda_stream:
            yield None  # already torch's current stream: everything is ordered on it
            return
        ext = self.torch.cuda.ExternalStream(stream, device=self.device)
        with self.torch.cuda.stream(ext):
            yield ext

    def merge_local(self, ids, dists, n, k, stream=None):
        """Pack, exchange (one all-gather) and merge already computed local
        results (tensors [nq, k], [nq, k], [nq] -- or [S, nq, k], [S, nq, k],
        [S, nq] for S local shards -- written on `stream`).  The
        packed words, the gathered buffer and the merged outputs are allocated
        with `stream` current, so their zero-fills, the pack, the collective
        and the merge are all ordered on it; the inputs are recorded on it so
        the caching allocator cannot hand their memory out while it still
        reads them."""
        t = self.torch
        with self._on(stream) as st:
            if st is not None:
                for x in (ids, dists, n):
                    x.record_stream(st)
            if ids.dim() == 3:
                packed = t.stack([self.pack(t, ids[s], dists[s], n[s], k, stream) for s in range(ids.shape[0])])
            else:
                packed = self.pack(t, ids, dists, n, k, stream)
            g = exchange_packed(t, self.dist, packed)
            return self.merge(t, g, self.offsets, k, stream)

    def _out(self, nq, k):
        t = self.torch
        S = len(self.indexes)
        lead = (S,) if S > 1 else ()
        return (t.zeros(lead + (nq, k), dtype=t.int32, device=self.device),
                t.zeros(lead + (nq, k), dtype=t.float32, device=self.device),
                t.zeros(lead + (nq,), dtype=t.int32, device=self.device))

    def _each(self, seeds, seed_off):
        """(index, slice selector) for every local shard; given seeds name one
        shard's local ids, so they are taken only with one local shard."""
        if len(self.indexes) > 1 and seeds is not None:
            raise ValueError("ShardedIndex: given seeds are local ids of one shard; with %d local shards use tree "
                             "or random seeds, or search each shard and call merge_local" % len(self.indexes))
        if len(self.indexes) == 1:
            return [(self.indexes[0], None)]
        return [(ix, s) for s, ix in enumerate(self.indexes)]

    def search_device(self, d_queries, query_bytes, nq, k, epsilon, seeds=None, seed_off=None, stream=None,
                      visited_hash_log2=0, edge_size=-1, seed_mode=None):
        """Local graph search of nq device queries on every local shard (one
        after another on `stream`), then the exchange and merge; returns
        global (ids, dists, n) tensors."""
        from .device import SEED_GIVEN, SEED_TREE
        with self._on(stream):  # the outputs' zero-fill is ordered before the search on `stream`
            ids, ds, n = self._out(nq, k)
        mode = seed_mode if seed_mode is not None else (SEED_GIVEN if seeds is not None else SEED_TREE)
        for ix, s in self._each(seeds, seed_off):
            oi, od, on = (ids, ds, n) if s is None else (ids[s], ds[s], n[s])
            ix.search_device(d_queries, query_bytes, nq, oi.data_ptr(), od.data_ptr(), on.data_ptr(), None,
                             k=k, epsilon=epsilon, edge_size=edge_size, seed_mode=mode, d_seeds=seeds,
                             d_seed_off=seed_off, stream=stream, visited_hash_log2=visited_hash_log2)
        return self.merge_local(ids, ds, n, k, stream)

    def qg_search_device(self, d_queries, query_bytes, nq, k, epsilon, result_expansion=3.0, seeds=None,
                         seed_off=None, stream=None, visited_hash_log2=-1, seed_mode=None):
        """C5's form: the NGTQG search (QuantizedGraph.h:354-372) of nq device
        queries on every local shard's quantized graph (exact rerank of
        k * expansion included), then the same exchange and merge of the
        reranked top-k."""
        from .device import SEED_GIVEN, SEED_TREE
        with self._on(stream):
            ids, ds, n = self._out(nq, k)
        mode = seed_mode if seed_mode is not None else (SEED_GIVEN if seeds is not None else SEED_TREE)
        for ix, s in self._each(seeds, seed_off):
            oi, od, on = (ids, ds, n) if s is None else (ids[s], ds[s], n[s])
            ix.qg_search_device(d_queries, query_bytes, nq, oi.data_ptr(), od.data_ptr(), on.data_ptr(), None,
                                k=k, epsilon=epsilon, result_expansion=result_expansion, seed_mode=mode,
                                d_seeds=seeds, d_seed_off=seed_off, stream=stream,
                                visited_hash_log2=visited_hash_log2)
        return self.merge_local(ids, ds, n, k, stream)


class RcclShardComm(object):
    """The C ABI's sharded search (shard_api.cpp) for callers without
    torch.distributed: an RCCL communicator of one rank per GPU, and one call
    that searches the batch on this rank's shard, all-gathers the packed
    per-shard top-k and merges them on the device."""
    ID_BYTES = 128

    @staticmethod
    def unique_id():
        import ctypes
        L = lib()
        buf = (ctypes.c_uint8 * RcclShardComm.ID_BYTES)()
        if L.ngt_amd_shard_unique_id(buf, RcclShardComm.ID_BYTES) != 0:
            raise NativeError(L.ngt_amd_last_error().decode())
        return bytes(buf)

    def __init__(self, device, rank, world, uid):
        import ctypes
        self.L = lib()
        self.world = world
        self.h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * len(uid)).from_buffer_copy(uid)
        if self.L.ngt_amd_shard_comm_create(ctypes.byref(self.h), device, rank, world, buf, len(uid)) != 0:
            raise NativeError(self.L.ngt_amd_last_error().decode())

    def set_offsets(self, offsets):
        """Store every rank's id offset on the device once; later searches
        pass offsets=None and only enqueue (ngt_amd_shard_comm_set_offsets)."""
        off = np.ascontiguousarray(offsets, dtype=np.uint32)
        if self.L.ngt_amd_shard_comm_set_offsets(self.h, off.ctypes.data) != 0:
            raise NativeError(self.L.ngt_amd_last_error().decode())

    def synchronize(self, stream=None):
        """Wait for the enqueued sharded searches; raises if any shard's
        search overflowed (ngt_amd_shard_comm_synchronize)."""
        if self.L.ngt_amd_shard_comm_synchronize(self.h, stream) != 0:
            raise NativeError(self.L.ngt_amd_last_error().decode())

    def search_device(self, index, d_queries, query_bytes, nq, offsets, d_ids, d_dists, d_n, k=10, epsilon=0.1,
                      radius=-1.0, edge_size=-1, seed_mode=0, d_seeds=None, d_seed_off=None, stream=None,
                      visited_hash_log2=0, qg=False, result_expansion=3.0):
        """offsets: every rank's id offset (copied, and the call synchronizes),
        or None after set_offsets (the call only enqueues)."""
        import ctypes
        from ._sigs import QgSearchParams, SearchParams
        off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint32)
        if qg:
            prm = QgSearchParams(k, epsilon, result_expansion, radius, seed_mode, visited_hash_log2)
            fn = self.L.ngt_amd_sharded_qg_search_device
        else:
            prm = SearchParams(k, epsilon, radius, edge_size, seed_mode, 0, visited_hash_log2, 0)
            fn = self.L.ngt_amd_sharded_search_device
        if fn(self.h, index.h, ctypes.byref(prm), d_queries, query_bytes, nq, d_seeds, d_seed_off,
              None if off is None else off.ctypes.data, d_ids, d_dists, d_n, stream) != 0:
            raise NativeError(self.L.ngt_amd_last_error().decode())

    def close(self):
        if self.h:
            self.L.ngt_amd_shard_comm_destroy(self.h)
            self.h = None
