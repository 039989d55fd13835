"""Object repository sharded across GPUs (BASELINE config C4).

One process per GPU.  Rank r holds shard r -- objects with global ids
``offset_r + 1 .. offset_r + n_r`` as its own index (rows, graph) in HBM --
and every rank searches every query on its shard.  The one exchange step is
an all-gather of the per-shard result lists (``k`` x {uint32 id, float
distance} per query, RCCL over xGMI when the process group is ``nccl``),
after which every rank merges the lists on its device with
``ngt_amd_merge_results_device`` (ObjectDistance ordering: distance, then
global id -- the result one index over the union would rank).

The exchange is backend-agnostic (torch.distributed collectives on tensors of
the merge's device); the CPU tests run it over ``gloo``.
"""
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
    """All ranks' shard offsets, in rank order."""
    world = dist.get_world_size()
    t = torch.tensor([offset], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [int(x.item()) for x in out]


def exchange(torch, dist, ids, dists, n):
    """All-gather of the local result lists: [nq, k] ids/dists and [nq] counts
    -> [world, nq, k] and [world, nq] on every rank (one collective per array,
    Q*k*8 B per rank)."""
    world = dist.get_world_size()
    out = []
    for t in (ids, dists, n):
        # rank-major concatenation along dim 0 (the layout every backend accepts)
        g = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(g, t.contiguous())
        out.append(g.view((world,) + tuple(t.shape)))
    return tuple(out)


def merge_device(torch, g_ids, g_d, g_n, offsets, k, stream=None):
    """Device merge of gathered shard lists (ngt_amd_merge_results_device)."""
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
    DeviceIndex (ids 1..n_r local); `offset` its global id offset."""

    def __init__(self, torch, dist, index, offset, device, merge=merge_device):
        self.torch, self.dist, self.index = torch, dist, index
        self.device = device
        self.offsets = gather_offsets(torch, dist, offset, device)
        self.merge = merge

    def merge_local(self, ids, dists, n, k, stream=None):
        """Exchange + merge of already computed local results (tensors)."""
        g_ids, g_d, g_n = exchange(self.torch, self.dist, ids, dists, n)
        return self.merge(self.torch, g_ids, g_d, g_n, self.offsets, k, stream)

    def search_device(self, d_queries, query_bytes, nq, k, epsilon, seeds=None, seed_off=None, stream=None,
                      visited_hash_log2=0, edge_size=-1, seed_mode=None):
        """Local graph search of nq device queries on this shard, then the
        exchange and merge; returns global (ids, dists, n) tensors."""
        from .device import SEED_GIVEN, SEED_TREE
        torch = self.torch
        ids = torch.zeros((nq, k), dtype=torch.int32, device=self.device)
        ds = torch.zeros((nq, k), dtype=torch.float32, device=self.device)
        n = torch.zeros((nq,), dtype=torch.int32, device=self.device)
        mode = seed_mode if seed_mode is not None else (SEED_GIVEN if seeds is not None else SEED_TREE)
        self.index.search_device(d_queries, query_bytes, nq, ids.data_ptr(), ds.data_ptr(), n.data_ptr(), None,
                                 k=k, epsilon=epsilon, edge_size=edge_size, seed_mode=mode, d_seeds=seeds,
                                 d_seed_off=seed_off, stream=stream, visited_hash_log2=visited_hash_log2)
        return self.merge_local(ids, ds, n, k, stream)
