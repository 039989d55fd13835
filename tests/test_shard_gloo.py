"""The multi-GPU path (repository sharded one shard per rank)
rehearsed on CPU with world_size 2 over gloo: shard bounds, the all-gather of
per-shard result lists and the global-id merge must reproduce one index over
the union.  Per-shard results come from the oracle's exact linear search
(test infrastructure); the merge here is a numpy checker of the device
merge's contract (tests/test_gpu_shard.py runs the device merge itself)."""
import os
import socket

import numpy as np
import pytest

import oracle_py as O
from ngt_amd.shard import ShardedIndex, shard_bounds

N, DIM, NQ, K = 1500, 16, 12, 10


def _data():
    rng = np.random.default_rng(42)
    rows = np.zeros((N + 1, DIM), np.float32)
    rows[1:] = rng.random((N, DIM), dtype=np.float32)
    # exact ties across shards: duplicate vectors in both halves
    rows[N - 3] = rows[5]
    rows[N - 2] = rows[6]
    qs = rng.random((NQ, DIM), dtype=np.float32)
    qs[0] = rows[5]
    return rows, qs


def numpy_pack(torch, ids, dists, n, k, stream=None):
    """Checker of ngt_amd_pack_results_device's contract: distance bits << 32 |
    local id per valid slot, 0 for empty slots."""
    i = ids.numpy().view(np.uint32).astype(np.uint64)
    d = dists.numpy().view(np.uint32).astype(np.uint64)
    valid = (np.arange(k)[None, :] < n.numpy()[:, None]) & (i != 0)
    return torch.from_numpy(np.where(valid, (d << np.uint64(32)) | i, np.uint64(0)).view(np.int64))


def numpy_merge(torch, g_packed, offsets, k, stream=None):
    """Checker of ngt_amd_merge_packed_device's contract."""
    w = g_packed.numpy().view(np.uint64)
    world, nq = w.shape[0], w.shape[1]
    out_i = torch.zeros((nq, k), dtype=torch.int32)
    out_d = torch.zeros((nq, k), dtype=torch.float32)
    out_n = torch.zeros((nq,), dtype=torch.int32)
    for q in range(nq):
        cand = []
        for s in range(world):
            for j in range(k):
                x = int(w[s, q, j])
                if x:
                    d = np.array([x >> 32], np.uint32).view(np.float32)[0]
                    cand.append((float(d), (x & 0xFFFFFFFF) + offsets[s]))
        cand.sort()
        for j, (d, i) in enumerate(cand[:k]):
            out_i[q, j] = i
            out_d[q, j] = d
        out_n[q] = min(k, len(cand))
    return out_i, out_d, out_n


class _Shard(object):
    """Stand-in for a DeviceIndex on CPU tensors: search_device writes the
    shard's precomputed local results through the output pointers, as the
    library writes device memory."""

    def __init__(self, ids, ds, n):
        self.ids, self.ds, self.n = ids, ds, n
        self.calls = 0

    def search_device(self, d_queries, query_bytes, nq, d_ids, d_dists, d_n, d_counters, **kw):
        import ctypes
        assert nq == self.n.shape[0]
        ctypes.memmove(d_ids, self.ids.ctypes.data, self.ids.nbytes)
        ctypes.memmove(d_dists, self.ds.ctypes.data, self.ds.nbytes)
        ctypes.memmove(d_n, self.n.ctypes.data, self.n.nbytes)
        self.calls += 1


def _worker(rank, world, port, q, per_rank=1, via_search=False):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows, qs = _data()
        # S = per_rank local shards: rank r holds shards r*S .. r*S+S-1
        offs, all_ids, all_ds, all_n = [], [], [], []
        for s in range(per_rank):
            off, cnt = shard_bounds(N, world * per_rank, rank * per_rank + s)
            shard = np.zeros((cnt + 1, DIM), np.float32)
            shard[1:] = rows[off + 1:off + 1 + cnt]
            ids = np.zeros((NQ, K), np.int32)
            ds = np.zeros((NQ, K), np.float32)
            n = np.zeros(NQ, np.int32)
            for i in range(NQ):
                oi, od = O.linear_search("l2", shard, qs[i], K)[:2]
                n[i] = len(oi)
                ids[i, :n[i]] = oi
                ds[i, :n[i]] = od
            offs.append(off)
            all_ids.append(ids)
            all_ds.append(ds)
            all_n.append(n)
        if via_search:
            # ShardedIndex.search_device searches EVERY local shard
            shards = [_Shard(all_ids[s], all_ds[s], all_n[s]) for s in range(per_rank)]
            sx = ShardedIndex(torch, dist, shards if per_rank > 1 else shards[0], offs if per_rank > 1 else offs[0],
                              torch.device("cpu"), pack=numpy_pack, merge=numpy_merge)
            gi, gd, gn = sx.search_device(None, 0, NQ, K, 0.1)
            assert all(sh.calls == 1 for sh in shards)
        elif per_rank == 1:
            sx = ShardedIndex(torch, dist, None, offs[0], torch.device("cpu"), pack=numpy_pack, merge=numpy_merge)
            gi, gd, gn = sx.merge_local(torch.from_numpy(all_ids[0]), torch.from_numpy(all_ds[0]),
                                        torch.from_numpy(all_n[0]), K)
        else:
            sx = ShardedIndex(torch, dist, [None] * per_rank, offs, torch.device("cpu"), pack=numpy_pack,
                              merge=numpy_merge)
            gi, gd, gn = sx.merge_local(torch.from_numpy(np.stack(all_ids)), torch.from_numpy(np.stack(all_ds)),
                                        torch.from_numpy(np.stack(all_n)), K)
        q.put((rank, offs, None, sx.offsets, gi.numpy(), gd.numpy(), gn.numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_partition():
    for n, w in [(10, 3), (1_000_000, 8), (7, 8), (12_500_000, 8)]:
        spans = [shard_bounds(n, w, r) for r in range(w)]
        assert sum(c for _, c in spans) == n
        assert spans[0][0] == 0
        for (o0, c0), (o1, _) in zip(spans, spans[1:]):
            assert o1 == o0 + c0


@pytest.mark.timeout(300)
@pytest.mark.parametrize("per_rank,via_search", [(1, False), (3, False), (1, True), (3, True)])
def test_sharded_search_equals_union_gloo(per_rank, via_search):
    """world 2; per_rank 3: every rank holds three shards (C4/C5's index
    served as several shards per GPU), six lists merged per query.
    via_search: through ShardedIndex.search_device, which must search every
    local shard (not only the first) before the one all-gather."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, per_rank, via_search)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    outs = []
    t0 = time.time()
    while len(outs) < 2 and time.time() - t0 < 240:
        try:
            outs.append(q.get(timeout=2))
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert len(outs) == 2
    outs.sort()
    rows, qs = _data()
    assert outs[0][3] == outs[1][3] == outs[0][1] + outs[1][1]
    assert outs[0][3] == [shard_bounds(N, 2 * per_rank, s)[0] for s in range(2 * per_rank)]
    for rank, off, cnt, offsets, gi, gd, gn in outs:
        for i in range(NQ):
            oi, od = O.linear_search("l2", rows, qs[i], K)[:2]
            assert int(gn[i]) == len(oi)
            assert list(gi[i, :gn[i]]) == list(oi), (rank, i)
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32))
