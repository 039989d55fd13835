"""GPU side of the sharded path: the device merge kernels
(ngt_amd_merge_results_device, ngt_amd_pack_results_device +
ngt_amd_merge_packed_device) against a numpy merge of the same lists, and the
full ShardedIndex pipeline (local exact or NGTQG search -> one packed RCCL
all-gather -> device merge) on a one-rank nccl group, against the oracle and
the reference's own NGTQG results."""
import os
import socket

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def np_merge(ids, ds, n, offsets, k):
    S, nq, _ = ids.shape
    oi = np.zeros((nq, k), np.uint32)
    od = np.zeros((nq, k), np.float32)
    on = np.zeros(nq, np.uint32)
    for q in range(nq):
        c = sorted((float(ds[s, q, j]), int(ids[s, q, j]) + offsets[s]) for s in range(S) for j in range(n[s, q]))
        for j, (d, i) in enumerate(c[:k]):
            oi[q, j], od[q, j] = i, d
        on[q] = min(k, len(c))
    return oi, od, on


@pytest.mark.parametrize("S,k", [(2, 10), (8, 10), (8, 100), (3, 1)])
def test_merge_kernel_matches_numpy(S, k):
    import torch
    from ngt_amd.shard import merge_device
    rng = np.random.default_rng(S * 100 + k)
    nq = 300
    ids = np.zeros((S, nq, k), np.uint32)
    ds = np.zeros((S, nq, k), np.float32)
    n = rng.integers(0, k + 1, size=(S, nq)).astype(np.uint32)
    n[:, 0] = k
    offsets = [s * 1000 for s in range(S)]
    for s in range(S):
        for q in range(nq):
            d = np.sort(rng.integers(0, 50, k).astype(np.float32) / np.float32(7))  # many exact ties
            ids[s, q] = rng.choice(np.arange(1, 1000), k, replace=False)
            order = np.lexsort((ids[s, q], d))
            ids[s, q], ds[s, q] = ids[s, q][order], d[order]
    dev = torch.device("cuda:0")
    gi, gd, gn = merge_device(torch, torch.from_numpy(ids.view(np.int32)).to(dev), torch.from_numpy(ds).to(dev),
                              torch.from_numpy(n.view(np.int32)).to(dev), offsets, k)
    torch.cuda.synchronize()
    ei, ed, en = np_merge(ids, ds, n, offsets, k)
    gi, gd, gn = gi.cpu().numpy().view(np.uint32), gd.cpu().numpy(), gn.cpu().numpy()
    assert np.array_equal(gn, en)
    for q in range(nq):
        assert list(gi[q, :gn[q]]) == list(ei[q, :en[q]]), q
        assert np.array_equal(gd[q, :gn[q]].view(np.uint32), ed[q, :en[q]].view(np.uint32))


@pytest.mark.parametrize("S,k", [(2, 10), (8, 10), (8, 100), (3, 1)])
def test_pack_and_packed_merge_match_numpy(S, k):
    """The exchange message (ngt_amd_pack_results_device: distance bits << 32 |
    local id, 0 = empty) and its merge (ngt_amd_merge_packed_device) against a
    numpy merge, with ragged lists, empty lists and exact distance ties."""
    import torch
    from ngt_amd.shard import merge_packed_device, pack_device
    rng = np.random.default_rng(S * 31 + k)
    nq = 257
    ids = np.zeros((S, nq, k), np.uint32)
    ds = np.zeros((S, nq, k), np.float32)
    n = rng.integers(0, k + 1, size=(S, nq)).astype(np.uint32)
    n[:, 0] = k
    n[:, 1] = 0
    offsets = [s * 1000 for s in range(S)]
    for s in range(S):
        for q in range(nq):
            d = np.sort(rng.integers(0, 50, k).astype(np.float32) / np.float32(7))
            ids[s, q] = rng.choice(np.arange(1, 1000), k, replace=False)
            order = np.lexsort((ids[s, q], d))
            ids[s, q], ds[s, q] = ids[s, q][order], d[order]
    dev = torch.device("cuda:0")
    packed = []
    for s in range(S):
        packed.append(pack_device(torch, torch.from_numpy(ids[s].view(np.int32)).to(dev),
                                  torch.from_numpy(ds[s]).to(dev), torch.from_numpy(n[s].view(np.int32)).to(dev), k))
    g = torch.stack(packed)
    torch.cuda.synchronize()
    w = g.cpu().numpy().view(np.uint64)
    for s in range(S):
        for q in range(0, nq, 17):
            for j in range(k):
                exp = (int(ds[s, q, j].view(np.uint32)) << 32 | int(ids[s, q, j])) if j < n[s, q] else 0
                assert int(w[s, q, j]) == exp, (s, q, j)
    gi, gd, gn = merge_packed_device(torch, g, offsets, k)
    torch.cuda.synchronize()
    ei, ed, en = np_merge(ids, ds, n, offsets, k)
    gi, gd, gn = gi.cpu().numpy().view(np.uint32), gd.cpu().numpy(), gn.cpu().numpy()
    assert np.array_equal(gn, en)
    for q in range(nq):
        assert list(gi[q, :gn[q]]) == list(ei[q, :en[q]]), q
        assert np.array_equal(gd[q, :gn[q]].view(np.uint32), ed[q, :en[q]].view(np.uint32))


def test_sharded_index_one_rank_nccl():
    import torch
    import torch.distributed as dist
    from ngt_amd.device import SEED_GIVEN, DeviceIndex
    from ngt_amd.shard import ShardedIndex, shard_bounds
    from test_gpu_parity import _random_graph
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        n, dim, deg, nq = 4000, 32, 16, 64
        rows, offs, edges = _random_graph(n, dim, deg, 9)
        off, cnt = shard_bounds(n - 1, 1, 0)
        ix = DeviceIndex("l2", "float", dim)
        ix.set_objects(rows)
        ix.set_graph(offs, edges)
        rng = np.random.default_rng(4)
        qs = rng.random((nq, dim), dtype=np.float32)
        seeds = np.stack([rng.choice(np.arange(1, n), 8, replace=False) for _ in range(nq)]).astype(np.uint32)
        d_q = torch.from_numpy(qs).to(dev)
        d_s = torch.from_numpy(seeds.reshape(-1).view(np.int32)).to(dev)
        d_o = torch.arange(0, nq + 1, dtype=torch.int64, device=dev) * 8
        sx = ShardedIndex(torch, dist, ix, off, dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        gi, gd, gn = sx.search_device(d_q.data_ptr(), dim * 4, nq, 10, 0.2, seeds=d_s.data_ptr(),
                                      seed_off=d_o.data_ptr(), stream=stream, edge_size=0, seed_mode=SEED_GIVEN)
        torch.cuda.synchronize()
        ref_t = (gi.clone(), gd.clone(), gn.clone())
        gi, gd, gn = gi.cpu().numpy().view(np.uint32), gd.cpu().numpy(), gn.cpu().numpy()
        for i in range(nq):
            oid, od, _ = O.search("l2", rows, offs, edges, qs[i], seeds[i], 10, np.float32(0.2))
            assert list(gi[i, :gn[i]]) == list(oid + off), i
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), od.view(np.uint32))
        # the same search, pack, collective and merge on a side stream: outputs
        # allocated and zero-filled there, inputs recorded on it (ngt_amd/shard.py)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        for _ in range(3):
            si, sd, sn = sx.search_device(d_q.data_ptr(), dim * 4, nq, 10, 0.2, seeds=d_s.data_ptr(),
                                          seed_off=d_o.data_ptr(), stream=side.cuda_stream, edge_size=0,
                                          seed_mode=SEED_GIVEN)
        side.synchronize()
        assert torch.equal(si, ref_t[0]) and torch.equal(sd.view(torch.int32), ref_t[1].view(torch.int32))
        assert torch.equal(sn, ref_t[2])
        ix.close()

        # C5's form: the NGTQG search on the shard, then the same exchange and
        # merge -- on the reference's C1 quantized graph, against the
        # reference's own NGTQG::Index::search results (tests/golden/c1_qg)
        from test_gpu_qg import device_qg, state
        _, _, _, _, _, _, _, z, meta, dim, _ = state("c1_qg")
        qix = device_qg("c1_qg")
        qsq = z["queries"].astype(np.float32)
        d_q = torch.from_numpy(qsq).to(dev)
        sq = ShardedIndex(torch, dist, qix, 0, dev)
        from ngt_amd.device import SEED_TREE
        for key in ("10_0.05_3", "20_0.03_3", "10_0.1_2"):
            k, eps, exp = key.split("_")
            gi, gd, gn = sq.qg_search_device(d_q.data_ptr(), dim * 4, len(qsq), int(k), float(eps),
                                             result_expansion=float(exp), stream=stream, seed_mode=SEED_TREE)
            torch.cuda.synchronize()
            gi, gd, gn = gi.cpu().numpy().view(np.uint32), gd.cpu().numpy(), gn.cpu().numpy()
            for qi in range(len(qsq)):
                n = int(z["n_" + key][qi])
                ref_ids = z["ids_" + key][qi][:n]
                valid = ref_ids != 0  # the reference pads a short rerank with {0, 0}
                assert int(gn[qi]) == int(valid.sum()), (key, qi)
                assert list(gi[qi, :gn[qi]]) == list(ref_ids[valid]), (key, qi)
                assert np.array_equal(gd[qi, :gn[qi]].view(np.uint32),
                                      z["dist_" + key][qi][:n][valid].view(np.uint32)), (key, qi)
        qix.close()
    finally:
        dist.destroy_process_group()


def test_rccl_sharded_search_c_abi():
    """The C ABI's sharded search (ngt_amd_sharded_search_device /
    _qg_search_device: per-shard search, pack, one RCCL all-gather, device
    merge) on a one-rank communicator: exact search against the oracle with a
    global id offset, NGTQG search against the reference's C1 results."""
    import torch
    from ngt_amd.device import SEED_GIVEN, SEED_TREE, DeviceIndex
    from ngt_amd.shard import RcclShardComm
    from test_gpu_parity import _random_graph
    dev = torch.device("cuda:0")
    comm = RcclShardComm(0, 0, 1, RcclShardComm.unique_id())
    try:
        n, dim, deg, nq, k, off = 4000, 32, 16, 64, 10, 1000
        rows, offs, edges = _random_graph(n, dim, deg, 11)
        ix = DeviceIndex("l2", "float", dim)
        ix.set_objects(rows)
        ix.set_graph(offs, edges)
        rng = np.random.default_rng(5)
        qs = rng.random((nq, dim), dtype=np.float32)
        seeds = np.stack([rng.choice(np.arange(1, n), 8, replace=False) for _ in range(nq)]).astype(np.uint32)
        d_q = torch.from_numpy(qs).to(dev)
        d_s = torch.from_numpy(seeds.reshape(-1).view(np.int32)).to(dev)
        d_o = torch.arange(0, nq + 1, dtype=torch.int64, device=dev) * 8
        oi = torch.zeros((nq, k), dtype=torch.int32, device=dev)
        od = torch.zeros((nq, k), dtype=torch.float32, device=dev)
        on = torch.zeros((nq,), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        comm.search_device(ix, d_q.data_ptr(), dim * 4, nq, [off], oi.data_ptr(), od.data_ptr(), on.data_ptr(), k=k,
                           epsilon=0.2, edge_size=0, seed_mode=SEED_GIVEN, d_seeds=d_s.data_ptr(),
                           d_seed_off=d_o.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        gi, gd, gn = oi.cpu().numpy().view(np.uint32), od.cpu().numpy(), on.cpu().numpy()
        for i in range(nq):
            oid, odist, _ = O.search("l2", rows, offs, edges, qs[i], seeds[i], k, np.float32(0.2))
            assert list(gi[i, :gn[i]]) == list(oid + off), i
            assert np.array_equal(gd[i, :gn[i]].view(np.uint32), odist.view(np.uint32))

        # asynchronous form: offsets stored once, two batches enqueued back to
        # back on a side stream, one synchronize
        comm.set_offsets([off])
        side = torch.cuda.Stream(dev)
        outs = [tuple(torch.full(sh, -1, dtype=dt, device=dev) for sh, dt in
                      (((nq, k), torch.int32), ((nq, k), torch.float32), ((nq,), torch.int32))) for _ in range(2)]
        side.wait_stream(torch.cuda.current_stream(dev))
        for a, b, c in outs:
            comm.search_device(ix, d_q.data_ptr(), dim * 4, nq, None, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                               k=k, epsilon=0.2, edge_size=0, seed_mode=SEED_GIVEN, d_seeds=d_s.data_ptr(),
                               d_seed_off=d_o.data_ptr(), stream=side.cuda_stream)
        comm.synchronize(side.cuda_stream)
        for a, b, c in outs:
            assert np.array_equal(a.cpu().numpy().view(np.uint32), gi)
            assert np.array_equal(b.cpu().numpy().view(np.uint32), gd.view(np.uint32))
            assert np.array_equal(c.cpu().numpy(), gn)
        ix.close()

        # a shard whose unchecked-set spill overflows (capacity forced to one
        # key): the flag travels with the all-gathered message and the
        # synchronize reports it instead of a silently truncated list
        from ngt_amd import NativeError
        os.environ["NGT_AMD_SPILL_CAP"] = "1"
        os.environ["NGT_AMD_CQ_CAP"] = "64"
        try:
            ix2 = DeviceIndex("l2", "float", dim)
            ix2.set_objects(rows)
            ix2.set_graph(offs, edges)
            a, b, c = outs[0]
            comm.search_device(ix2, d_q.data_ptr(), dim * 4, nq, None, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                               k=k, epsilon=1.0, edge_size=0, seed_mode=SEED_GIVEN, d_seeds=d_s.data_ptr(),
                               d_seed_off=d_o.data_ptr(), stream=stream)
            with pytest.raises(NativeError, match="truncated"):
                comm.synchronize(stream)
            comm.synchronize(stream)  # the flag is cleared once reported
            ix2.close()
        finally:
            del os.environ["NGT_AMD_SPILL_CAP"]
            del os.environ["NGT_AMD_CQ_CAP"]

        from test_gpu_qg import device_qg, state
        _, _, _, _, _, _, _, z, meta, dim, _ = state("c1_qg")
        qix = device_qg("c1_qg")
        qsq = z["queries"].astype(np.float32)
        d_q = torch.from_numpy(qsq).to(dev)
        for key in ("10_0.05_3", "20_0.03_3"):
            k, eps, exp = key.split("_")
            k = int(k)
            oi = torch.zeros((len(qsq), k), dtype=torch.int32, device=dev)
            od = torch.zeros((len(qsq), k), dtype=torch.float32, device=dev)
            on = torch.zeros((len(qsq),), dtype=torch.int32, device=dev)
            comm.search_device(qix, d_q.data_ptr(), dim * 4, len(qsq), [0], oi.data_ptr(), od.data_ptr(),
                               on.data_ptr(), k=k, epsilon=float(eps), seed_mode=SEED_TREE, stream=stream, qg=True,
                               result_expansion=float(exp))
            torch.cuda.synchronize()
            gi, gd, gn = oi.cpu().numpy().view(np.uint32), od.cpu().numpy(), on.cpu().numpy()
            for qi in range(len(qsq)):
                n = int(z["n_" + key][qi])
                ref_ids = z["ids_" + key][qi][:n]
                valid = ref_ids != 0
                assert int(gn[qi]) == int(valid.sum()), (key, qi)
                assert list(gi[qi, :gn[qi]]) == list(ref_ids[valid]), (key, qi)
                assert np.array_equal(gd[qi, :gn[qi]].view(np.uint32),
                                      z["dist_" + key][qi][:n][valid].view(np.uint32)), (key, qi)
        qix.close()
    finally:
        comm.close()
