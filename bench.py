#!/usr/bin/env python3
"""bench.py -- NGT distance hot path on MI355X.

Metric (BASELINE.json): QPS at recall@10 = 0.95 on 1M x 128-d float L2
(config 2: 1M synthetic U[0,1) vectors, ONNG-style graph, 1 x MI355X), plus the
search kernel's achieved HBM GB/s against the 8 TB/s peak.

A *step* = one batched best-first search (NeighborhoodGraph::searchReadOnlyGraph
semantics, lib/NGT/Graph.cpp:398-495) of the 10,000-query batch over the index,
with queries, seeds, objects and graph already resident in HBM.

Untimed setup: deterministic splitmix64 data (base seed 0x4E4754, queries
base+1), graph construction (exact kNN by torch GEMM + top-k, then the
ONNG-style out/in edge selection), exact ground truth with the HIP linear
search, and an epsilon sweep to the smallest epsilon with recall@10 >= 0.95.

Multi-GPU (torchrun): every rank searches its own 10,000-query batch on its own
replica of the index ("replicas", weak scaling); no collective sits in the
data path.  Timing: barrier + synchronize on both sides of exactly K steps, max
over ranks, rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASE_SEED = 0x4E4754
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# data: splitmix64 -> float((x >> 40) * 2^-24), identical in every container
# ---------------------------------------------------------------------------
def splitmix_uniform(n, d, seed, chunk=1 << 22):
    out = np.empty(n * d, np.float32)
    gamma = np.uint64(0x9E3779B97F4A7C15)
    m1, m2 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)
    with np.errstate(over="ignore"):
        for s in range(0, n * d, chunk):
            e = min(n * d, s + chunk)
            z = np.uint64(seed) + (np.arange(s + 1, e + 1, dtype=np.uint64) * gamma)
            z = (z ^ (z >> np.uint64(30))) * m1
            z = (z ^ (z >> np.uint64(27))) * m2
            z = z ^ (z >> np.uint64(31))
            out[s:e] = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))
    return out.reshape(n, d)


# ---------------------------------------------------------------------------
# graph construction (setup only; SURVEY.md 8(f) row 1 is the native builder)
# ---------------------------------------------------------------------------
def build_graph(torch, X, knn_k, out_deg, in_deg, max_deg, dev, chunk=4096):
    """X: [N, D] float32 on device (objects 1..N).  Returns CSR (offsets[N+2],
    edges) over ids 1..N with each list sorted by (distance, id)."""
    N = X.shape[0]
    norms = (X * X).sum(1)
    knn_i = torch.empty((N, knn_k), dtype=torch.int32, device=dev)
    knn_d = torch.empty((N, knn_k), dtype=torch.float32, device=dev)
    t0 = time.time()
    for s in range(0, N, chunk):
        e = min(N, s + chunk)
        d = torch.addmm(norms[None, :], X[s:e], X.t(), beta=1.0, alpha=-2.0)
        d += norms[s:e, None]
        r = torch.arange(e - s, device=dev)
        d[r, r + s] = float("inf")
        v, i = torch.topk(d, knn_k, dim=1, largest=False, sorted=True)
        knn_i[s:e] = i.to(torch.int32)
        knn_d[s:e] = v.clamp_min(0).sqrt()
        del d, v, i
    torch.cuda.synchronize()
    log("kNN(%d) over %d objects in %.1f s" % (knn_k, N, time.time() - t0))
    # ONNG-style edge selection (GraphReconstructor::reconstructGraph idea):
    # first `out_deg` neighbours as outgoing edges, reverse edges from every node
    # that has v among its first `in_deg` neighbours.
    src = torch.arange(N, device=dev, dtype=torch.int64)
    fs = src[:, None].expand(N, out_deg).reshape(-1)
    fd = knn_i[:, :out_deg].reshape(-1).to(torch.int64)
    fw = knn_d[:, :out_deg].reshape(-1)
    rs = knn_i[:, :in_deg].reshape(-1).to(torch.int64)
    rd = src[:, None].expand(N, in_deg).reshape(-1)
    rw = knn_d[:, :in_deg].reshape(-1)
    s_all = torch.cat([fs, rs])
    d_all = torch.cat([fd, rd])
    w_all = torch.cat([fw, rw])
    del fs, fd, fw, rs, rd, rw
    # dedup (src, dst)
    key = s_all * N + d_all
    key, order = torch.sort(key)
    keep = torch.ones_like(key, dtype=torch.bool)
    keep[1:] = key[1:] != key[:-1]
    order = order[keep]
    s_all, d_all, w_all = s_all[order], d_all[order], w_all[order]
    # sort each list by (distance, id): stable sorts, least significant first
    o = torch.argsort(d_all, stable=True)
    s_all, d_all, w_all = s_all[o], d_all[o], w_all[o]
    o = torch.argsort(w_all, stable=True)
    s_all, d_all, w_all = s_all[o], d_all[o], w_all[o]
    o = torch.argsort(s_all, stable=True)
    s_all, d_all = s_all[o], d_all[o]
    # cap the degree
    counts = torch.bincount(s_all, minlength=N)
    starts = torch.cumsum(counts, 0) - counts
    rank = torch.arange(s_all.numel(), device=dev) - starts[s_all]
    m = rank < max_deg
    s_all, d_all = s_all[m], d_all[m]
    counts = torch.bincount(s_all, minlength=N)
    offsets = torch.zeros(N + 2, dtype=torch.int64, device=dev)
    offsets[2:] = torch.cumsum(counts, 0)   # node v (1-based) -> offsets[v]..offsets[v+1]
    edges = (d_all + 1).to(torch.int32)      # 1-based ids
    torch.cuda.synchronize()
    log("graph: %d edges, mean degree %.1f, max %d (%.1f s)" % (
        edges.numel(), edges.numel() / N, int(counts.max()), time.time() - t0))
    return offsets, edges


def random_seeds(nrows, nq, seed_size):
    """GraphIndex::getRandomSeeds (lib/NGT/Index.h:775-801) over the process
    rand() stream (the reference never reseeds it for graph-only search)."""
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    repo = nrows - 1
    seeds = np.zeros((nq, seed_size), np.uint32)
    for q in range(nq):
        got = []
        while len(got) < seed_size:
            r = (float(libc.rand()) + 1.0) / (2147483647.0 + 2.0)
            idx = int(np.floor(repo * r)) + 1
            if idx not in got:
                got.append(idx)
        seeds[q] = got
    return seeds


def recall_at(ids, gt, k):
    hit = 0
    for a, b in zip(ids[:, :k], gt[:, :k]):
        hit += len(set(a.tolist()) & set(b.tolist()))
    return hit / float(gt.shape[0] * k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--target", type=float, default=0.95)
    ap.add_argument("--knn", type=int, default=128)
    ap.add_argument("--out-deg", type=int, default=48)
    ap.add_argument("--in-deg", type=int, default=96)
    ap.add_argument("--max-deg", type=int, default=160)
    ap.add_argument("--seed-size", type=int, default=10)
    ap.add_argument("--eps", type=str, default="")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--visited", type=int, default=-1,
                    help="visited set: -1 HBM bitmap (this workload visits ~1e5 ids/query), 0 LDS hash")
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from ngt_amd.device import COUNTERS, SEED_GIVEN, DeviceIndex

    N, D, NQ, K = args.n, args.dim, args.nq, args.k
    dp = ((D - 1) // 16 + 1) * 16
    t0 = time.time()
    base = splitmix_uniform(N, D, BASE_SEED)
    qry = splitmix_uniform(NQ, D, BASE_SEED + 1 + rank * 0x1000)
    log("data generated in %.1f s" % (time.time() - t0))

    # HBM layout: padded row-major slab, row 0 = dummy (ObjectRepository.h:37-40)
    rows = torch.zeros((N + 1, dp), dtype=torch.float32, device=dev)
    rows[1:, :D] = torch.from_numpy(base).to(dev)
    qdev = torch.zeros((NQ, dp), dtype=torch.float32, device=dev)
    qdev[:, :D] = torch.from_numpy(qry).to(dev)
    offsets, edges = build_graph(torch, rows[1:, :D], args.knn, args.out_deg, args.in_deg, args.max_deg, dev)

    ix = DeviceIndex("l2", "float", D, device=local)
    ix.set_objects_device(rows.data_ptr(), N + 1)
    ix.set_graph_device(offsets.data_ptr(), edges.data_ptr(), edges.numel())
    ix.set_search_property(0, 30, 20, args.seed_size, 0)

    # exact ground truth with the HIP linear search (linearSearch semantics)
    t0 = time.time()
    gt_i = torch.zeros((NQ, K), dtype=torch.int32, device=dev)
    gt_d = torch.zeros((NQ, K), dtype=torch.float32, device=dev)
    gt_n = torch.zeros((NQ,), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ix.linear_search_device(qdev.data_ptr(), dp * 4, NQ, K, gt_i.data_ptr(), gt_d.data_ptr(), gt_n.data_ptr(),
                            stream=stream)
    torch.cuda.synchronize()
    gt = gt_i.cpu().numpy()
    log("ground truth in %.1f s" % (time.time() - t0))

    seeds = random_seeds(N + 1, NQ, args.seed_size)
    d_seeds = torch.from_numpy(seeds.reshape(-1).astype(np.int32)).to(dev)
    d_soff = torch.arange(0, NQ + 1, dtype=torch.int64, device=dev) * args.seed_size
    out_i = torch.zeros((NQ, K), dtype=torch.int32, device=dev)
    out_d = torch.zeros((NQ, K), dtype=torch.float32, device=dev)
    out_n = torch.zeros((NQ,), dtype=torch.int32, device=dev)
    cnt = torch.zeros((NQ, COUNTERS), dtype=torch.int64, device=dev)

    def run(eps):
        ix.search_device(qdev.data_ptr(), dp * 4, NQ, out_i.data_ptr(), out_d.data_ptr(), out_n.data_ptr(),
                         cnt.data_ptr(), k=K, epsilon=eps, edge_size=0, seed_mode=SEED_GIVEN,
                         d_seeds=d_seeds.data_ptr(), d_seed_off=d_soff.data_ptr(), stream=stream,
                         visited_hash_log2=args.visited)

    # epsilon search (ngt eval semantics: mean recall@k over the queries):
    # the smallest epsilon whose recall@k reaches the target, by bisection
    sweep = []

    def measure(eps):
        run(eps)
        torch.cuda.synchronize()
        r = recall_at(out_i.cpu().numpy(), gt, K)
        sweep.append((round(eps, 5), r, ix.last_search_kernel_ms()))
        log("eps %.4f recall@%d %.4f kernel %.2f ms" % (eps, K, r, sweep[-1][2]))
        return r

    if args.eps:
        cands = [float(x) for x in args.eps.split(",")]
        chosen = cands[-1]
        for eps in cands:
            if measure(eps) >= args.target:
                chosen = eps
                break
    else:
        lo, hi = 0.0, 0.05
        while measure(hi) < args.target and hi < 2.0:
            lo, hi = hi, hi * 2
        while hi - lo > 0.002:
            mid = 0.5 * (lo + hi)
            if measure(mid) >= args.target:
                hi = mid
            else:
                lo = mid
        chosen = hi
    rec = measure(chosen)
    if dist is not None:
        # all ranks use the largest epsilon any rank needed
        t = torch.tensor([chosen], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        chosen = float(t.item())
        run(chosen)
        torch.cuda.synchronize()
        rec = recall_at(out_i.cpu().numpy(), gt, K)

    for _ in range(args.warmup):
        run(chosen)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run(chosen)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-launch duration of the search kernel: HIP events recorded by the
    # library around the kernel on the stream it runs on
    kms = []
    for _ in range(3):
        run(chosen)
        torch.cuda.synchronize()
        kms.append(ix.last_search_kernel_ms())
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    qps = NQ * world * args.steps / elapsed

    # roofline of the search kernel: algorithmic bytes per launch
    # B(q) = U(q)*Dp*4 + E(q)*4 + Dp*4 + k*8   
    c = cnt.cpu().numpy().astype(np.float64)
    U, E = c[:, 0].sum(), c[:, 4].sum()
    if "stamps" in os.environ.get("NGT_AMD_LIB", ""):
        tot = c[:, [5, 6, 7, 3]].mean(0)
        log("phase cycles/query: pop %.3g adjacency+visited %.3g eval %.3g accept+rest %.3g (sum %.3g)" % (
            tot[0], tot[1], tot[2], tot[3], tot.sum()))
    alg_bytes = U * dp * 4 + E * 4 + NQ * (dp * 4 + K * 8)
    kernel_ms = float(np.mean(kms)) if kms else float("nan")
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = measured_traffic("kNN%d out%d in%d max%d" % (args.knn, args.out_deg, args.in_deg, args.max_deg), chosen)

    cpu = None
    if rank == 0 and not args.no_cpu and world == 1:
        cpu = cpu_baseline(rows, offsets, edges, qry, seeds, chosen, K, dp, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "QPS at recall@10=0.95, 1M x 128-d float L2; achieved HBM GB/s vs peak",
            "value": qps,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (splitmix64 U[0,1), seed 0x4E4754)",
            "config": {"workload": "C2: %d x %d float L2 graph search, %d queries/step/GPU, k=%d" % (N, D, NQ, K),
                       "recall_at_10": rec, "epsilon": chosen, "edge_size": "all",
                       "graph": "kNN%d out%d in%d max%d" % (args.knn, args.out_deg, args.in_deg, args.max_deg),
                       "seeds": "getRandomSeeds (%d)" % args.seed_size,
                       "distance_computations_per_query": U / NQ,
                       "expansions_per_query": float(c[:, 2].mean()),
                       "edges_read_per_query": E / NQ,
                       "max_unchecked_per_query": float(c[:, 5].max()),
                       "visited_set": "hbm-bitmap" if args.visited < 0 else "lds-hash",
                       "parallelism": "replicas x%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                         "kernel_ms": kernel_ms, "algorithmic_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "sweep": sweep,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def measured_traffic(graph, eps):
    """HBM bytes per launch of the search kernel from the committed PMC passes
    (profiles/traffic.json, written from rocprofv3 FETCH_SIZE/WRITE_SIZE) for this
    exact graph and epsilon; NGT_BENCH_TRAFFIC_BYTES overrides; else None."""
    tf = os.environ.get("NGT_BENCH_TRAFFIC_BYTES")
    if tf:
        return float(tf)
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "traffic.json")) as f:
            entries = json.load(f)["entries"]
    except (OSError, ValueError, KeyError):
        return None
    for e in entries:
        if e["graph"] == graph and abs(e["epsilon"] - eps) < 1e-7:
            return float(e["traffic_bytes"])
    return None


def cpu_baseline(rows, offsets, edges, qry, seeds, eps, K, dp, budget_s):
    """The oracle restatement (scalar, 1 thread) on a bounded sample of the
    same workload: same graph, seeds and epsilon, queries until the budget."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    t0 = time.time()
    h_rows = rows.cpu().numpy()
    h_off = offsets.cpu().numpy().astype(np.uint64)
    h_edges = edges.cpu().numpy().astype(np.uint32)
    log("cpu baseline: host copy %.1f s" % (time.time() - t0))
    done = 0
    t0 = time.perf_counter()
    while done < qry.shape[0] and time.perf_counter() - t0 < budget_s:
        q = np.zeros(dp, np.float32)
        q[:qry.shape[1]] = qry[done]
        O.search("l2", h_rows, h_off, h_edges, q, seeds[done], K, np.float32(eps), edge_size=0)
        done += 1
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": "%d of the 10000 queries (same graph, seeds, epsilon), oracle/ngt_oracle.c "
                      "searchReadOnlyGraph restatement, 1 thread, %.1f s" % (done, el)}


if __name__ == "__main__":
    main()
