#!/usr/bin/env python3
"""bench.py -- NGT distance hot path on MI355X.

Metric (BASELINE.json): QPS at recall@10 = 0.95 on 1M x 128-d float L2
(config C2: 1M synthetic U[0,1) vectors, ONNG-style graph, 1 x MI355X), plus the
search kernel's achieved HBM GB/s against the 8 TB/s peak.

A *step* = one batched best-first search (NeighborhoodGraph::searchReadOnlyGraph
semantics, lib/NGT/Graph.cpp:398-495) of the 10,000-query batch over the index,
with queries, seeds, objects and graph already resident in HBM.

Modes (`--mode`; the default is the headline):
  exact  C2 (or `--config c3`: 1M x 960 cosine).  With N ranks every rank
         searches its own 10,000-query batch on its own replica ("replicas",
         weak scaling, no collective in the data path).
  qg     the NGTQG quantized graph (QuantizedGraph.h:192-320) on the same
         graph: 4-bit codes, dsub = 1 (M = 128 subspaces x 16 centroids),
         exact rerank of k * result_expansion (C5's per-GPU search shape).
  capi   the drop-in C API on the C2 index: single-query ngt_search_index
         latency (sequential calls) and the throughput of --threads
         concurrent single-query callers (coalesced into batched launches,
         ngt_amd/csrc/coalesce.h); its own JSON line, not the headline.
  shard  C4's form: the object repository sharded one shard per rank (--n
         objects per rank, global ids offset by rank), every rank searches
         every query on its shard, one RCCL all-gather of the packed per-shard
         top-k and a device merge (ngt_amd/shard.py); QPS of the whole
         sharded index.  With --qg, C5's form: every shard is an NGTQG
         quantized graph (per-shard quantizer, encoder, quantized graph).

Untimed setup: deterministic splitmix64 data (base seed 0x4E4754, queries
base+1), graph construction (exact kNN by torch GEMM + top-k, then the
ONNG-style out/in edge selection), exact ground truth with the HIP linear
search, and an epsilon sweep to the smallest epsilon with recall@10 >= 0.95.
Timing: barrier + synchronize on both sides of exactly K steps, max over
ranks, rank 0 prints one JSON line.
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
# MI355X_MICROARCH.md 'Indexed rows: gather into LDS': uniformly random rows of a
# 38 MB table (Infinity-Cache resident) gathered at 8.6 TB/s chip-wide -- the
# measured rate for a table the Infinity Cache holds (a lower bound of its peak)
IC_GATHER_GBS = 8600.0
HEADLINE = "QPS at recall@10=0.95, 1M x 128-d float L2; achieved HBM GB/s vs peak"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# data: splitmix64 -> float((x >> 40) * 2^-24), identical in every container.
# Element e of the stream (row-major over the whole data set) depends only on
# e, so a shard generates its own rows without the others.
# ---------------------------------------------------------------------------
def splitmix_uniform(n, d, seed, row0=0, chunk=1 << 22):
    out = np.empty(n * d, np.float32)
    gamma = np.uint64(0x9E3779B97F4A7C15)
    m1, m2 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)
    e0 = row0 * d
    with np.errstate(over="ignore"):
        for s in range(0, n * d, chunk):
            e = min(n * d, s + chunk)
            z = np.uint64(seed) + (np.arange(e0 + s + 1, e0 + e + 1, dtype=np.uint64) * gamma)
            z = (z ^ (z >> np.uint64(30))) * m1
            z = (z ^ (z >> np.uint64(27))) * m2
            z = z ^ (z >> np.uint64(31))
            out[s:e] = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))
    return out.reshape(n, d)


# ---------------------------------------------------------------------------
# graph construction (setup only; SURVEY.md 8(f) row 1 is the native builder)
# ---------------------------------------------------------------------------
def build_graph(torch, X, knn_k, out_deg, in_deg, max_deg, dev, cosine=False, chunk=4096):
    """X: [N, D] float32 on device (objects 1..N).  Returns CSR (offsets[N+2],
    edges) over ids 1..N with each list sorted by (distance, id)."""
    N = X.shape[0]
    if cosine:
        Xn = X / X.norm(dim=1, keepdim=True).clamp_min(1e-30)
    else:
        norms = (X * X).sum(1)
    knn_i = torch.empty((N, knn_k), dtype=torch.int32, device=dev)
    knn_d = torch.empty((N, knn_k), dtype=torch.float32, device=dev)
    t0 = time.time()
    for s in range(0, N, chunk):
        e = min(N, s + chunk)
        if cosine:
            d = 1.0 - Xn[s:e] @ Xn.t()
        else:
            d = torch.addmm(norms[None, :], X[s:e], X.t(), beta=1.0, alpha=-2.0)
            d += norms[s:e, None]
        r = torch.arange(e - s, device=dev)
        d[r, r + s] = float("inf")
        v, i = torch.topk(d, knn_k, dim=1, largest=False, sorted=True)
        knn_i[s:e] = i.to(torch.int32)
        knn_d[s:e] = v.clamp_min(0) if cosine else v.clamp_min(0).sqrt()
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


# the epsilon sweep stops doubling once one launch takes this long (the sweep
# is setup, not the measurement; a multi-second launch means the graph needs
# an epsilon that no serving configuration would use)
SWEEP_KERNEL_MS_CAP = float(os.environ.get("NGT_BENCH_SWEEP_MS_CAP", "3000"))


def tune_epsilon(measure, target, eps_list=None, lo=0.0, hi=0.05, tol=0.0005, last_ms=None):
    """Smallest epsilon whose mean recall@k reaches the target (ngt eval
    semantics, Optimizer.h:400): given candidates, or by doubling + bisection.
    last_ms() = the kernel time of the latest measurement: the doubling stops
    at SWEEP_KERNEL_MS_CAP (the result is then the last epsilon tried, whose
    recall the line reports)."""
    if eps_list:
        for eps in eps_list:
            if measure(eps) >= target:
                return eps
        return eps_list[-1]
    while measure(hi) < target and hi < 4.0:
        if last_ms is not None and last_ms() > SWEEP_KERNEL_MS_CAP:
            log("eps sweep: %.1f ms per launch at eps %.4f exceeds the %.0f ms cap; stopping" % (
                last_ms(), hi, SWEEP_KERNEL_MS_CAP))
            return hi
        # a search's cost grows steeply with epsilon on high-dimensional data:
        # double while launches are cheap, then creep up
        grow = 2.0 if last_ms is None or last_ms() < SWEEP_KERNEL_MS_CAP / 100.0 else 1.25
        lo, hi = hi, hi * grow
    while hi - lo > tol:
        mid = 0.5 * (lo + hi)
        if measure(mid) >= target:
            hi = mid
        else:
            lo = mid
    return hi


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`bench.py --gpus N` run without a torch.distributed launcher: start N
    fresh rank processes of this same command (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment), one per GPU.  This parent
    never imports torch and never touches a GPU, and it does not exec: the
    ranks are children, rank 0's JSON line is relayed to stdout and the exit
    status is the first failing rank's (the others are then stopped)."""
    import signal
    import subprocess
    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    import threading
    chunks = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log("rank %d exited with %d; stopping the others" % (procs.index(p), code))
                stop()
        time.sleep(0.05)
    reader.join(10)
    out = b"".join(chunks).decode(errors="replace")
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if rc == 0 and lines:
        print(lines[-1], flush=True)
    elif rc == 0:
        log("rank 0 printed no result line")
        rc = 1
    return rc


def dry_run(args, result_out):
    """The launcher's contract without a GPU (tests/test_bench_launcher.py):
    every rank joins a gloo group, runs --steps timed steps of rank-dependent
    length between barriers, and rank 0 prints the line with the max over
    ranks, the ranks seen and the per-rank times."""
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if os.environ.get("NGT_BENCH_DRYRUN_FAIL_RANK") == str(rank):
        raise SystemExit("bench: dry run: rank %d fails on request" % rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ones = torch.ones(1)
    dist.all_reduce(ones)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.01 * (rank + 1))
    dist.barrier()
    elapsed = time.perf_counter() - t0
    ranks = [None] * world
    dist.all_gather_object(ranks, {"rank": rank, "pid": os.getpid(), "elapsed": elapsed,
                                   "local_rank": int(os.environ.get("LOCAL_RANK", "0"))})
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": world * args.steps / float(t.item()), "unit": "steps/s",
                          "n_gpus": int(ones.item()), "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": float(t.item()) / args.steps * 1e3, "ranks": ranks}),
              file=result_out, flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--shard-n", type=int, default=1_250_000, help="shard line: objects per shard")
    ap.add_argument("--shard-count", type=int, default=8, help="shard line: shards of the whole index")
    ap.add_argument("--shard-qg-line", choices=["on", "off"], default="on",
                    help="with the shard line: also C5's form (every shard an NGTQG quantized graph) over the same "
                         "shards, as its 'qg_form' key")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: gloo ranks time rank-dependent sleeps (no search)")
    ap.add_argument("--shard-line", choices=["auto", "on", "off"], default="auto",
                    help="attach C4's 10M index sharded over the ranks (8/N shards of 1.25M per rank) as the "
                         "'shard' key; auto = on for the default C2 run with more than one rank")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", choices=["exact", "qg", "shard", "capi"], default="exact")
    ap.add_argument("--threads", type=int, default=128,
                    help="C-API lines: concurrent callers T (runs at 1, T and 2T threads; the serving grid has one "
                         "worker per CU but one)")
    ap.add_argument("--qg", action="store_true", help="with --mode shard: NGTQG shards (C5's form)")
    ap.add_argument("--config", choices=["c2", "c3"], default="c2")
    ap.add_argument("--n", type=int, default=0, help="objects (per shard in --mode shard)")
    ap.add_argument("--shards-per-gpu", type=int, default=1, help="--mode shard: shards each rank holds")
    ap.add_argument("--shard-sample", type=int, default=2000, help="--mode shard: oracle parity sample (queries)")
    ap.add_argument("--dim", type=int, default=0)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--target", type=float, default=0.95)
    ap.add_argument("--graph", choices=["knn", "anng"], default="knn",
                    help="knn: exact kNN graph built in setup (out/in edges); anng: this library's own "
                         "ngt_create_index ANNG (GraphAndTreeIndex::createIndex on the device)")
    ap.add_argument("--anng-edges", type=int, default=10, help="--graph anng: edgeSizeForCreation (ngt create -E)")
    ap.add_argument("--anng-batch", type=int, default=200,
                    help="--graph anng: batchSizeForCreation (ngt create -b, Command.cpp:41; int16, Graph.h:517)")
    ap.add_argument("--anng-dir", type=str, default="",
                    help="--graph anng: keep the saved index here, or open it if an earlier run saved it")
    ap.add_argument("--edge-size", type=int, default=None,
                    help="sc.edgeSize of the searches (getEdgeSize, Graph.h:675-692): -1 = the index's "
                         "EdgeSizeForSearch (an `ngt create` index: 40), 0 = every edge; default -1 for "
                         "--graph anng, 0 for the kNN graph")
    ap.add_argument("--seeds", choices=["random", "tree"], default=None,
                    help="random: getRandomSeeds (graph-only search); tree: the DVP tree's leaf "
                         "(GraphAndTreeIndex::search, `ngt search`'s default); default tree for --graph anng")
    # the kNN surrogate graph (build_graph): kNN256 -> 64 out + 224 in edges,
    # <= 256 per node (the padded adjacency's limit).  Round 5's sweep
    # (profiles/r5e, r5k, r5l): denser graphs need fewer expansions for the same
    # recall (C2: 327 vs 576 per query, 16.2 vs 18.7 ms per search than kNN128
    # out48 in96 max160)
    ap.add_argument("--knn", type=int, default=256)
    ap.add_argument("--out-deg", type=int, default=64)
    ap.add_argument("--in-deg", type=int, default=224)
    ap.add_argument("--max-deg", type=int, default=256)
    ap.add_argument("--seed-size", type=int, default=10)
    ap.add_argument("--eps", type=str, default="")
    ap.add_argument("--expansion", type=float, default=3.0,
                    help="NGTQG result_expansion (ngtqg_search's default 3.0, NGTQ/Capi.cpp:44)")
    ap.add_argument("--qg-expansions", type=str, default="",
                    help="--mode qg: result_expansion candidates; epsilon is tuned to the target for each and the "
                         "one whose full-batch launch is shortest is timed")
    ap.add_argument("--qg-line", choices=["auto", "on", "off"], default="auto",
                    help="attach NGTQG (ngtqg quantize on the device) over the same saved 1M ANNG as the 'qg' key "
                         "(a child run of --mode qg --graph anng); auto = on for the default single-GPU C2 run")
    ap.add_argument("--qg-edges", type=int, default=128, help="NGTQG max edges per node")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--sweep-nq", type=int, default=2000, help="queries per epsilon-sweep launch")
    ap.add_argument("--latency-queries", type=int, default=100, help="single-query launches timed after the bench")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pmc-launches", type=int, default=0,
                    help="after the epsilon is set: run this many launches of the timed configuration and exit")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams consecutive steps alternate over (default 3, or 1 when three streams' "
                         "visited scratch -- rows x 16 waves per CU each -- would exceed 0.6 of the HBM)")
    ap.add_argument("--streams-ab", type=str, default="",
                    help="experiment: after the timed steps, time the same steps over each of these stream counts "
                         "(logged and reported as config.stream_ab_ms_per_step; the line's value is --streams)")
    ap.add_argument("--anng-line", choices=["auto", "on", "off"], default="auto",
                    help="attach the NGT-built index's line (a child run of --graph anng) as the 'anng' key; "
                         "auto = on for the default single-GPU C2 run")
    ap.add_argument("--capi-line", choices=["auto", "on", "off"], default="auto",
                    help="with --graph anng: the drop-in C API (ngt_open_index + ngt_search_index from a pthreads C "
                         "client) on the same saved index as the 'capi' key; auto = on for the 1M ANNG")
    ap.add_argument("--c3-line", choices=["auto", "on", "off"], default="auto",
                    help="attach C3 (1M x 960 cosine, a child run of --config c3) as the 'c3' key; auto = on for "
                         "the default single-GPU C2 run")
    ap.add_argument("--visited", type=int, default=-2,
                    help="visited set: -2 HBM epochs of accepted ids, -1 HBM epochs of every evaluated id "
                         "(C2 visits ~1e5 ids/query), 0 LDS hash")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start the N ranks ourselves (before torch)
        return launch_ranks(args)
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%s" % (args.gpus, os.environ.get("WORLD_SIZE")))
    # stdout carries exactly one JSON line: everything else written to fd 1
    # (RCCL's init banner, library chatter) goes to stderr
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.dry_run:
        return dry_run(args, result_out)
    qgm = args.mode == "qg" or (args.mode == "shard" and args.qg)
    if args.edge_size is None:
        args.edge_size = -1 if args.graph == "anng" else 0
    if args.seeds is None:
        # an index with a DVP tree seeds from it: GraphAndTreeIndex::search and
        # NGTQG::Index::search (QuantizedGraph.h:354-372) alike
        args.seeds = "tree" if args.graph == "anng" else "random"
    es_prop = 40 if args.graph == "anng" else 0  # the prf's EdgeSizeForSearch (Command.cpp:40)
    if qgm and args.visited == -2:
        args.visited = -1  # the QG search marks accepted ids only by definition (QuantizedGraph.h:241-266)
    c3 = args.config == "c3"
    if not args.n:
        args.n = 1_250_000 if args.mode == "shard" else 1_000_000
    if not args.dim:
        args.dim = 960 if c3 else 128
    metric = "cosine" if c3 else "l2"

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    n_ranks = 1
    if world > 1 or args.mode == "shard":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        # n_gpus = the ranks that actually joined the RCCL group
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)
        n_ranks = int(t.item())
        if n_ranks != args.gpus:
            raise SystemExit("bench: %d ranks joined RCCL, --gpus %d" % (n_ranks, args.gpus))

    if args.streams is None:
        # every stream has its own launch context with slots x rows visited
        # bytes; three of them at 12.5M rows (51 GB each) squeeze each other's
        # slot counts, and a long launch gains nothing from the overlap
        props = torch.cuda.get_device_properties(dev)
        per_ctx = (args.n + 1) * 16 * props.multi_processor_count
        args.streams = 3 if 3 * per_ctx <= 0.6 * props.total_memory else 1
    from ngt_amd.device import COUNTERS, SEED_GIVEN, SEED_TREE, DeviceIndex
    if args.mode == "capi":
        return capi_bench(args, torch, dev, result_out)
    if args.mode == "shard":
        return shard_bench(args, torch, dist, dev, rank, world, local, result_out, qgm)

    N, D, NQ, K = args.n, args.dim, args.nq, args.k
    dp = ((D - 1) // 16 + 1) * 16
    shard = args.mode == "shard"
    t0 = time.time()
    if shard:
        from ngt_amd.shard import ShardedIndex
        offset = rank * N
        base = splitmix_uniform(N, D, BASE_SEED, row0=offset)
        qry = splitmix_uniform(NQ, D, BASE_SEED + 1)
    else:
        offset = 0
        base = splitmix_uniform(N, D, BASE_SEED)
        qry = splitmix_uniform(NQ, D, BASE_SEED + 1 + rank * 0x1000)
    log("data generated in %.1f s" % (time.time() - t0))

    # HBM layout: padded row-major slab, row 0 = dummy (ObjectRepository.h:37-40)
    rows = torch.zeros((N + 1, dp), dtype=torch.float32, device=dev)
    rows[1:, :D] = torch.from_numpy(base).to(dev)
    qraw = torch.from_numpy(qry).to(dev)
    build_s = None
    tree = None
    anng_check = None
    capi_dir = None
    capi_tmp = False
    if (args.graph == "anng" and args.mode == "exact" and world == 1 and not args.pmc_launches and N == 1_000_000
            and D == 128 and args.anng_batch == 200 and (args.capi_line == "on" or args.capi_line == "auto")):
        # the C-API line opens the index this run saves (ngt_save_index) from disk
        import tempfile
        if not args.anng_dir:
            capi_dir = args.anng_dir = tempfile.mkdtemp(prefix="ngt_anng_capi_")
            capi_tmp = True
        else:
            capi_dir = args.anng_dir
    if args.graph == "anng":
        # the index a user of `ngt create -d 128 -o f -D 2 -E <e>` gets, built
        # through the drop-in C API (ngt_create_graph_and_tree,
        # ngt_batch_append_index, ngt_create_index -> this library's device
        # construction, ngt_save_index), checked against the reference's own
        # build of the same data (tests/golden/c2_anng_ref.json), and searched
        # on the device index that handle serves (ngt_get_device_index)
        if N > 2_000_000 or args.anng_batch != 200:
            # an index too large to write in the reference's format per run (or
            # one built with another `ngt create -b` than the reference check's):
            # the same device construction, driven in id ranges with progress
            ix, offsets, edges, tree, build_s, anng_check, cx = build_anng_device(args, torch, dev, rows, N, D,
                                                                                 es_prop, local)
        else:
            ix, offsets, edges, tree, build_s, anng_check, cx = build_anng_capi(args, torch, dev, base, N, D, es_prop)
    else:
        ix = DeviceIndex(metric, "float", D, device=local)
        ix.set_objects_device(rows.data_ptr(), N + 1)
        offsets, edges = build_graph(torch, rows[1:, :D], args.knn, args.out_deg, args.in_deg, args.max_deg, dev,
                                     cosine=c3)
        ix.set_search_property(es_prop, 30, 20, args.seed_size, 0)
        ix.set_graph_device(offsets.data_ptr(), edges.data_ptr(), edges.numel())
    es_resolved = int(ix.resolve_edge_size(args.edge_size, 0.1))
    stream = torch.cuda.current_stream(dev).cuda_stream
    # queries prepared on the device like Index::allocateObject (pad; normalize
    # for the normalized metrics)
    qdev = torch.zeros((NQ, dp), dtype=torch.float32, device=dev)
    ix.prepare_queries_device(qraw.data_ptr(), NQ, qdev.data_ptr(), stream=stream)
    sx = ShardedIndex(torch, dist, ix, offset, dev) if shard else None

    # exact ground truth with the HIP linear search (linearSearch semantics)
    t0 = time.time()
    gt_i = torch.zeros((NQ, K), dtype=torch.int32, device=dev)
    gt_d = torch.zeros((NQ, K), dtype=torch.float32, device=dev)
    gt_n = torch.zeros((NQ,), dtype=torch.int32, device=dev)
    ix.linear_search_device(qdev.data_ptr(), dp * 4, NQ, K, gt_i.data_ptr(), gt_d.data_ptr(), gt_n.data_ptr(),
                            stream=stream)
    if shard:
        gt_i, gt_d, gt_n = sx.merge_local(gt_i, gt_d, gt_n, K, stream)
    torch.cuda.synchronize()
    gt = gt_i.cpu().numpy()
    log("ground truth in %.1f s" % (time.time() - t0))
    scan = None
    if not shard and not qgm:
        # the exact scan itself as a search method (recall 1.0): the batch
        # linear search timed on the same resident queries
        sms = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ix.linear_search_device(qdev.data_ptr(), dp * 4, NQ, K, gt_i.data_ptr(), gt_d.data_ptr(),
                                    gt_n.data_ptr(), stream=stream)
            e1.record()
            torch.cuda.synchronize()
            sms.append(e0.elapsed_time(e1))
        if not np.array_equal(gt_i.cpu().numpy(), gt):
            raise SystemExit("bench: exact scan not deterministic")
        ms = float(min(sms))
        macs = 3.0 * N * NQ * (dp + 16)  # bf16 hi/lo passes incl. the norm column
        scan = {"qps": NQ / (ms * 1e-3), "ms": ms, "recall_at_10": 1.0,
                "kernel": "ngt_scan_mfma_kernel (bf16 hi/lo MFMA filter + comparator recompute)" if K <= 16
                else "ngt_linear_scan_l2f_kernel",
                "effective_tflops": 3.0 * N * NQ * dp / (ms * 1e-3) / 1e12,
                "mfma_bf16_frac": 2.0 * macs / (ms * 1e-3) / 2.5e15}
        log("exact scan: %.2f ms per %d queries (%.0f QPS)" % (ms, NQ, scan["qps"]))

    if args.seeds == "tree":
        if tree is None:
            raise SystemExit("bench: --seeds tree needs an index with a DVP tree (--graph anng)")
        # GraphAndTreeIndex::getSeedsFromTree on the device, once (the seed
        # lists are the search's input, like the random ones below)
        seeds, d_seeds, d_soff = tree_seed_lists(ix, qdev, dp, NQ, K, dev, torch)
    else:
        seeds = random_seeds(N + 1, NQ, args.seed_size)
        d_seeds = torch.from_numpy(seeds.reshape(-1).astype(np.int32)).to(dev)
        d_soff = torch.arange(0, NQ + 1, dtype=torch.int64, device=dev) * args.seed_size
    # consecutive steps alternate over `--streams` HIP streams (each with its
    # own output buffers and, inside the library, its own launch scratch), so
    # a step's kernel starts while the previous step's last queries drain
    stream_ab = [int(x) for x in args.streams_ab.split(",")] if args.streams_ab else []
    nstreams = 1 if shard else max([1, args.streams] + stream_ab)
    streams = [stream] + [torch.cuda.Stream(dev).cuda_stream for _ in range(nstreams - 1)]
    bufs = [(torch.zeros((NQ, K), dtype=torch.int32, device=dev), torch.zeros((NQ, K), dtype=torch.float32, device=dev),
             torch.zeros((NQ,), dtype=torch.int32, device=dev), torch.zeros((NQ, COUNTERS), dtype=torch.int64, device=dev))
            for _ in range(nstreams)]
    out_i, out_d, out_n, cnt = bufs[0]
    result = {"ids": out_i}

    if qgm:
        # ngtqg quantize on the device: codebooks (dsub = 1, 16 centroids,
        # 1600-object sample as the reference's dynamic k-means), encoder,
        # quantized graph (QuantizedGraph.h:456-475)
        t0 = time.time()
        h_base = np.zeros((min(N, 1600) + 1, D), np.float32)
        h_base[1:] = base[:min(N, 1600)]
        qg_local = ix.qg_train_ngt(h_base, dsub=1)  # ngtqg_quantize's kmeansWithNGT codebooks
        t1 = time.time()
        ix.qg_encode(return_codes=False)
        ix.qg_build_graph(None, args.qg_edges)
        torch.cuda.synchronize()
        qg_record_bytes = int(ix.L.ngt_amd_qg_record_bytes(ix.h))
        log("quantizer (kmeansWithNGT, %d subspaces) %.1f s + encoder + quantized graph %.1f s (degree <= %d); "
            "packed search layout %.2f GB (%.0f B per node)" % (D, t1 - t0, time.time() - t1, ix.qg_max_degree(),
                                                               qg_record_bytes / 1e9, qg_record_bytes / max(1, N)))

    def run(eps, si=0, visited=None, nq=NQ):
        oi, od, on, oc = bufs[si]
        visited = args.visited if visited is None else visited
        if qgm:
            ix.qg_search_device(qdev.data_ptr(), dp * 4, nq, oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                                oc.data_ptr(), k=K, epsilon=eps, result_expansion=args.expansion,
                                seed_mode=SEED_GIVEN, d_seeds=d_seeds.data_ptr(), d_seed_off=d_soff.data_ptr(),
                                stream=streams[si], visited_hash_log2=visited)
            if shard:
                result["ids"] = sx.merge_local(out_i, out_d, out_n, K, stream)[0]
            return
        ix.search_device(qdev.data_ptr(), dp * 4, nq, oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                         oc.data_ptr(), k=K, epsilon=eps, edge_size=args.edge_size, seed_mode=SEED_GIVEN,
                         d_seeds=d_seeds.data_ptr(), d_seed_off=d_soff.data_ptr(), stream=streams[si],
                         visited_hash_log2=visited)
        if shard:
            result["ids"] = sx.merge_local(out_i, out_d, out_n, K, stream)[0]

    sweep = []
    # the sweep runs on the first `sweep_nq` queries (shards: the whole batch,
    # the merged recall needs every rank's results), the chosen epsilon is
    # then checked on the whole batch and raised in small steps if needed
    sweep_nq = NQ if shard else min(NQ, args.sweep_nq)

    def measure(eps, nq=None):
        nq = sweep_nq if nq is None else nq
        run(eps, nq=nq)
        torch.cuda.synchronize()
        r = recall_at(result["ids"].cpu().numpy()[:nq], gt[:nq], K)
        sweep.append((round(eps, 5), r, ix.last_search_kernel_ms(), nq))
        log("eps %.4f recall@%d %.4f kernel %.2f ms (%d queries)" % (eps, K, r, sweep[-1][2], nq))
        return r

    def tune():
        eps = tune_epsilon(measure, args.target, [float(x) for x in args.eps.split(",")] if args.eps else None,
                           last_ms=lambda: sweep[-1][2] * NQ / max(1, sweep[-1][3]))
        r = measure(eps, NQ)
        for _ in range(20):
            if r >= args.target or args.eps:
                break
            eps = round(eps * 1.02 + 1e-4, 5)
            r = measure(eps, NQ)
        return eps, r

    expansion_sweep = None
    if qgm and args.qg_expansions and not args.eps:
        # NGTQG's two knobs: for every result_expansion candidate the smallest
        # epsilon reaching the target, then the one whose whole-batch launch
        # (the last measurement of its tuning) is shortest
        expansion_sweep = []
        for ex in [float(x) for x in args.qg_expansions.split(",")]:
            args.expansion = ex
            eps_x, rec_x = tune()
            expansion_sweep.append({"result_expansion": ex, "epsilon": eps_x, "recall_at_10": rec_x,
                                    "kernel_ms": sweep[-1][2]})
            log("result_expansion %g: epsilon %.5f recall@%d %.4f, %.2f ms per %d-query launch" % (
                ex, eps_x, K, rec_x, sweep[-1][2], NQ))
        best = pick_expansion(expansion_sweep, args.target)
        args.expansion, chosen = best["result_expansion"], best["epsilon"]
        rec = measure(chosen, NQ)
    else:
        chosen, rec = tune()
    if dist is not None and not shard:
        # replicas: all ranks use the largest epsilon any rank needed
        t = torch.tensor([chosen], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        chosen = float(t.item())
        rec = measure(chosen, NQ)

    order_exp = os.environ.get("NGT_BENCH_ORDER", "")
    if order_exp and not shard and not qgm:
        # EXPERIMENT (never the product line): the single launch's tail against
        # the order queries are pulled in.  "oracle": longest first by the
        # expansions of the last run; "centroid": by the query's distance to
        # the data's mean (a cheap predictor).  Prints per-order kernel times.
        run(chosen)
        torch.cuda.synchronize()
        ne0 = cnt[:, 2].cpu().numpy().astype(np.float64)
        cen = rows[1:, :D].mean(0)
        dc = (qdev[:, :D] - cen).norm(dim=1).cpu().numpy()
        rr = np.corrcoef(dc, ne0)[0, 1]
        log("order experiment: corr(expansions, |q - mean|) = %.3f" % rr)
        dump = os.environ.get("NGT_BENCH_DUMP")
        if dump:
            np.savez(dump, expansions=ne0, counters=cnt.cpu().numpy(), epsilon=chosen, centroid_dist=dc)
        tree_mode = args.seeds == "tree"
        for name, perm in (("given", np.arange(NQ)), ("oracle", np.argsort(-ne0, kind="stable")),
                           ("centroid_asc", np.argsort(dc, kind="stable")),
                           ("centroid_desc", np.argsort(-dc, kind="stable"))):
            pt = torch.from_numpy(perm).to(dev)
            q2 = qdev[pt].contiguous()
            s2 = None if tree_mode else d_seeds.view(NQ, -1)[pt].contiguous().view(-1)
            ts = []
            for _ in range(3):
                oi, od, on, oc = bufs[0]
                ix.search_device(q2.data_ptr(), dp * 4, NQ, oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                                 oc.data_ptr(), k=K, epsilon=chosen, edge_size=args.edge_size,
                                 seed_mode=SEED_TREE if tree_mode else SEED_GIVEN,
                                 d_seeds=None if tree_mode else s2.data_ptr(),
                                 d_seed_off=None if tree_mode else d_soff.data_ptr(), stream=streams[0],
                                 visited_hash_log2=args.visited)
                torch.cuda.synchronize()
                ts.append(ix.last_search_kernel_ms())
            log("order %s: kernel %.2f ms (min of 3: %.2f)" % (name, float(np.mean(ts)), float(np.min(ts))))
        return
    if args.pmc_launches:
        # counter passes (scripts/pmc_r3.sh): exactly this many more launches of
        # the timed configuration, nothing else of the bench
        for _ in range(args.pmc_launches):
            run(chosen)
            torch.cuda.synchronize()
        print(json.dumps({"pmc_launches": args.pmc_launches, "epsilon": chosen, "recall_at_10": rec,
                          "launches_before": len(sweep), "kernel_ms_last": ix.last_search_kernel_ms()}),
              file=result_out, flush=True)
        return
    ns_timed = 1 if shard else max(1, args.streams)
    for i in range(max(args.warmup, ns_timed)):
        run(chosen, i % ns_timed)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run(chosen, i % ns_timed)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    stream_ms = {}
    for n in stream_ab:
        # EXPERIMENT (not the line's value): the same steps alternating over n streams
        for i in range(max(args.warmup, n)):
            run(chosen, i % n)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steps):
            run(chosen, i % n)
        torch.cuda.synchronize()
        stream_ms[n] = (time.perf_counter() - t1) / args.steps * 1e3
        log("streams %d: %.2f ms per step" % (n, stream_ms[n]))
    # per-launch duration of the search kernel: HIP events recorded by the
    # library around the kernel on the stream it runs on
    kms = []
    for _ in range(3):
        run(chosen)
        torch.cuda.synchronize()
        kms.append(ix.last_search_kernel_ms())
    filtered = (not qgm) and ix.last_search_filtered()
    budget = 0 if qgm else ix.last_search_budget()
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # replicas: every rank searched its own batch; shard: every rank searched
    # the same batch on its part of one index
    qps = NQ * (1 if shard else world) * args.steps / elapsed

    c = cnt.cpu().numpy().astype(np.float64)
    c_timed = c
    evals_per_query = None
    if not qgm and args.visited == -2:
        # The timed runs keep only accepted ids in the visited set, so their
        # counters include re-evaluations of rejected neighbours.  One more
        # run with every evaluated id in the set gives the reference's distinct
        # distance count U(q) for the algorithmic bytes -- and must return
        # exactly the same ids and distances.
        evals_per_query = float(c[:, 0].mean())
        fast = [t.clone() for t in (out_i, out_d, out_n)]
        run(chosen, 0, visited=-1)
        torch.cuda.synchronize()
        same = (torch.equal(fast[0], out_i) and torch.equal(fast[1].view(torch.int32), out_d.view(torch.int32))
                and torch.equal(fast[2], out_n))
        if not same:
            raise SystemExit("bench: accepted-only visited set changed the results")
        log("accepted-only visited set: results identical; %.0f evaluations/query vs %.0f distinct" % (
            evals_per_query, float(cnt[:, 0].double().mean())))
        c = cnt.cpu().numpy().astype(np.float64)
    ne = c[:, 2]
    log("expansions/query: mean %.0f p50 %.0f p90 %.0f p99 %.0f max %.0f" % (
        ne.mean(), np.percentile(ne, 50), np.percentile(ne, 90), np.percentile(ne, 99), ne.max()))
    la_form = -1 if qgm else ix.last_search_lookahead()
    if la_form >= 0 and "stamps" not in os.environ.get("NGT_AMD_LIB", ""):
        log("lookahead form %d: %.0f speculative expansions discarded/query (%.0f committed)" % (
            la_form, c[:, 3].mean(), ne.mean()))
    kernel_ms = float(np.mean(kms)) if kms else float("nan")
    graph = ("kNN%d out%d in%d max%d" % (args.knn, args.out_deg, args.in_deg, args.max_deg) if args.graph == "knn"
             else "ANNG E%d (ngt_create_index on the device)" % args.anng_edges
             + ("" if args.anng_batch == 200 else ", batchSizeForCreation %d" % args.anng_batch))
    if qgm:
        # B(q) = sum_exp ceil(deg/16)*16*(M/2) + deg*4 + (seeds + k*expansion)*Dp*4  
        me = (D + 1) // 2 * 2
        alg_bytes = c[:, 4].sum() * 8 * me + c[:, 0].sum() * 4 + c[:, 3].sum() * dp * 4 + NQ * (dp * 4 + K * 8)
        kname = "ngt_qg_search_kernel"
    elif filtered:
        # the filtered kernel's own minimum: every distinct neighbour's 1-byte
        # filter row, the f32 row of the seeds and of every neighbour the bound
        # could not reject, adjacency, query, results:
        # B(q) = (U(q) - S(q))*Dp + (S(q) + X(q))*Dp*4 + E(q)*4 + Dp*4 + k*8
        alg_bytes = ((c[:, 0] - c[:, 7]).sum() * dp + (c[:, 7] + c[:, 6]).sum() * dp * 4 + c[:, 4].sum() * 4
                     + NQ * (dp * 4 + K * 8))
        kname = "ngt_graph_search_kernel"
    else:
        # B(q) = U(q)*Dp*4 + E(q)*4 + Dp*4 + k*8   
        alg_bytes = c[:, 0].sum() * dp * 4 + c[:, 4].sum() * 4 + NQ * (dp * 4 + K * 8)
        kname = "ngt_graph_search_kernel"
    if not qgm and la_form >= 0:
        kname = "ngt_graph_search_la_kernel"  # the lookahead kernel (search_la.hip) ran the timed launches
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    literal = literal_bytes(c, dp, NQ, K, qgm, D)
    split = None
    if filtered and not qgm:
        # where the algorithmic bytes come from: the 1-byte filter copy (N x Dp
        # bytes, 128 MB at C2 -- a table the 256 MiB Infinity Cache holds) and
        # the f32 rows, adjacency, queries and results (tables beyond it)
        fbytes = (c[:, 0] - c[:, 7]).sum() * dp
        mall_table = (N + 1) * dp
        split = {"filter_copy_bytes": fbytes, "filter_copy_table_bytes": mall_table,
                 "filter_copy_fits_infinity_cache": mall_table <= 256 * 2 ** 20,
                 "other_bytes": alg_bytes - fbytes,
                 "other_gbs": (alg_bytes - fbytes) / (kernel_ms * 1e-3) / 1e9}
    traffic, tentry = measured_traffic(args.mode, args.config, graph, chosen, args.visited, filtered)
    if "stamps" in os.environ.get("NGT_AMD_LIB", "") and args.mode == "exact":
        tot = c[:, [5, 6, 1, 7, 3]].mean(0)
        if ix.last_search_lookahead() >= 0:
            log("lookahead phase cycles/query: pop+targets %.3g adjacency %.3g filter %.3g exact %.3g commit %.3g "
                "(sum %.3g); steps/query %.0f" % (tot[0], tot[1], tot[2], tot[3], tot[4], tot.sum(), c[:, 4].mean()))
        else:
            log("phase cycles/query: pop %.3g adjacency+visited %.3g filter %.3g eval %.3g accept+rest %.3g "
                "(sum %.3g)" % (tot[0], tot[1], tot[2], tot[3], tot[4], tot.sum()))
    if "lacount" in os.environ.get("NGT_AMD_LIB", "") and ix.last_search_lookahead() >= 0:
        m = c_timed.mean(0)  # the timed launches' (visited set as timed) counters
        log("lookahead line accounting/query: list entries %.0f, epoch probes %.0f, exact rows %.0f, spill keys "
            "written %.0f read %.0f, refills %.0f; expansions %.0f" % (m[7], m[6], m[4], m[1], m[3], m[5], m[2]))
    if "stamps" in os.environ.get("NGT_AMD_LIB", "") and args.mode == "qg":
        tot = c[:, [4, 5, 6, 7]].mean(0)
        log("phase cycles/query: pop %.3g ids %.3g codes+adc %.3g accept %.3g (sum %.3g)" % (
            tot[0], tot[1], tot[2], tot[3], tot.sum()))

    # single-query launches (the reference's callers issue one query at a
    # time, Capi.cpp:377-406): device time of nq=1 searches, sequentially
    latency = None
    if rank == 0 and not shard and not qgm and args.latency_queries > 0:
        lat = []
        lc = torch.zeros((args.latency_queries, COUNTERS), dtype=torch.int64, device=dev)
        for i in range(args.latency_queries):
            oi, od, on, _ = bufs[0]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ix.search_device(qdev[i:i + 1].data_ptr(), dp * 4, 1, oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                             lc[i:i + 1].data_ptr(), k=K, epsilon=chosen, edge_size=args.edge_size,
                             seed_mode=SEED_GIVEN, d_seeds=d_seeds.data_ptr(), d_seed_off=d_soff[i:i + 2].data_ptr(),
                             stream=stream, visited_hash_log2=0)
            e1.record()
            torch.cuda.synchronize()
            lat.append(e0.elapsed_time(e1))
        lat = np.array(lat)
        latency = {"queries": len(lat), "mean_ms": float(lat.mean()), "p50_ms": float(np.percentile(lat, 50)),
                   "p99_ms": float(np.percentile(lat, 99)), "form": ix.last_search_lookahead(),
                   "what": "one query per launch (nq=1), full visited set, device time incl. launch"}
        log("single-query launches: mean %.3f ms p50 %.3f p99 %.3f (lookahead form %d)" % (
            latency["mean_ms"], latency["p50_ms"], latency["p99_ms"], latency["form"]))
        lcc = lc.cpu().numpy().astype(np.float64)
        if "stamps" not in os.environ.get("NGT_AMD_LIB", ""):
            latency["expansions_mean"] = float(lcc[:, 2].mean())
        if "stamps" not in os.environ.get("NGT_AMD_LIB", ""):
            latency["stalled_pops_mean"] = float(lcc[:, 3].mean())
            log("single-query: %.0f expansions, %.0f of them waited for their list" % (
                lcc[:, 2].mean(), lcc[:, 3].mean()))
        else:
            tot = lcc[:, [5, 6, 1, 3, 7]].mean(0)
            sp = lcc[:, [0, 4, 2]].mean(0)
            log("single-query phase cycles (latency kernel): commit wave: pop %.3g wait %.3g list+visited %.3g "
                "accept %.3g feed %.3g (sum %.3g); speculation waves (summed): adjacency %.3g filter %.3g "
                "exact %.3g" % (tot[0], tot[1], tot[2], tot[3], tot[4], tot.sum(), sp[0], sp[1], sp[2]))
        if args.seeds == "tree" and args.edge_size == -1:
            # the same queries answered by the resident serving grid (what a
            # lone ngt_search_index call gets): host wall time per call
            served = []
            for i in range(args.latency_queries):
                t1 = time.perf_counter()
                r = ix.search_served(qry[i], k=K, epsilon=chosen)
                served.append(time.perf_counter() - t1)
                if r is None:
                    served = []
                    break
            if served:
                sv = np.array(served[1:] if len(served) > 1 else served) * 1e3
                latency["served_mean_ms"] = float(sv.mean())
                latency["served_p50_ms"] = float(np.percentile(sv, 50))
                log("single queries through the serving grid: mean %.3f ms p50 %.3f" % (
                    latency["served_mean_ms"], latency["served_p50_ms"]))

    cpu = parity = None
    if rank == 0 and not args.no_cpu and world == 1 and not shard:
        run(chosen, 0, visited=-1 if args.mode == "exact" and args.visited == -2 else None)
        torch.cuda.synchronize()
        full_cnt = cnt.cpu().numpy()
        run(chosen, 0)  # the timed configuration's own results
        torch.cuda.synchronize()
        gpu_out = (out_i.cpu().numpy().view(np.uint32), out_d.cpu().numpy(), out_n.cpu().numpy().view(np.uint32))
        cpu, parity = cpu_baseline(args, ix, rows, offsets, edges, qdev, seeds, chosen, metric, gpu_out, full_cnt,
                                   es_resolved=int(ix.resolve_edge_size(args.edge_size, chosen)),
                                   qg_local=qg_local if qgm else None)
        if scan is not None:
            scan["oracle_sample"] = scan_sample_check(rows, qdev, metric, K, gt_i, gt_d, gt_n)
        if cpu is not None:
            cpu["calibration"] = calibration()
    ref_check = None
    if rank == 0 and anng_check is not None and anng_check.get("reference"):
        ref_check = reference_fixture_check(ix, qdev, dp, K, dev, torch)
    capi = None
    if rank == 0 and capi_dir:
        capi = capi_anng_line(capi_dir, qry, gt, D, K, chosen, args.threads)
        if capi_tmp:
            import shutil
            shutil.rmtree(capi_dir, ignore_errors=True)

    if rank == 0:
        if args.mode == "exact" and not c3 and N > 2_000_000:
            metric_name = "QPS at recall@10=0.95, %d x %d-d float L2 on one GPU (C4's index as one graph)" % (N, D)
            workload = ("C4 on one GPU: %d x %d float L2, ONE device-built ANNG over all objects (not shards), "
                        "%d queries/step, k=%d" % (N, D, NQ, K))
        elif args.mode == "exact" and not c3:
            metric_name = HEADLINE
            workload = "C2: %d x %d float L2 graph search, %d queries/step/GPU, k=%d" % (N, D, NQ, K)
        elif args.mode == "exact":
            metric_name = "QPS at recall@10=0.95, 1M x 960-d float cosine; achieved HBM GB/s vs peak"
            workload = "C3: %d x %d float cosine graph search, %d queries/step/GPU, k=%d" % (N, D, NQ, K)
        elif args.mode == "qg":
            metric_name = "QPS at recall@10=0.95, %d x %d-d NGTQG quantized graph (L2); achieved HBM GB/s" % (N, D)
            workload = "C5 shape per GPU: %d x %d NGTQG (dsub=1, M=%d, 16 centroids), result_expansion %g, " \
                       "%d queries/step/GPU, k=%d" % (N, D, D, args.expansion, NQ, K)
        elif qgm:
            metric_name = "QPS at recall@10=0.95, %d x %d-d NGTQG sharded over %d GPUs" % (N * world, D, world)
            workload = "C5 form: %d objects per GPU shard (NGTQG dsub=1, M=%d, result_expansion %g), %d shards, " \
                       "%d queries/step over all shards, k=%d, one packed RCCL all-gather of per-shard top-k + " \
                       "device merge" % (N, D, args.expansion, world, NQ, K)
        else:
            metric_name = "QPS at recall@10=0.95, %d x %d-d float L2 sharded over %d GPUs" % (N * world, D, world)
            workload = "C4 form: %d objects per GPU shard, %d shards, %d queries/step over all shards, k=%d, " \
                       "one packed RCCL all-gather of per-shard top-k + device merge" % (N, world, NQ, K)
        line = {
            "metric": metric_name,
            "value": qps,
            "unit": "queries/s",
            "n_gpus": n_ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if not qgm else "u4-adc/u8-lut/f32-rerank",
            "data": "synthetic (splitmix64 U[0,1), seed 0x4E4754)",
            "config": {"workload": workload,
                       "recall_at_10": rec, "epsilon": chosen,
                       "edge_size": ("all" if args.edge_size == 0 else
                                     "%d (sc.edgeSize %d; the prf's EdgeSizeForSearch %d)" % (
                                         es_resolved, args.edge_size, es_prop)),
                       "graph": graph,
                       "seeds": ("getSeedsFromTree (DVP tree leaf, seed size %d)" % args.seed_size
                                 if args.seeds == "tree" else "getRandomSeeds (%d)" % args.seed_size),
                       "sweep_kernel_ms_cap": SWEEP_KERNEL_MS_CAP,
                       "distance_computations_per_query": float(c[:, 0].mean()),
                       "expansions_per_query": float(c[:, 2].mean()),
                       "visited_set": ("hbm-epochs, every evaluated id (accepted-only and the LDS filter are "
                                       "off for rows over 1 KiB)" if dp * 4 > 1024 and args.visited in (-1, -2) else
                                       {-2: "hbm-epochs+lds-filter, accepted ids only",
                                        -1: "hbm-epochs+lds-filter"}.get(args.visited, "lds-hash")),
                       "parallelism": ("shards x%d" % world) if shard else ("replicas x%d" % world),
                       "distance_filter": ("1-byte filter copy (lower bound rejects neighbours outside the "
                                           "exploration radius; exact f32 rows for the rest)" if filtered else "none"),
                       "streams": ns_timed},
            "roofline": {"bound": "unmeasured", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic, "kernel": kname,
                         "kernel_ms": kernel_ms, "algorithmic_bytes_per_launch": alg_bytes,
                         "bytes_definition": ("the filtered kernel's own bytes: 1-byte filter rows of every distinct "
                                              "neighbour + f32 rows of the survivors (DESIGN.md 4)" if filtered
                                              else "SURVEY.md 8(d) B(q)"),
                         # SURVEY.md 8(d)'s literal B(q) = U*Dp*4 + E*4 + Dp*4 + k*8: the reference
                         # algorithm's bytes.  Over the kernel time it is an EFFECTIVE rate, which the
                         # filter lets exceed the HBM peak (the kernel never reads most of those rows)
                         "literal_bytes_per_launch": literal,
                         "effective_gbs_literal": literal / (kernel_ms * 1e-3) / 1e9,
                         "effective_frac_literal": literal / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                         "infinity_cache_resident_share": ic_share(split, alg_bytes),
                         # the bytes from tables larger than the 256 MiB Infinity Cache (f32 rows,
                         # adjacency, quantized-graph records, visited epochs, queries, results): what
                         # has to come from HBM itself, over the same kernel time
                         "hbm_side_bytes_per_launch": alg_bytes * (1.0 - ic_share(split, alg_bytes)),
                         "hbm_side_gbs": alg_bytes * (1.0 - ic_share(split, alg_bytes)) / (kernel_ms * 1e-3) / 1e9,
                         "hbm_side_frac": (alg_bytes * (1.0 - ic_share(split, alg_bytes)) / (kernel_ms * 1e-3) / 1e9
                                           / PEAK_HBM_GBS),
                         # the bytes from the Infinity-Cache-resident table against the measured
                         # random-row gather rate of such a table
                         "ic_side_gbs": alg_bytes * ic_share(split, alg_bytes) / (kernel_ms * 1e-3) / 1e9,
                         "ic_side_frac": (alg_bytes * ic_share(split, alg_bytes) / (kernel_ms * 1e-3) / 1e9
                                          / IC_GATHER_GBS),
                         "ic_side_frac_per_step": (alg_bytes * ic_share(split, alg_bytes) / (elapsed / args.steps)
                                                   / 1e9 / IC_GATHER_GBS),
                         "ic_gather_peak_gbs": IC_GATHER_GBS,
                         # the same bytes over the whole step with launches overlapping on the streams
                         # (a single launch's last round of queries leaves the GPU part-empty)
                         "achieved_per_step": alg_bytes / (elapsed / args.steps) / 1e9,
                         "frac_per_step": alg_bytes / (elapsed / args.steps) / 1e9 / PEAK_HBM_GBS,
                         "bytes_split": split,
                         # the probe-and-resume schedule: one search = a probe dispatch (every query
                         # paused after `budget` expansions) + a resume dispatch, longest predicted first;
                         # kernel_ms spans both (ngt_amd_api.cpp run_search)
                         "search_dispatches": 2 if budget else 1,
                         "schedule_budget": budget},
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "sweep": sweep,
        }
        if stream_ms:
            line["config"]["stream_ab_ms_per_step"] = stream_ms
        if scan is not None:
            line["exact_scan"] = scan
        if build_s is not None:
            line["config"]["graph_build_s"] = build_s
        if anng_check is not None:
            line["config"]["construction_check"] = anng_check
        if ref_check is not None:
            line["config"]["reference_search_check"] = ref_check
        if latency is not None:
            line["single_query_latency"] = latency
        if capi is not None:
            line["capi"] = capi
        cn = tentry.get("counters_per_launch")
        if cn:
            # PMC evidence for what bounds the kernel (profiles/traffic.json):
            # share of wave-cycles issuing VALU, actual HBM bytes / algorithmic
            line["roofline"]["counters"] = {
                "source": tentry.get("source", ""), "SQ_INSTS_VALU": cn["SQ_INSTS_VALU"],
                "valu_wave_cycle_frac": cn["SQ_ACTIVE_INST_VALU"] / cn["SQ_WAVE_CYCLES"],
                "traffic_over_algorithmic": traffic / alg_bytes}
            if "TCC_HIT_sum" in cn:
                line["roofline"]["counters"].update({
                    "l2_hit_rate": tentry.get("l2_hit_rate"),
                    "dram_destined_read_frac": tentry.get("dram_destined_read_frac"),
                    "note": "FETCH_SIZE and TCC_EA0_RDREQ_DRAM count the L2's memory-side reads, Infinity-Cache "
                            "hits included; no TCC counter on gfx950 separates them"})
            if "SQ_WAIT_ANY" in cn:
                # the wave-cycle partition (MI355X_MICROARCH.md rocprofv3 PMC slots):
                # parked on s_waitcnt/barrier, issue-stalled, issuing
                w = cn["SQ_WAVE_CYCLES"]
                line["roofline"]["counters"].update({
                    "wait_any_frac": cn["SQ_WAIT_ANY"] / w, "wait_inst_any_frac": cn["SQ_WAIT_INST_ANY"] / w,
                    "active_inst_any_frac": cn["SQ_ACTIVE_INST_ANY"] / w,
                    "SQ_INSTS_LDS": cn.get("SQ_INSTS_LDS"),
                    "trace_avg_kernel_ms": tentry.get("trace_avg_kernel_ms")})
                # what bounds the kernel, from the wave-cycle partition
                si = tentry.get("simd_issue")
                if si:
                    # the SIMDs' issue in measured (GRBM) cycles, scripts/pmc_clk.sh
                    line["roofline"]["counters"]["simd_issue"] = si
                ta = tentry.get("texture_address")
                if ta:
                    # the texture address units' busy share over the same clock (PMC_TAG=ta pass)
                    line["roofline"]["counters"]["texture_address"] = ta
                line["roofline"]["bound"] = bound_from_counters(cn, ic_share(split, alg_bytes), si)
                line["roofline"]["bound_note"] = (
                    "from the SQ counters and the byte split: 'issue' when the SIMDs issue in >= 0.7 of their "
                    "GRBM-measured cycles (counters.simd_issue), 'latency' when >= 0.5 of the wave-cycles are "
                    "parked on s_waitcnt (dependent gathers), 'valu' when VALU issues on >= 0.5, "
                    "'infinity-cache' when most algorithmic bytes come from a table the 256 MiB Infinity Cache "
                    "holds, else 'hbm'; achieved/frac are against the 8 TB/s HBM figure, hbm_side_frac counts "
                    "only the bytes from tables beyond the Infinity Cache, ic_side_frac the IC-resident bytes "
                    "against the measured 8.6 TB/s Infinity-Cache gather rate")
        if qgm:
            line["config"]["result_expansion"] = args.expansion
            if expansion_sweep is not None:
                line["config"]["result_expansion_sweep"] = expansion_sweep
            line["config"]["qg_layout"] = (
                {"packed_record_bytes": qg_record_bytes, "bytes_per_node": qg_record_bytes / N,
                 "what": "per node ceil(deg/16) code blocks of 8*Me bytes + 16 {id, key word} entries per block "
                         "(QuantizedGraph.h:74-113's per-node blocks); a popped key names its record and length"}
                if qg_record_bytes else {"fixed_stride_code_bytes_per_node": int(ix.L.ngt_amd_qg_code_stride(ix.h))})
            line["config"]["adc_distances_per_query"] = float(c[:, 0].mean())
            line["config"]["accepted_per_query"] = float(c[:, 1].mean())
            line["config"]["exact_distances_per_query"] = float(c[:, 3].mean())
        else:
            line["config"]["edges_read_per_query"] = float(c[:, 4].mean())
            if filtered:
                line["config"]["exact_neighbour_distances_per_query"] = float(c[:, 6].mean())
            if evals_per_query is not None:
                line["config"]["evaluations_per_query"] = evals_per_query
        headline_run = args.mode == "exact" and not c3 and args.graph == "knn" and world == 1
        want_anng = args.anng_line == "on" or (args.anng_line == "auto" and headline_run)
        want_qg = args.qg_line == "on" or (args.qg_line == "auto" and headline_run and N == 1_000_000
                                           and not args.pmc_launches)
        if want_anng or want_qg:
            # the ANNG line builds and saves the 1M ANNG here; the QG line
            # quantizes that same index
            import shutil
            import tempfile
            index_dir = tempfile.mkdtemp(prefix="ngt_anng_")
            try:
                if want_anng:
                    line["anng"] = anng_child_line(args, index_dir)
                if want_qg:
                    line["qg"] = qg_child_line(args, index_dir)
            finally:
                shutil.rmtree(index_dir, ignore_errors=True)
        want_c3 = args.c3_line == "on" or (args.c3_line == "auto" and headline_run and N == 1_000_000
                                           and not args.pmc_launches)
        if want_c3:
            line["c3"] = c3_child_line(args)
    want_shard = args.shard_line == "on" or (args.shard_line == "auto" and args.mode == "exact" and not c3
                                             and args.graph == "knn" and world > 1 and not args.pmc_launches)
    if want_shard:
        # C4: the same 10M index at every N -- 8 shards of
        # 1.25M objects, 8/N of them on each rank, one RCCL all-gather per
        # step, merged recall and an oracle parity sample (strong scaling:
        # the index and the batch are fixed, the ranks share them)
        ix.close()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        if dist is None:  # --shard-line on with one rank: a one-rank RCCL group
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        sargs = argparse.Namespace(**vars(args))
        sargs.mode, sargs.qg, sargs.eps, sargs.n = "shard", False, "", args.shard_n
        sargs.shards_per_gpu = max(1, args.shard_count // world)
        sargs.steps = max(3, min(args.steps, 10))
        sargs.warmup = 1
        log("shard line: C4 as %d x %d shards of %d objects%s" % (
            world, sargs.shards_per_gpu, sargs.n, ", then C5's NGTQG form over the same shards"
            if args.shard_qg_line == "on" else ""))
        t0 = time.time()
        sl = shard_bench(sargs, torch, dist, dev, rank, world, local, None, False, emit=False,
                         also_qg=args.shard_qg_line == "on")
        if rank == 0:
            sl.pop("sweep", None)
            sl["scaling"] = "strong"
            if "qg_form" in sl:
                sl["qg_form"]["scaling"] = "strong"  # the same fixed index, the ranks share it
            sl["wall_s"] = time.time() - t0
            line["shard"] = sl
    if rank == 0:
        print(json.dumps(line), file=result_out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


def pick_expansion(sweep, target, tie=1.03, default=3.0):
    """The result_expansion whose tuned whole-batch launch is fastest among
    those reaching the target recall (all of them if none does); launches
    within `tie` of the fastest are run-to-run noise, and among those the one
    nearest the C API's default (NGTQ/Capi.cpp:44) is taken, so the pick
    repeats from run to run."""
    ok = [e for e in sweep if e["recall_at_10"] >= target] or sweep
    fastest = min(e["kernel_ms"] for e in ok)
    return min([e for e in ok if e["kernel_ms"] <= fastest * tie],
               key=lambda e: (abs(e["result_expansion"] - default), e["result_expansion"]))


def literal_bytes(c, dp, nq, k, qgm, dim):
    """SURVEY.md 8(d)'s algorithmic bytes of the reference algorithm from the
    counters of a full-visited-set run: exact B(q) = U*Dp*4 + E*4 + Dp*4 + k*8;
    NGTQG B(q) = sum ceil(deg/16)*16*(M/2) + deg*4 + (seeds + k*expansion)*Dp*4."""
    if qgm:
        me = (dim + 1) // 2 * 2
        return float(c[:, 4].sum() * 8 * me + c[:, 0].sum() * 4 + c[:, 3].sum() * dp * 4 + nq * (dp * 4 + k * 8))
    return float(c[:, 0].sum() * dp * 4 + c[:, 4].sum() * 4 + nq * (dp * 4 + k * 8))


def ic_share(split, alg_bytes):
    """Share of the algorithmic bytes that come from tables the 256 MiB
    Infinity Cache can hold (the 1-byte filter copy at C2: 128 MB)."""
    if not split or not split.get("filter_copy_fits_infinity_cache"):
        return 0.0
    return float(split["filter_copy_bytes"] / alg_bytes)


def bound_from_counters(cn, ic_resident_share=0.0, simd_issue=None):
    """What bounds the kernel, from the SQ counters (MI355X_MICROARCH.md
    rocprofv3 PMC): the SIMDs issuing in at least 0.7 of their cycles (the
    GRBM-clocked pass, scripts/pmc_clk.sh) = instruction issue, however long
    each wave waits -- the other waves of its SIMD fill the gaps; else more
    than half the wave-cycles parked on s_waitcnt = dependent-gather latency;
    else VALU-issue bound if VALU issues on more than half; else the memory
    system -- the Infinity Cache when most of the algorithmic bytes come from
    a table it holds (the C2 filter copy), HBM otherwise."""
    w = cn["SQ_WAVE_CYCLES"]
    if simd_issue and simd_issue.get("simd_issue_util", 0.0) >= 0.7:
        return "issue"
    if cn.get("SQ_WAIT_ANY", 0) / w >= 0.5:
        return "latency"
    if cn.get("SQ_ACTIVE_INST_VALU", 0) / w >= 0.5:
        return "valu"
    if ic_resident_share >= 0.5:
        return "infinity-cache"
    return "hbm"


def group_members(pgid):
    """Pids of live processes in process group pgid (from /proc)."""
    pids = []
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open("/proc/%s/stat" % d) as f:
                st = f.read()
        except OSError:
            continue
        fields = st[st.rfind(")") + 2:].split()
        if len(fields) > 2 and fields[0] != "Z" and int(fields[2]) == pgid:
            pids.append(int(d))
    return pids


def run_reaped(argv, timeout, env=None, capture_stderr=False, what="child"):
    """Run a child command in its own session (process group) and wait for it;
    afterwards anything it left behind in that group is terminated, so no
    process of this bench outlives it.  Returns (returncode, stdout, stderr)."""
    import signal
    import subprocess
    import threading
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE if capture_stderr else None, env=env,
                         start_new_session=True)
    # the pipes are drained by threads and the wait is for the child itself:
    # a leftover holding the pipes open must not keep this call waiting
    got = {}
    readers = [threading.Thread(target=lambda n, f: got.__setitem__(n, f.read()), args=(n, f), daemon=True)
               for n, f in (("out", p.stdout), ("err", p.stderr)) if f is not None]
    for t in readers:
        t.start()
    try:
        p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        log("%s: no exit after %d s; stopping its process group" % (what, timeout))
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
    left = group_members(p.pid)
    if left:
        log("%s left %d process(es) behind (%s); terminating them" % (what, len(left), left))
        try:
            os.killpg(p.pid, signal.SIGTERM)
            for _ in range(50):
                if not group_members(p.pid):
                    break
                time.sleep(0.1)
            if group_members(p.pid):
                os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
    for t in readers:
        t.join(10)
    return (p.returncode, (got.get("out") or b"").decode(errors="replace"),
            (got.get("err") or b"").decode(errors="replace"))


def child_line(args, name, extra, cpu_seconds, latency_queries):
    """One of the lines measured beside the headline: a child process of this
    bench with its own roofline, cpu_baseline and parity sample (its JSON line
    without the sweep), or {"error": ...} if it fails."""
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + extra + [
        "--anng-line", "off", "--c3-line", "off", "--qg-line", "off",
        "--steps", str(max(3, min(args.steps, 5))), "--warmup", "1",
        "--cpu-seconds", str(min(args.cpu_seconds, cpu_seconds)), "--latency-queries", str(latency_queries)]
    if args.no_cpu:
        cmd.append("--no-cpu")
    t0 = time.time()
    log("%s line: %s" % (name, " ".join(cmd[2:])))
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    rc, stdout, _ = run_reaped(cmd, 900, env=env, what="%s line" % name)
    out = [l for l in stdout.splitlines() if l.startswith("{")]
    if rc != 0 or not out:
        log("%s line failed (rc %d)" % (name, rc))
        return {"error": "child run failed", "rc": rc}
    d = json.loads(out[-1])
    d.pop("sweep", None)
    d["child_wall_s"] = time.time() - t0
    log("%s line: %.0f QPS at recall %.4f, frac %.3f (%.0f s)" % (
        name, d["value"], d["config"]["recall_at_10"], d["roofline"]["frac"], d["child_wall_s"]))
    return d


def anng_child_line(args, index_dir):
    """The index a `ngt create` user has, measured beside the headline: the
    1M ANNG (E 10) built on the device through the C API (files identical to
    the reference's build, saved to index_dir), searched at the prf's
    EdgeSizeForSearch 40 (Command.cpp:39, Graph.h:675-692) from DVP-tree
    seeds; with its `capi` sub-key (the drop-in C API on the saved index)."""
    return child_line(args, "ANNG", ["--graph", "anng", "--anng-dir", index_dir], 8.0, 20)


def qg_child_line(args, index_dir):
    """BASELINE config 5's path on one GPU: `ngtqg quantize` on the device
    (kmeansWithNGT codebooks, encoder, quantized graph of <= 128 edges;
    QuantizedGraph.h:456-475) over the 1M ANNG the ANNG line saved (opened
    with ngt_open_index; rebuilt if that line failed), searched with
    NGTQG::Index::search from DVP-tree seeds (QuantizedGraph.h:354-372) at the
    result_expansion / epsilon pair that reaches recall@10 0.95 fastest."""
    return child_line(args, "QG", ["--mode", "qg", "--graph", "anng", "--anng-dir", index_dir,
                                   "--qg-expansions", "2,3,4,6"], 10.0, 0)


def c3_child_line(args):
    """C3 (BASELINE config 3: 1M x 960 float cosine, kNN graph, the cosine
    filter) measured beside the headline."""
    return child_line(args, "C3", ["--config", "c3"], 10.0, 0)


def capi_anng_line(index_dir, Q, gt, D, K, eps, threads):
    """The drop-in C API on the 1M ANNG this run built and saved: a pthreads
    C client (tests/cxx/capi_threads.c) opens the directory with
    ngt_open_index and issues single-query ngt_search_index calls
    (Capi.cpp:377-406) -- 1 thread (latency), `threads` and 2x `threads`
    concurrent callers at the bench's epsilon -- and, for parity, the
    reference fixture's 200 queries at its epsilon on one thread: the ids
    must equal `ngt search`'s own output on the reference's build of the same
    data (tests/golden/c2_anng_ref.npz)."""
    t0 = time.time()
    runs = capi_c_client(index_dir, Q, gt, D, K, eps, threads)
    z = np.load(os.path.join(ROOT, "tests", "golden", "c2_anng_ref.npz"))
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "c2_anng_ref.json")))
    n = z["ids"].shape[0]
    eps_ref = float(meta["sweep"]["epsilon"])
    ref_runs = capi_c_client(index_dir, Q[:n], gt[:n], D, K, eps_ref, 1, plan=[(1, n)], keep_ids=True)
    got = ref_runs[0].pop("ids")
    same = all(np.array_equal(got[q, :int(z["n"][q])], z["ids"][q, :int(z["n"][q])].astype(got.dtype))
               and not got[q, int(z["n"][q]):].any() for q in range(n))
    best = max(runs, key=lambda r: r["qps"])
    one = [r for r in runs if r["threads"] == 1][0]
    out = {"what": "ngt_open_index + single-query ngt_search_index calls from a pthreads C client "
                   "(tests/cxx/capi_threads.c) on the saved 1M ANNG (tree seeds, the prf's edge size 40)",
           "epsilon": eps, "single_thread_latency_ms": one["latency_ms"], "qps_best": best["qps"],
           "threads_best": best["threads"], "runs": runs,
           "reference_parity": {"queries": n, "epsilon": eps_ref, "ids_identical_to_ngt_search": bool(same),
                                "recall_at_10_vs_truth": ref_runs[0]["recall_at_10"]},
           "wall_s": time.time() - t0}
    log("C API on the ANNG: 1 thread %.2f ms/query, best %.0f QPS at %d threads; reference ids identical: %s" % (
        one["latency_ms"]["mean"], best["qps"], best["threads"], same))
    return out


def measured_traffic(mode, config, graph, eps, visited, filtered=False):
    """HBM bytes per launch of the search kernel from the committed PMC passes
    (profiles/traffic.json, written from rocprofv3 FETCH_SIZE/WRITE_SIZE) for this
    exact workload and epsilon; NGT_BENCH_TRAFFIC_BYTES overrides; else None."""
    tf = os.environ.get("NGT_BENCH_TRAFFIC_BYTES")
    if tf:
        return float(tf), {}
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            entries = json.load(f)["entries"]
    except (OSError, ValueError, KeyError):
        return None, {}
    for e in reversed(entries):  # the newest entry for the workload
        if (e.get("mode", "exact") == mode and e.get("config", "c2") == config and e["graph"] == graph
                and e.get("visited", -1) == visited and abs(e["epsilon"] - eps) < 1e-7
                and bool(e.get("filtered", False)) == bool(filtered)):
            return float(e["traffic_bytes"]), e
    return None, {}


def calibration():
    """The oracle port against the reference itself, measured in the build
    container on the same 1M ANNG, queries and epsilon
    (tests/golden/make_c2_anng_fixture.py -> c2_anng_ref.json): the port's
    single-thread QPS over the reference's.  On the GPU box only the port can
    run; value / ratio is its reference-equivalent rate."""
    path = os.path.join(ROOT, "tests", "golden", "c2_anng_ref.json")
    if not os.path.exists(path):
        return None
    t = json.load(open(path))["timing"]
    return {"where": "build container (%d CPUs), 1M x 128 ANNG built by the reference, %d queries, eps %g" % (
                t["container_cores"], t["queries"], t["epsilon"]),
            "reference_qps_1thread": t["reference_qps_1thread"], "port_qps_1thread": t["port_qps_1thread"],
            "ratio_port_over_reference_1thread": t["ratio_port_over_reference_1thread"],
            "port_identical_to_reference": t["port_identical_to_reference"]}


def sha256_file(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def build_anng_device(args, torch, dev, rows, N, D, es_prop, local):
    """GraphAndTreeIndex::createIndex (Index.cpp:1158-1257) of N HBM-resident
    rows with this library's device construction (ngt_amd_build_begin /
    _insert over id ranges, the path ngt_create_index takes), then the graph
    and DVP tree installed for search on the same index."""
    from ngt_amd.device import DeviceIndex
    ix = DeviceIndex("l2", "float", D, device=local)
    ix.set_objects_device(rows.data_ptr(), N + 1)
    t0 = time.time()
    step = 250_000
    for first in range(1, N + 1, step):
        if first == 1:
            import ctypes as _ct
            from ngt_amd._sigs import BuildParams
            prm = BuildParams(args.anng_edges, es_prop, args.anng_batch, args.seed_size, 0.1, 0)
            if ix.L.ngt_amd_build_begin(ix.h, _ct.byref(prm)) != 0:
                raise SystemExit("bench: ngt_amd_build_begin failed")
        if ix.L.ngt_amd_build_insert(ix.h, first, min(N + 1, first + step)) != 0:
            from ngt_amd import lib
            raise SystemExit("bench: device construction failed: " + lib().ngt_amd_last_error().decode())
        log("ANNG construction: %d of %d objects inserted (%.0f s)" % (min(N, first + step - 1), N, time.time() - t0))
    build_s = time.time() - t0
    offs, ids, _ = ix.build_graph()
    tree = ix.build_tree()
    ix.set_graph(offs, ids)
    ix.set_tree(tree)
    ix.set_search_property(es_prop, 30, 20, args.seed_size, 0)
    log("ANNG (E=%d, batch %d) of %d objects built on the device in %.1f s; %d edges, mean degree %.1f" % (
        args.anng_edges, args.anng_batch, N, build_s, len(ids), len(ids) / N))
    offsets = torch.from_numpy(offs.astype(np.int64)).to(dev)
    edges = torch.from_numpy(ids.astype(np.int32)).to(dev)
    return ix, offsets, edges, tree, build_s, {"reference": None, "built": "device, ngt_amd_build_insert in id ranges"}, None


def build_anng_capi(args, torch, dev, data, N, D, es_prop):
    """ANNG + DVP tree through the C API, saved in the reference's format; the
    saved files' sha256 against the reference build of the same data."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import ngt_files as F
    from ngt_amd import base as capi
    keep = args.anng_dir
    if keep and os.path.exists(os.path.join(keep, "grp")):
        # a directory an earlier run of this bench built and saved: opened with
        # ngt_open_index (the construction check belongs to the run that built it)
        cx = capi.Index(keep)
        offs, ids, _ = F.read_grp(os.path.join(keep, "grp"))
        tree = F.read_tre(os.path.join(keep, "tre"), D, np.float32)
        log("ANNG opened from %s (built by an earlier run)" % keep)
        return (cx.device_index(), torch.from_numpy(offs.astype(np.int64)).to(dev),
                torch.from_numpy(ids.astype(np.int32)).to(dev), tree, None, {"reference": None, "reopened": keep}, cx)
    tmp = keep or tempfile.mkdtemp(prefix="ngt_anng_")
    if keep:
        os.makedirs(os.path.dirname(os.path.abspath(keep)), exist_ok=True)
    capi.Index.create(tmp, D, edge_size_for_creation=args.anng_edges, edge_size_for_search=es_prop)
    cx = capi.Index(tmp)
    t0 = time.time()
    cx.batch_append(data)
    cx.build_index()
    build_s = time.time() - t0
    cx.save()
    log("ANNG (E=%d) built through the C API in %.1f s (ngt_create_index on the device)" % (args.anng_edges, build_s))
    check = {"reference": None}
    ref_path = os.path.join(ROOT, "tests", "golden", "c2_anng_ref.json")
    if os.path.exists(ref_path) and N == 1_000_000 and D == 128 and args.anng_edges == 10 and es_prop == 40:
        ref = json.load(open(ref_path))
        got = {f: sha256_file(os.path.join(tmp, f)) for f in ("obj", "grp", "tre")}
        same = {f: got[f] == ref["build"]["sha256"][f] for f in got}
        check = {"reference": "ngt create -d 128 -o f -D 2 -E 10 on the same data (%.0f s on %d CPUs)" % (
                     ref["build"]["build_s"], ref["build"]["cpus"]),
                 "files_identical": same}
        log("construction vs the reference's files: %s" % same)
    offs, ids, _ = F.read_grp(os.path.join(tmp, "grp"))
    tree = F.read_tre(os.path.join(tmp, "tre"), D, np.float32)
    offsets = torch.from_numpy(offs.astype(np.int64)).to(dev)
    edges = torch.from_numpy(ids.astype(np.int32)).to(dev)
    log("ANNG: %d edges, mean degree %.1f" % (edges.numel(), edges.numel() / N))
    ix = cx.device_index()
    if not keep:
        shutil.rmtree(tmp, ignore_errors=True)
    return ix, offsets, edges, tree, build_s, check, cx


def reference_fixture_check(ix, qdev, dp, K, dev, torch):
    """The device search of the reference fixture's queries at its epsilon
    (tree seeds, the prf's edge size) against `ngt search`'s own output on its
    own build of the same data (tests/golden/c2_anng_ref.npz): identical ids,
    distances within the printed precision."""
    from ngt_amd.device import SEED_TREE
    path = os.path.join(ROOT, "tests", "golden", "c2_anng_ref.npz")
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "c2_anng_ref.json")))
    z = np.load(path)
    n = z["ids"].shape[0]
    eps = float(meta["sweep"]["epsilon"])
    oi = torch.zeros((n, K), dtype=torch.int32, device=dev)
    od = torch.zeros((n, K), dtype=torch.float32, device=dev)
    on = torch.zeros((n,), dtype=torch.int32, device=dev)
    ix.search_device(qdev.data_ptr(), dp * 4, n, oi.data_ptr(), od.data_ptr(), on.data_ptr(), None, k=K,
                     epsilon=eps, edge_size=-1, seed_mode=SEED_TREE, stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    gi, gd, gn = oi.cpu().numpy().view(np.uint32), od.cpu().numpy(), on.cpu().numpy()
    ids_same = bool(np.array_equal(gn, z["n"].astype(gn.dtype)))
    dist_ok = True
    for q in range(n if ids_same else 0):
        m = int(gn[q])
        ids_same = ids_same and np.array_equal(gi[q, :m], z["ids"][q, :m])
        dist_ok = dist_ok and np.allclose(gd[q, :m], z["dists"][q, :m], rtol=1e-5, atol=0)
    rec = recall_at(gi.astype(np.int64), z["truth"].astype(np.int64), K)
    t = meta["timing"]
    out = {"queries": n, "epsilon": eps, "ids_identical": ids_same, "distances_within_print_precision": dist_ok,
           "recall_at_10_vs_reference_truth": rec,
           "reference_qps_1thread_container": t["reference_qps_1thread"],
           "reference_ms_per_query_1thread_container": t["reference_ms_per_query_1thread"]}
    log("reference fixture (%d queries, eps %g): ids identical %s, distances %s" % (n, eps, ids_same, dist_ok))
    if not (ids_same and dist_ok):
        raise SystemExit("bench: the device search differs from the reference's own ngt search output")
    return out


def tree_seed_lists(ix, qdev, dp, nq, k, dev, torch):
    """Tree seeds of every query (getSeedsFromTree, Index.h:1524-1567) from
    the device: one k-result graph search with seed_mode TREE would also
    produce them, but the lists themselves are what the oracle leg needs, so
    they come from ngt_amd_tree_seeds_device as [nq][<=seed stride] + counts."""
    L = ix.L
    stride = 128
    d_s = torch.zeros((nq, stride), dtype=torch.int32, device=dev)
    d_c = torch.zeros((nq,), dtype=torch.int32, device=dev)
    rc = L.ngt_amd_tree_seeds_device(ix.h, qdev.data_ptr(), dp * 4, nq, k, d_s.data_ptr(), stride,
                                     d_c.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    if rc != 0:
        raise SystemExit("bench: tree seeds failed: %s" % L.ngt_amd_last_error().decode())
    torch.cuda.synchronize()
    cnt = d_c.cpu().numpy().astype(np.int64)
    s = d_s.cpu().numpy().view(np.uint32)
    seeds = [s[i, :cnt[i]].copy() for i in range(nq)]
    off = np.zeros(nq + 1, np.int64)
    off[1:] = np.cumsum(cnt)
    flat = np.concatenate(seeds).astype(np.uint32)
    return seeds, torch.from_numpy(flat.view(np.int32)).to(dev), torch.from_numpy(off).to(dev)


def write_ngt_index(path, rows, offsets, edges, dim):
    """The C2 index in the reference's on-disk format (graph-only index, so
    searches take getRandomSeeds): prf (PropertySet, Common.h:573-666), obj
    (Repository<Object>: n, then '+' and dim floats per slot, Common.h:1776-1837,
    ObjectSpace.h:297-312), grp (n, then '+', uint32 count and {uint32 id, float
    distance} per edge, then the prevsize vector, Graph.h:151-158).  Edge
    distances are written as 0 (the search never reads them)."""
    os.makedirs(path, exist_ok=True)
    n = rows.shape[0]
    with open(os.path.join(path, "prf"), "w") as f:
        for k, v in [("Dimension", dim), ("DistanceType", "L2"), ("EdgeSizeForCreation", 10),
                     ("EdgeSizeForSearch", 0), ("GraphType", "ANNG"), ("IndexType", "Graph"),
                     ("ObjectType", "Float-4"), ("SeedSize", 10), ("SeedType", "None")]:
            f.write("%s\t%s\n" % (k, v))
    rec = np.zeros((n, 1 + 4 * dim), np.uint8)
    rec[:, 0] = ord("+")
    rec[:, 1:] = np.ascontiguousarray(rows[:, :dim]).view(np.uint8).reshape(n, 4 * dim)
    rec[0, 0] = ord("-")
    with open(os.path.join(path, "obj"), "wb") as f:
        f.write(np.uint64(n).tobytes())
        f.write(rec[:1, :1].tobytes())
        f.write(rec[1:].tobytes())
    deg = np.diff(offsets.astype(np.int64))
    with open(os.path.join(path, "grp"), "wb") as f:
        f.write(np.uint64(n).tobytes())
        f.write(b"-")
        pair = np.zeros((len(edges), 2), np.uint32)
        pair[:, 0] = edges
        for v in range(1, n):
            a, b = int(offsets[v]), int(offsets[v + 1])
            f.write(b"+")
            f.write(np.uint32(b - a).tobytes())
            f.write(pair[a:b].tobytes())
        f.write(np.uint32(0).tobytes())
    return deg


def capi_bench(args, torch, dev, result_out):
    """Single-query latency and concurrent-caller throughput of the drop-in
    ngt_search_index (Capi.cpp:346-375) on the C2 data and graph."""
    import tempfile
    import threading
    from ngt_amd import base
    N, D, NQ, K = args.n, args.dim, args.nq, args.k
    t0 = time.time()
    X = splitmix_uniform(N, D, BASE_SEED)
    Q = splitmix_uniform(NQ, D, BASE_SEED + 1)
    rows = torch.zeros((N + 1, D), dtype=torch.float32, device=dev)
    rows[1:] = torch.from_numpy(X).to(dev)
    offsets, edges = build_graph(torch, rows[1:], args.knn, args.out_deg, args.in_deg, args.max_deg, dev)
    h_rows, h_off, h_edges = rows.cpu().numpy(), offsets.cpu().numpy(), edges.cpu().numpy().astype(np.uint32)
    del rows, offsets, edges
    torch.cuda.empty_cache()
    tmp = tempfile.mkdtemp(prefix="ngt_c2_")
    write_ngt_index(tmp, h_rows, h_off, h_edges, D)
    log("C2 index written in the reference format (%.1f s)" % (time.time() - t0))
    t0 = time.time()
    ix = base.Index(tmp)
    gi, _, _ = ix.batch_linear_search(Q, K)
    gt = gi.astype(np.int64)
    log("opened + ground truth (batched C API linear search) in %.1f s" % (time.time() - t0))

    def recall(eps, nq=2000):
        bi, bd, bn = ix.batch_search(Q[:nq], K, eps, -1.0, -1, graph_only=True)
        return recall_at(bi.astype(np.int64), gt[:nq], K)

    eps = tune_epsilon(recall, args.target, [float(x) for x in args.eps.split(",")] if args.eps else None)
    rec = recall(eps, NQ)
    log("epsilon %.4f recall@10 %.4f (batched C API, graph-only random seeds)" % (eps, rec))
    # batched C API
    t0 = time.perf_counter()
    ix.batch_search(Q, K, eps, -1.0, -1, graph_only=True)
    batched_qps = NQ / (time.perf_counter() - t0)
    # single-query latency: sequential ngt_search_index calls
    lat = []
    for i in range(min(200, NQ)):
        t1 = time.perf_counter()
        ix.search(Q[i].astype(np.float64), K, eps)
        lat.append(time.perf_counter() - t1)
    lat = np.array(lat) * 1e3
    # concurrent single-query callers
    L = ix._L
    b0, s0 = ctypes.c_uint64(), ctypes.c_uint64()
    L.ngt_get_coalesce_stats(ix.index, ctypes.byref(b0), ctypes.byref(s0), ix.err)
    per = max(1, min(NQ // args.threads, 200))
    barrier = threading.Barrier(args.threads + 1)
    hits = [0] * args.threads

    def worker(t):
        barrier.wait()
        h = 0
        for j in range(per):
            i = t * per + j
            r = ix.search(Q[i].astype(np.float64), K, eps)
            h += len(set(x.id for x in r) & set(gt[i].tolist()))
        hits[t] = h
        barrier.wait()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(args.threads)]
    for t in th:
        t.start()
    barrier.wait()
    t1 = time.perf_counter()
    barrier.wait()
    el = time.perf_counter() - t1
    for t in th:
        t.join()
    b1, s1 = ctypes.c_uint64(), ctypes.c_uint64()
    L.ngt_get_coalesce_stats(ix.index, ctypes.byref(b1), ctypes.byref(s1), ix.err)
    nconc = args.threads * per
    py_threads = {"qps": nconc / el, "recall_at_10": sum(hits) / float(nconc * K), "threads": args.threads,
                  "coalesced_launches": int(b1.value - b0.value),
                  "mean_coalesced_batch": (s1.value - s0.value) / max(1, b1.value - b0.value),
                  "what": "Python threads through ctypes (GIL-bound client)"}
    # the same calls from a C client (tests/cxx/capi_threads.c, pthreads): the
    # reference's own call pattern with nothing between callers and library
    cres = capi_c_client(tmp, Q, gt, D, K, eps, args.threads)
    best = max(cres, key=lambda r: r["qps"] if r["threads"] == args.threads else -1)
    line = {"metric": "C-API ngt_search_index on C2 (1M x 128 L2): single-query latency and %d-thread throughput"
                      % args.threads,
            "value": best["qps"], "unit": "queries/s", "n_gpus": 1, "higher_is_better": True,
            "dtype": "f32", "data": "synthetic (splitmix64 U[0,1), seed 0x4E4754)",
            "config": {"workload": "C2 graph written as an NGT index directory, opened with ngt_open_index",
                       "epsilon": eps, "recall_at_10_batched": rec,
                       "recall_at_10_concurrent": sum(hits) / float(nconc * K),
                       "seeds": "getRandomSeeds (graph-only index)", "threads": args.threads,
                       "queries_per_thread": per,
                       "coalesced_launches": int(b1.value - b0.value),
                       "mean_coalesced_batch": (s1.value - s0.value) / max(1, b1.value - b0.value)},
            "single_query_latency_ms": {"mean": float(lat.mean()), "p50": float(np.percentile(lat, 50)),
                                        "p99": float(np.percentile(lat, 99)), "calls": len(lat),
                                        "client": "Python ctypes, sequential"},
            "c_client_runs": cres, "value_from": best,
            "python_threads": py_threads,
            "batched_capi_qps": batched_qps}
    print(json.dumps(line), file=result_out, flush=True)
    ix.close()


def shard_bench(args, torch, dist, dev, rank, world, local, result_out, qgm, emit=True, also_qg=False):
    """C4's and C5's form: the object repository as
    world x S shards of --n objects, rank r holding shards r*S .. r*S+S-1
    (global ids offset by shard * n), every shard an independent index with
    its own graph (and, with --qg, its own NGTQG quantizer, encoder and
    quantized graph).  A step searches the whole batch on every shard -- the
    S local shards concurrently on S streams -- packs the S top-k lists into
    the rank's one RCCL all-gather message and merges world * S lists on the
    device (ngt_amd/shard.py).  S > 1 serves an index larger than one graph a
    run can build on one GPU (C4's 10M on one GPU: S = 8 shards of 1.25M)."""
    from ngt_amd.device import COUNTERS, SEED_GIVEN, DeviceIndex
    from ngt_amd.shard import ShardedIndex
    N, D, NQ, K = args.n, args.dim, args.nq, args.k
    S = max(1, args.shards_per_gpu)
    dp = ((D - 1) // 16 + 1) * 16
    t0 = time.time()
    qry = splitmix_uniform(NQ, D, BASE_SEED + 1)
    shards = []
    for s in range(S):
        off = (rank * S + s) * N
        base = splitmix_uniform(N, D, BASE_SEED, row0=off)
        rows = torch.zeros((N + 1, dp), dtype=torch.float32, device=dev)
        rows[1:, :D] = torch.from_numpy(base).to(dev)
        ix = DeviceIndex("l2", "float", D, device=local)
        ix.set_objects_device(rows.data_ptr(), N + 1)
        offsets, edges = build_graph(torch, rows[1:, :D], args.knn, args.out_deg, args.in_deg, args.max_deg, dev)
        ix.set_search_property(0, 30, 20, args.seed_size, 0)
        ix.set_graph_device(offsets.data_ptr(), edges.data_ptr(), edges.numel())
        sh = {"ix": ix, "rows": rows, "offsets": offsets, "edges": edges, "off": off, "qg_local": None}
        if qgm:
            # ngtqg quantize of this shard: kmeansWithNGT codebooks from its
            # first 1,600 objects, encoder, quantized graph (QuantizedGraph.h:456-475)
            h_base = np.zeros((min(N, 1600) + 1, D), np.float32)
            h_base[1:] = base[:min(N, 1600)]
            sh["qg_local"] = ix.qg_train_ngt(h_base, dsub=1)
            ix.qg_encode(return_codes=False)
            ix.qg_build_graph(None, args.qg_edges)
        del base
        shards.append(sh)
        torch.cuda.synchronize()
        log("shard %d/%d (offset %d) ready at %.1f s" % (s + 1, S, off, time.time() - t0))
    setup_s = time.time() - t0
    ix0 = shards[0]["ix"]
    main = torch.cuda.current_stream(dev)
    qraw = torch.from_numpy(qry).to(dev)
    qdev = torch.zeros((NQ, dp), dtype=torch.float32, device=dev)
    ix0.prepare_queries_device(qraw.data_ptr(), NQ, qdev.data_ptr(), stream=main.cuda_stream)
    sx = ShardedIndex(torch, dist, [sh["ix"] for sh in shards], [sh["off"] for sh in shards], dev)

    def buffers():
        return (torch.zeros((S, NQ, K), dtype=torch.int32, device=dev),
                torch.zeros((S, NQ, K), dtype=torch.float32, device=dev),
                torch.zeros((S, NQ), dtype=torch.int32, device=dev))

    # exact ground truth of the whole index: every shard's linear search, merged
    t1 = time.time()
    gi, gd, gn = buffers()
    for s, sh in enumerate(shards):
        sh["ix"].linear_search_device(qdev.data_ptr(), dp * 4, NQ, K, gi[s].data_ptr(), gd[s].data_ptr(),
                                      gn[s].data_ptr(), stream=main.cuda_stream)
    gt = sx.merge_local(gi, gd, gn, K, main.cuda_stream)[0].cpu().numpy()
    del gi, gd, gn
    log("ground truth (%d shard scans + merge) in %.1f s" % (S * world, time.time() - t1))

    seeds = random_seeds(N + 1, NQ, args.seed_size)
    d_seeds = torch.from_numpy(seeds.reshape(-1).astype(np.int32)).to(dev)
    d_soff = torch.arange(0, NQ + 1, dtype=torch.int64, device=dev) * args.seed_size
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    def measure_form(qgm):
        """Tune, time and check one form of the sharded index (exact graph
        search, or NGTQG over the same shards); rank 0 gets its line."""
        out_i, out_d, out_n = buffers()
        cnt = torch.zeros((S, NQ, COUNTERS), dtype=torch.int64, device=dev)
        merged = {}

        def search_shard(s, eps, st, visited):
            ix = shards[s]["ix"]
            if qgm:
                ix.qg_search_device(qdev.data_ptr(), dp * 4, NQ, out_i[s].data_ptr(), out_d[s].data_ptr(),
                                    out_n[s].data_ptr(), cnt[s].data_ptr(), k=K, epsilon=eps,
                                    result_expansion=args.expansion, seed_mode=SEED_GIVEN, d_seeds=d_seeds.data_ptr(),
                                    d_seed_off=d_soff.data_ptr(), stream=st, visited_hash_log2=visited)
            else:
                ix.search_device(qdev.data_ptr(), dp * 4, NQ, out_i[s].data_ptr(), out_d[s].data_ptr(),
                                 out_n[s].data_ptr(), cnt[s].data_ptr(), k=K, epsilon=eps, edge_size=0,
                                 seed_mode=SEED_GIVEN, d_seeds=d_seeds.data_ptr(), d_seed_off=d_soff.data_ptr(),
                                 stream=st, visited_hash_log2=visited)

        # the NGTQG search marks accepted ids by definition (QuantizedGraph.h:241-266)
        vis_default = -1 if qgm and args.visited == -2 else args.visited

        def run(eps, visited=None):
            visited = vis_default if visited is None else visited
            # the shard streams wait for the previous step's pack (it reads out_*)
            for st in streams:
                st.wait_stream(main)
            for s in range(S):
                search_shard(s, eps, streams[s].cuda_stream, visited)
            for st in streams:
                main.wait_stream(st)
            merged["r"] = sx.merge_local(out_i, out_d, out_n, K, main.cuda_stream)

        sweep = []

        def measure(eps):
            run(eps)
            torch.cuda.synchronize()
            r = recall_at(merged["r"][0].cpu().numpy(), gt, K)
            sweep.append((round(eps, 5), r, None, NQ))
            log("eps %.4f merged recall@%d %.4f" % (eps, K, r))
            return r

        chosen = tune_epsilon(measure, args.target, [float(x) for x in args.eps.split(",")] if args.eps else None)
        rec = measure(chosen)
        for _ in range(20):
            if rec >= args.target or args.eps:
                break
            chosen = round(chosen * 1.02 + 1e-4, 5)
            rec = measure(chosen)
        if args.pmc_launches:
            # counter passes: exactly this many more steps of the timed
            # configuration (S shard searches each), nothing else of the bench
            for _ in range(args.pmc_launches):
                run(chosen)
                torch.cuda.synchronize()
            if rank == 0:
                print(json.dumps({"pmc_launches": args.pmc_launches, "shards_per_gpu": S, "epsilon": chosen,
                                  "recall_at_10": rec}), file=result_out, flush=True)
            if dist is not None:
                dist.destroy_process_group()
            return
        for _ in range(max(1, args.warmup)):
            run(chosen)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            run(chosen)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t1
        if dist is not None:
            t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        qps = NQ * args.steps / elapsed
        res = [x.clone() for x in merged["r"]]
        # per-launch kernel time: each shard's search alone on the main stream
        kms = []
        for s in range(S):
            search_shard(s, chosen, main.cuda_stream, vis_default)
            torch.cuda.synchronize()
            kms.append(shards[s]["ix"].last_search_kernel_ms())
        filtered = (not qgm) and ix0.last_search_filtered()
        # the schedule budget of those launches (0: single dispatches)
        budget = 0 if qgm else shards[S - 1]["ix"].last_search_budget()
        split = None  # (the exact mode's filter-copy split is not kept per shard)
        if not qgm and args.visited == -2:
            # the reference's distinct distance counts (every evaluated id in the
            # visited set) for the algorithmic bytes; the results must not change
            run(chosen, visited=-1)
            torch.cuda.synchronize()
            same = all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(res, merged["r"]))
            if not same:
                raise SystemExit("bench: accepted-only visited set changed the merged results")
        c = cnt.cpu().numpy().astype(np.float64).reshape(S * NQ, COUNTERS)
        if qgm:
            me = (D + 1) // 2 * 2
            alg_bytes = (c[:, 4].sum() * 8 * me + c[:, 0].sum() * 4 + c[:, 3].sum() * dp * 4
                         + S * NQ * (dp * 4 + K * 8))
            kname = "ngt_qg_search_kernel"
        elif filtered:
            alg_bytes = ((c[:, 0] - c[:, 7]).sum() * dp + (c[:, 7] + c[:, 6]).sum() * dp * 4 + c[:, 4].sum() * 4
                         + S * NQ * (dp * 4 + K * 8))
            kname = "ngt_graph_search_kernel"
        else:
            alg_bytes = c[:, 0].sum() * dp * 4 + c[:, 4].sum() * 4 + S * NQ * (dp * 4 + K * 8)
            kname = "ngt_graph_search_kernel"
        kernel_ms = float(np.mean(kms))
        per_launch = alg_bytes / S
        achieved = per_launch / (kernel_ms * 1e-3) / 1e9
        literal = literal_bytes(c, dp, S * NQ, K, qgm, D) / S

        cpu = parity = None
        if not args.no_cpu:
            # every rank checks its own shards against the oracle; with several
            # ranks the candidates are all-gathered and every rank checks the merge
            cpu, parity = shard_parity_sample(args, shards, qdev, seeds, chosen, res, qgm, dist=dist)

        if rank == 0:
            total = N * S * world
            if qgm:
                metric_name = "QPS at recall@10=0.95, %d x %d-d NGTQG sharded over %d GPUs" % (total, D, world)
                workload = ("C5 form: %d objects per GPU as %d NGTQG shards of %d (dsub=1, M=%d, result_expansion %g), "
                            "%d GPUs, %d queries/step over all shards, k=%d, one packed RCCL all-gather of per-shard "
                            "top-k + device merge" % (N * S, S, N, D, args.expansion, world, NQ, K))
            else:
                metric_name = "QPS at recall@10=0.95, %d x %d-d float L2 sharded over %d GPUs" % (total, D, world)
                workload = ("C4 form: %d objects per GPU as %d shards of %d, %d GPUs, %d queries/step over all shards, "
                            "k=%d, one packed RCCL all-gather of per-shard top-k + device merge" % (
                                N * S, S, N, world, NQ, K))
            line = {
                "metric": metric_name, "value": qps, "unit": "queries/s", "n_gpus": dist.get_world_size() if dist is not None else 1,
                "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None,
                "dtype": "f32" if not qgm else "u4-adc/u8-lut/f32-rerank",
                "data": "synthetic (splitmix64 U[0,1), seed 0x4E4754)",
                "config": {"workload": workload, "objects_total": total, "shards_per_gpu": S, "objects_per_shard": N,
                           "recall_at_10": rec, "epsilon": chosen,
                           "graph": "kNN%d out%d in%d max%d per shard" % (args.knn, args.out_deg, args.in_deg,
                                                                         args.max_deg),
                           "seeds": "getRandomSeeds (%d)" % args.seed_size, "setup_s": setup_s,
                           "distance_filter": "1-byte filter copy" if filtered else "none",
                           "parallelism": "shards x%d (%d per GPU, one stream each)" % (S * world, S),
                           "distance_computations_per_query_per_shard": float(c[:, 0].mean()),
                           "expansions_per_query_per_shard": float(c[:, 2].mean())},
                "roofline": {"bound": "unmeasured", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": achieved / PEAK_HBM_GBS, "traffic": None, "kernel": kname,
                             "kernel_ms": kernel_ms, "algorithmic_bytes_per_launch": per_launch,
                             "bytes_definition": ("the filtered kernel's own bytes (DESIGN.md 4)" if filtered
                                                  else "SURVEY.md 8(d) B(q)"),
                             "literal_bytes_per_launch": literal,
                             "effective_gbs_literal": literal / (kernel_ms * 1e-3) / 1e9,
                             "effective_frac_literal": literal / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                             "infinity_cache_resident_share": (
                                 (c[:, 0] - c[:, 7]).sum() * dp / S / per_launch
                                 if filtered and (N + 1) * dp <= 256 * 2 ** 20 else 0.0),
                             "what": "one shard's search launch alone (mean over the %d local shards)" % S,
                             "achieved_per_step": alg_bytes / (elapsed / args.steps) / 1e9,
                             "frac_per_step": alg_bytes / (elapsed / args.steps) / 1e9 / PEAK_HBM_GBS,
                             "bytes_split": split,
                             # the probe-and-resume schedule: one search = a probe dispatch (every query
                             # paused after `budget` expansions) + a resume dispatch, longest predicted first;
                             # kernel_ms spans both (ngt_amd_api.cpp run_search)
                             "search_dispatches": 2 if budget else 1,
                             "schedule_budget": budget},
                "cpu_baseline": cpu, "parity_sample": parity, "sweep": sweep}
            if qgm:
                line["config"]["result_expansion"] = args.expansion
        return line if rank == 0 else None

    line = measure_form(qgm)
    if args.pmc_launches:
        return
    if True:
        if also_qg and not qgm:
            # C5's form over the same shards: ngtqg quantize of every shard
            # (kmeansWithNGT codebooks from its first 1,600 objects, encoder,
            # quantized graph; QuantizedGraph.h:456-475), then the same
            # tuning, timing, all-gather + merge and oracle parity sample
            t1 = time.time()
            for sh in shards:
                h_base = np.zeros((min(N, 1600) + 1, D), np.float32)
                h_base[1:] = splitmix_uniform(min(N, 1600), D, BASE_SEED, row0=sh["off"])
                sh["qg_local"] = sh["ix"].qg_train_ngt(h_base, dsub=1)
                sh["ix"].qg_encode(return_codes=False)
                sh["ix"].qg_build_graph(None, args.qg_edges)
            torch.cuda.synchronize()
            log("shards quantized (NGTQG) in %.1f s" % (time.time() - t1))
            qline = measure_form(True)
            if rank == 0:
                qline.pop("sweep", None)
                qline["config"]["quantize_s"] = time.time() - t1
                line["qg_form"] = qline
    if rank == 0:
        if not emit:
            return line
        print(json.dumps(line), file=result_out, flush=True)
    if dist is not None and emit:
        dist.destroy_process_group()


def shard_parity_sample(args, shards, qdev, seeds, eps, merged, qgm, dist=None):
    """The first --shard-sample queries of the batch through the oracle on
    every shard (searchReadOnlyGraph restatement, or the NGTQG search from the
    oracle's own LUTs on the shard's codebooks), merged on the host by
    (distance, global id): ids and float bits must equal the device's merged
    results (abort otherwise).  With several ranks each rank runs the oracle
    on its own shards, the candidate lists are all-gathered (one object
    collective) and every rank checks the merge.  The oracle's time (the max
    over ranks) is the CPU baseline of the whole sharded index on the hosts'
    cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    K = args.k
    n = min(args.shard_sample, qdev.shape[0])
    h_q = qdev[:n].cpu().numpy()
    model, ncpu, threads = host_cpu()
    isa = O.host_isa()
    L = O.native_lib(isa)
    el = 0.0
    # per query: (distance, global id, distance bits) of every local shard's results
    cand = [[] for _ in range(n)]
    for sh in shards:
        h_rows = sh["rows"].cpu().numpy()
        h_off = sh["offsets"].cpu().numpy().astype(np.uint64)
        h_edges = sh["edges"].cpu().numpy().astype(np.uint32)
        if qgm:
            ids, codes = sh["ix"].qg_get_graph()
            deg = (ids != 0).sum(1).astype(np.uint64)
            qoff = np.zeros(len(deg) + 1, np.uint64)
            qoff[1:] = np.cumsum(deg)
            qg = {"M": args.dim, "qids": ids[ids != 0].astype(np.uint32), "qoff": qoff,
                  "code_off": np.arange(len(deg) + 1, dtype=np.uint64) * np.uint64(codes.shape[1]),
                  "codes": np.ascontiguousarray(codes.reshape(-1))}
            qgo = {"M": args.dim, "dim": args.dim, "dsub": 1, "global": np.zeros(args.dim, np.float32),
                   "local": oracle_codebooks(sh["qg_local"])}
            t0 = time.perf_counter()
            lut, sc, to = qg_luts_oracle(O, qgo, h_q, n)
            oi, od, on, _ = O.qg_search_batch(qg, h_rows, h_q, seeds[:n], K, eps, args.expansion, lut, sc, to,
                                              threads=threads, L=L)
        else:
            t0 = time.perf_counter()
            oi, od, on, _ = O.search_batch("l2", h_rows, h_off, h_edges, h_q, seeds[:n], K, np.float32(eps),
                                           edge_size=0, threads=threads, L=L)
        el += time.perf_counter() - t0
        bits = od.view(np.uint32)
        for q in range(n):
            for j in range(int(on[q])):
                cand[q].append((float(od[q, j]), int(oi[q, j]) + sh["off"], int(bits[q, j])))
        del h_rows, h_off, h_edges
    world = 1 if dist is None else dist.get_world_size()
    el_max, cores = el, threads
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, {"cand": cand, "el": el, "threads": threads})
        cand = [[c for g in got for c in g["cand"][q]] for q in range(n)]
        el_max = max(g["el"] for g in got)
        cores = sum(g["threads"] for g in got)
    gi = merged[0][:n].cpu().numpy().view(np.uint32)
    gd = merged[1][:n].cpu().numpy().view(np.uint32)
    gn = merged[2][:n].cpu().numpy()
    same = True
    for q in range(n):
        best = sorted(cand[q], key=lambda t: (t[0], t[1]))[:K]
        if int(gn[q]) != len(best) or any(int(gi[q, j]) != b[1] or int(gd[q, j]) != b[2]
                                          for j, b in enumerate(best)):
            same = False
            log("shard parity: query %d differs" % q)
            break
    nsh = len(shards) * world
    parity = {"queries": n, "identical": same, "shards": nsh,
              "checked": "merged ids and float32 distance bits vs the oracle on every shard + host merge"
                         + (" (each rank's shards on its own host cores, candidates all-gathered)" if world > 1
                            else "")}
    if not same:
        raise SystemExit("bench: sharded results differ from the oracle: %s" % parity)
    log("shard parity sample: %d queries identical to the oracle over %d shards (%.1f s on %d threads%s)" % (
        n, nsh, el_max, cores, ", max over %d ranks" % world if world > 1 else ""))
    what = "NGTQG search restatement (oracle LUTs)" if qgm else "searchReadOnlyGraph restatement"
    cpu = {"value": n / el_max, "unit": "queries/s", "cores": cores, "kind": "port",
           "sample": "first %d queries over all %d shards, oracle/ngt_oracle.c %s built -O3 -march=x86-64-%s, "
                     "one query per thread per shard on %d threads per rank x %d ranks, %.1f s (max over ranks); "
                     "host: %s, %d CPUs" % (n, nsh, what, isa, threads, world, el_max, model, ncpu),
           "all_physical_cores": all_cores_note(n / el_max, cores)}
    return cpu, parity


def capi_c_client(index_dir, Q, gt, D, K, eps, threads, plan=None, keep_ids=False):
    """tests/cxx/capi_threads.c compiled here with gcc against include/ and
    libngt_amd.so, run as a child process on the index directory: sequential
    single-query latency, `threads` concurrent callers and twice as many.
    The calls are answered by the resident serving grid (serve.cpp; its grid
    launches and answered calls are in each run's `launches` / `served`);
    requests it does not take fall back to group-committed launches."""
    exe = os.path.join(index_dir, "capi_threads")
    rc, _, err = run_reaped(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-o", exe,
                             os.path.join(ROOT, "tests", "cxx", "capi_threads.c"), "-L", os.path.join(ROOT, "ngt_amd"),
                             "-lngt_amd", "-Wl,-rpath," + os.path.join(ROOT, "ngt_amd"), "-lpthread", "-lm"], 120,
                            capture_stderr=True, what="gcc capi_threads.c")
    if rc != 0:
        raise SystemExit("bench: capi_threads.c did not compile: %s" % err[-2000:])
    qpath = os.path.join(index_dir, "queries.f32")
    np.ascontiguousarray(Q, np.float32).tofile(qpath)
    out = []
    for t, calls in plan or [(1, 300), (threads, 200), (2 * threads, 150)]:
        ids_path = os.path.join(index_dir, "ids.u32")
        rc, stdout, err = run_reaped([exe, index_dir, qpath, str(Q.shape[0]), str(D), str(K), repr(float(eps)), str(t),
                                      str(calls), ids_path], 600, env=dict(os.environ), capture_stderr=True,
                                     what="C client (%d threads)" % t)
        if rc != 0:
            raise SystemExit("bench: capi_threads failed: %s" % err[-2000:])
        res = json.loads(stdout.strip().splitlines()[-1])
        for ln in [x for x in err.splitlines() if x.startswith("[serve]")][:20]:
            log("C client %d threads: %s" % (t, ln))
        ids = np.fromfile(ids_path, np.uint32).reshape(-1, K).astype(np.int64)
        qi = np.arange(ids.shape[0]) % Q.shape[0]
        res["recall_at_10"] = recall_at(ids, gt[qi], K)
        if keep_ids:
            res["ids"] = ids
        out.append(res)
        log("C client: %d threads: %.0f QPS, latency mean %.3f ms p99 %.3f, recall %.4f (%d grid launches)" % (
            t, res["qps"], res["latency_ms"]["mean"], res["latency_ms"]["p99"], res["recall_at_10"],
            res.get("launches", -1)))
    return out


def physical_cores():
    """Physical cores of the host (lscpu: cores per socket x sockets), or None."""
    try:
        import subprocess
        per, sockets = None, None
        for line in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines():
            if line.startswith("Core(s) per socket:"):
                per = int(line.split(":", 1)[1])
            elif line.startswith("Socket(s):"):
                sockets = int(line.split(":", 1)[1])
        return per * sockets if per and sockets else None
    except (OSError, ValueError):
        return None


def all_cores_note(value, threads):
    """The CPU baseline scaled linearly to every physical core of the host (one
    query per thread, nothing shared: the best case for the CPU) -- the GPU/CPU
    ratio against the whole host is the reported ratio x threads / cores."""
    cores = physical_cores()
    if not cores:
        return None
    return {"physical_cores": cores, "value_at_all_physical_cores_linear": value * cores / threads,
            "ratio_factor": threads / float(cores),
            "note": "measured on %d threads (the lease's CPU affinity); at all %d physical cores, scaled linearly, "
                    "the CPU would reach %.0f queries/s, so every GPU/CPU ratio against this baseline shrinks by "
                    "x%.3f" % (threads, cores, value * cores / threads, threads / float(cores))}


def host_cpu():
    """lscpu's model name and CPU count, and the threads the baseline may use
    (the process's affinity, capped by OMP_NUM_THREADS when set)."""
    model, ncpu = "unknown", os.cpu_count() or 1
    try:
        import subprocess
        for line in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
            elif line.startswith("CPU(s):"):
                ncpu = int(line.split(":", 1)[1])
    except (OSError, ValueError):
        pass
    threads = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS"):
        threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    return model, ncpu, max(1, threads)


def scan_sample_check(rows, qdev, metric, k, gt_i, gt_d, gt_n, nsample=16):
    """The exact scan's results on the first nsample queries against the
    oracle's linearSearch restatement on all host cores: identical ids and
    distance bits required (abort otherwise)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    t0 = time.time()
    _, _, threads = host_cpu()
    h_rows = rows.cpu().numpy()
    h_q = qdev[:nsample].cpu().numpy()
    oi, od, on = O.linear_search_batch(metric, h_rows, h_q, k, threads=threads, L=O.native_lib(O.host_isa()))
    gi = gt_i[:nsample].cpu().numpy().view(np.uint32)
    gd = gt_d[:nsample].cpu().numpy()
    gn = gt_n[:nsample].cpu().numpy().view(np.uint32)
    same = bool(np.array_equal(on, gn))
    for q in range(nsample if same else 0):
        m = int(on[q])
        same = same and np.array_equal(oi[q, :m], gi[q, :m]) and np.array_equal(
            od[q, :m].view(np.uint32), gd[q, :m].view(np.uint32))
    if not same:
        raise SystemExit("bench: exact scan differs from the oracle on the sample")
    log("exact scan: %d-query oracle sample identical (%.1f s)" % (nsample, time.time() - t0))
    return {"queries": nsample, "identical": True}


def oracle_codebooks(local):
    """[M][16][dsub] centroids (local ids 1..16) -> the oracle's layout, the
    local codebook index's object slots [M][17][dsub] with the dummy slot 0
    (ObjectRepository.h:37-40; tests/golden/ngt_files.py read_qg)."""
    M, _, dsub = local.shape
    out = np.zeros((M, 17, dsub), np.float32)
    out[:, 1:, :] = local
    return out


def qg_luts_oracle(O, qgo, h_q, n):
    luts, scs, tos = [], [], []
    for i in range(n):
        lut, sc, to = O.qg_lut(qgo, h_q[i])
        luts.append(lut)
        scs.append(sc)
        tos.append(to)
    return np.stack(luts), np.array(scs, np.float32), np.array(tos, np.float32)


def cpu_baseline(args, ix, rows, offsets, edges, qdev, seeds, eps, metric, gpu_out, gpu_cnt, es_resolved=0,
                 qg_local=None):
    """The CPU baseline and the parity sample in one: the oracle restatement
    (oracle/ngt_oracle.c, the reference's 16-lane FMA order) built -O3 for the
    host's widest ISA (x86-64-v4 AVX-512, else v3) with one query per thread on
    every host core the process may use, on a bounded prefix of the same batch
    (same graph, seeds, epsilon; for qg the same quantized graph and LUTs).
    Its ids and float distances must equal the GPU's timed results bit for bit
    (abort otherwise); its distance counts must equal the GPU's full-visited-set
    counters (exact) or work counters (qg)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    t0 = time.time()
    h_rows = rows.cpu().numpy()
    h_off = offsets.cpu().numpy().astype(np.uint64)
    h_edges = edges.cpu().numpy().astype(np.uint32)
    h_q = qdev.cpu().numpy()
    model, ncpu, threads = host_cpu()
    isa = O.host_isa()
    L = O.native_lib(isa)
    qg = None
    if args.mode == "qg":
        ids, codes = ix.qg_get_graph()
        deg = (ids != 0).sum(1).astype(np.uint64)
        qoff = np.zeros(len(deg) + 1, np.uint64)
        qoff[1:] = np.cumsum(deg)
        qg = {"M": args.dim, "qids": ids[ids != 0].astype(np.uint32),
              "qoff": qoff, "code_off": (np.arange(len(deg) + 1, dtype=np.uint64) * np.uint64(codes.shape[1])),
              "codes": np.ascontiguousarray(codes.reshape(-1))}
        # the LUTs from the oracle's createDistanceLookup (Quantizer.h:709-760)
        # on the same codebooks: the sample checks LUT + ADC + search
        qgo = {"M": args.dim, "dim": args.dim, "dsub": 1, "global": np.zeros(args.dim, np.float32),
               "local": oracle_codebooks(qg_local)}
        lut, sc, to = qg_luts_oracle(O, qgo, h_q, min(h_q.shape[0], 20000))
    log("cpu baseline: host copy %.1f s; %s, %d CPUs, %d threads, oracle %s build" % (
        time.time() - t0, model, ncpu, threads, isa))

    def run(lo, hi):
        if qg is not None:
            return O.qg_search_batch(qg, h_rows, h_q[lo:hi], seeds[lo:hi], args.k, eps, args.expansion,
                                     lut[lo:hi], sc[lo:hi], to[lo:hi], threads=threads, L=L)
        return O.search_batch(metric, h_rows, h_off, h_edges, h_q[lo:hi], seeds[lo:hi], args.k, np.float32(eps),
                              edge_size=es_resolved, threads=threads, L=L)

    # size the sample to the time budget from a short probe
    nq = h_q.shape[0]
    probe = min(nq, 2 * threads)
    t0 = time.perf_counter()
    outs = [run(0, probe)]
    dt = time.perf_counter() - t0
    done = probe
    target = int(probe * max(0.0, args.cpu_seconds - dt) / max(dt, 1e-6))
    t1 = time.perf_counter()
    if target > 0 and done < nq:
        hi = min(nq, done + max(threads, target // threads * threads))
        outs.append(run(done, hi))
        done = hi
    el = dt + (time.perf_counter() - t1)
    ci = np.concatenate([o[0] for o in outs])
    cd = np.concatenate([o[1] for o in outs])
    cn = np.concatenate([o[2] for o in outs])
    cc = np.concatenate([o[3] for o in outs])
    gi, gd, gn = gpu_out
    same = bool(np.array_equal(cn, gn[:done]))
    for i in (range(done) if same else ()):
        n = int(cn[i])
        if not (np.array_equal(ci[i, :n], gi[i, :n]) and
                np.array_equal(cd[i, :n].view(np.uint32), gd[i, :n].view(np.uint32))):
            same = False
            log("parity sample: query %d differs: cpu %s / gpu %s" % (i, ci[i, :n].tolist(), gi[i, :n].tolist()))
            break
    if qg is not None:
        # ADC distances, accepted, expansions, exact distances: the same work
        cnt_same = bool(np.array_equal(cc[:, :4], gpu_cnt[:done, :4].astype(np.uint64)))
    else:
        # distinct distance computations (the full-visited-set run's counters)
        cnt_same = bool(np.array_equal(cc[:, 0], gpu_cnt[:done, 0].astype(np.uint64)))
    parity = {"queries": done, "identical": same, "work_counters_identical": cnt_same,
              "checked": "ids, float32 distance bits, result counts" + (
                  ", ADC/accepted/expansion/exact counts" if qg is not None else ", distinct distance counts")}
    if not (same and cnt_same):
        raise SystemExit("bench: the device results differ from the oracle on the parity sample: %s" % parity)
    log("parity sample: %d queries identical to the oracle (ids, distance bits, work counters)" % done)
    what = ("NGTQG::Index::searchQuantizedGraph restatement (LUT, ADC, search and rerank from the raw "
            "queries on the kmeansWithNGT codebooks)" if qg is not None
            else "searchReadOnlyGraph restatement")
    cal = calibration()
    base = {"value": done / el, "unit": "queries/s", "cores": threads, "kind": "port",
            "reference_equivalent_value": (done / el / cal["ratio_port_over_reference_1thread"]) if cal else None,
            "sample": "first %d of the %d queries (same graph, seeds, epsilon), oracle/ngt_oracle.c %s built -O3 "
                      "-march=x86-64-%s (16-lane FMA order kept), one query per thread on %d threads, %.1f s; "
                      "host: %s, %d CPUs" % (done, nq, what, isa, threads, el, model, ncpu),
            "all_physical_cores": all_cores_note(done / el, threads)}
    return base, parity


def reap_children():
    """Before exiting: any child process of this bench still alive (there
    should be none -- every child runs through run_reaped) is named on stderr
    and terminated, so nothing outlives the run."""
    import signal
    me = os.getpid()
    left = []
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open("/proc/%s/stat" % d) as f:
                st = f.read()
        except OSError:
            continue
        fields = st[st.rfind(")") + 2:].split()
        if len(fields) > 1 and fields[0] != "Z" and int(fields[1]) == me:
            left.append(int(d))
    for pid in left:
        try:
            with open("/proc/%d/cmdline" % pid, "rb") as f:
                cmd = f.read().replace(b"\0", b" ").decode(errors="replace").strip()
        except OSError:
            cmd = "?"
        print("[bench] child %d still running at exit (%s); terminating it" % (pid, cmd), file=sys.stderr, flush=True)
        try:
            os.kill(pid, signal.SIGTERM)
        except ProcessLookupError:
            pass


if __name__ == "__main__":
    rc = main() or 0
    reap_children()
    sys.exit(rc)
