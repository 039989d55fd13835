#!/usr/bin/env python3
"""Exact scan (ngt_amd_linear_search_device) on C2/C3-shaped data: the
matrix-core filtered scan (scan_mfma.hip, default), the query-tiled FMA scan
(scan_kernels.hip, NGT_AMD_LINEAR_MFMA=0) and the quad-per-row kernel
(NGT_AMD_LINEAR_MFMA=0 NGT_AMD_LINEAR_TILED=0), each in a child process --
identical ids and distance bits required -- and their times.
usage: linear_check.py [n] [nq] [dim] [k] [metric] [modes]
  metric: l2 | cosine; modes: comma list of mfma,tiled,quad (default all
  that support the metric)"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ENVS = {"mfma": {}, "tiled": {"NGT_AMD_LINEAR_MFMA": "0"},
        "quad": {"NGT_AMD_LINEAR_MFMA": "0", "NGT_AMD_LINEAR_TILED": "0"}}


def run(n, nq, dim, k, metric, out):
    import torch
    import bench
    from ngt_amd.device import DeviceIndex
    dev = torch.device("cuda:0")
    dp = (dim + 15) // 16 * 16  # device rows and prepared queries are padded to dp floats
    rows = torch.zeros((n + 1, dp), dtype=torch.float32, device=dev)
    rows[1:, :dim] = torch.from_numpy(bench.splitmix_uniform(n, dim, bench.BASE_SEED)).to(dev)
    q = torch.zeros((nq, dp), dtype=torch.float32, device=dev)
    q[:, :dim] = torch.from_numpy(bench.splitmix_uniform(nq, dim, bench.BASE_SEED + 1)).to(dev)
    ix = DeviceIndex(metric, "float", dim)
    ix.set_objects_device(rows.data_ptr(), n + 1)
    oi = torch.zeros((nq, k), dtype=torch.int32, device=dev)
    od = torch.zeros((nq, k), dtype=torch.float32, device=dev)
    on = torch.zeros((nq,), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    times = []
    for rep in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        ix.linear_search_device(q.data_ptr(), dp * 4, nq, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(),
                                stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    np.savez(out, ids=oi.cpu().numpy(), d=od.cpu().numpy(), n=on.cpu().numpy(), ms=np.array(times))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        run(*[int(x) for x in sys.argv[2:6]], sys.argv[6], sys.argv[7])
        sys.exit(0)
    args = sys.argv[1:] + ["1000000", "10000", "128", "10", "l2", ""][len(sys.argv) - 1:]
    n, nq, dim, k = [int(x) for x in args[:4]]
    metric = args[4]
    modes = [m for m in (args[5] or "mfma,tiled,quad").split(",") if m]
    if metric != "l2":
        modes = [m for m in modes if m != "tiled"]
    res = {}
    for m in modes:
        out = "/tmp/lin_%s.npz" % m
        env = dict(os.environ, **ENVS[m])
        subprocess.check_call([sys.executable, __file__, "--child", str(n), str(nq), str(dim), str(k), metric, out],
                              env=env)
        res[m] = np.load(out)
    base = res[modes[-1]]
    line = {"n": n, "nq": nq, "dim": dim, "k": k, "metric": metric}
    same = True
    flop = 3.0 * n * nq * ((dim - 1) // 16 + 1) * 16  # the comparator's sub + FMA per dimension
    for m in modes:
        a = res[m]
        eq = (np.array_equal(a["n"], base["n"]) and np.array_equal(a["ids"], base["ids"]) and
              np.array_equal(a["d"].view(np.uint32), base["d"].view(np.uint32)))
        same = same and eq
        ms = float(np.min(a["ms"][1:]))
        line[m] = {"ms": a["ms"].tolist(), "identical_to_%s" % modes[-1]: bool(eq), "qps": nq / (ms * 1e-3),
                   "effective_tflops": flop / (ms * 1e-3) / 1e12}
    line["identical"] = bool(same)
    print(json.dumps(line))
    sys.exit(0 if same else 1)
