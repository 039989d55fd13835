#!/usr/bin/env python3
"""Exact scan (ngt_amd_linear_search_device) on C2-shaped data: the tiled
kernel (scan_kernels.hip) against the quad-per-row kernel (NGT_AMD_LINEAR_TILED=0
in a child process) -- identical ids and distance bits -- and its time.
usage: linear_check.py [n] [nq] [dim] [k]"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n, nq, dim, k, out):
    import torch
    import bench
    from ngt_amd.device import DeviceIndex
    dev = torch.device("cuda:0")
    dp = (dim + 15) // 16 * 16  # device rows and prepared queries are padded to dp floats
    rows = torch.zeros((n + 1, dp), dtype=torch.float32, device=dev)
    rows[1:, :dim] = torch.from_numpy(bench.splitmix_uniform(n, dim, bench.BASE_SEED)).to(dev)
    q = torch.zeros((nq, dp), dtype=torch.float32, device=dev)
    q[:, :dim] = torch.from_numpy(bench.splitmix_uniform(nq, dim, bench.BASE_SEED + 1)).to(dev)
    ix = DeviceIndex("l2", "float", dim)
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
        run(*[int(x) for x in sys.argv[2:6]], sys.argv[6])
        sys.exit(0)
    n, nq, dim, k = [int(x) for x in (sys.argv[1:5] + ["1000000", "10000", "128", "10"][len(sys.argv) - 1:])]
    res = {}
    for tiled in ("1", "0"):
        out = "/tmp/lin_%s.npz" % tiled
        env = dict(os.environ, NGT_AMD_LINEAR_TILED=tiled)
        subprocess.check_call([sys.executable, __file__, "--child", str(n), str(nq), str(dim), str(k), out], env=env)
        res[tiled] = np.load(out)
    a, b = res["1"], res["0"]
    same = (np.array_equal(a["n"], b["n"]) and np.array_equal(a["ids"], b["ids"]) and
            np.array_equal(a["d"].view(np.uint32), b["d"].view(np.uint32)))
    ms = float(np.min(a["ms"][1:]))
    flop = 3.0 * n * nq * ((dim - 1) // 16 + 1) * 16
    print(json.dumps({"n": n, "nq": nq, "dim": dim, "k": k, "identical": bool(same),
                      "tiled_ms": a["ms"].tolist(), "quad_ms": b["ms"].tolist(),
                      "tiled_tflops": flop / (ms * 1e-3) / 1e12, "frac_of_157": flop / (ms * 1e-3) / 157.3e12,
                      "qps": nq / (ms * 1e-3)}))
    sys.exit(0 if same else 1)
