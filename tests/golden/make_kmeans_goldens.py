#!/usr/bin/env python3
"""Fixtures pinning the NGTQG local-codebook training (kmeansWithNGT).

The reference's `ngtqg quantize` clusters each subspace with
NGT::Clustering::kmeansWithNGT, whose assignment searches run in an OpenMP
loop while the tree-seed thinning they call draws from the process-wide
rand() (lib/NGT/Index.h:1555-1559): with several threads its codebooks
change from run to run (two runs on the C1 ONNG agree on 55 of 128).  With
OMP_NUM_THREADS=1 it is deterministic; this script runs it that way (twice,
and requires identical output) on copies of c1_onng (dsub 1, M 128) and the
d20 index (dsub 4, M 5), and stores the local codebooks:

    tests/golden/qg_kmeans_st.npz   c1: [128][16] f32, d20: [5][16][4] f32

It also runs ngt_amd's restatement (ngt_amd/csrc/kmeans_ngt.h) with the
reference's own search through oracle/_ref/kmeans_harness and requires the
same centroids, bit for bit.  Reference binaries: oracle/ref.mk -> oracle/_ref/.
"""
import os
import shutil
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import ngt_files as F  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref")


def quantize(src, work, tag, extra):
    out = []
    for r in range(2):
        d = os.path.join(work, "%s_%d" % (tag, r))
        shutil.copytree(src, d, ignore=shutil.ignore_patterns("qg"))
        env = dict(os.environ, OMP_NUM_THREADS="1")
        subprocess.run([os.path.join(REF, "ngtqg"), "quantize"] + extra + [d], env=env, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=work)
        out.append(d)
    return out


def codebooks(index, M, dsub):
    cb = np.zeros((M, 16, dsub), np.float32)
    for m in range(M):
        rows, _ = F.read_obj(os.path.join(index, "qg", "local-%d" % m, "obj"), dsub, np.float32)
        cb[m] = rows[1:17, :dsub]
    return cb


def harness(rows, M, dsub, work):
    cb = np.zeros((M, 16, dsub), np.float32)
    for m in range(M):
        v = np.ascontiguousarray(rows[1:1601, m * dsub:(m + 1) * dsub], dtype=np.float32)
        path = os.path.join(work, "km.bin")
        with open(path, "wb") as f:
            f.write(struct.pack("<II", v.shape[0], dsub))
            f.write(v.tobytes())
        out = subprocess.run([os.path.join(REF, "kmeans_harness"), path, "0"], capture_output=True, text=True,
                             check=True).stdout
        cb[m] = np.array([float(x) for x in out.split()], np.float32).reshape(16, dsub)
    return cb


def main():
    work = tempfile.mkdtemp(prefix="ngt_kmeans_")
    res = {}
    for tag, src, dim, dsub, extra in (("c1", os.path.join(HERE, "c1_onng"), 128, 1, ["-E", "128"]),
                                       ("d20", os.path.join(HERE, "d20_qg"), 20, 4, ["-Q", "4", "-E", "64"])):
        M = dim // dsub
        a, b = quantize(src, work, tag, extra)
        ca, cbk = codebooks(a, M, dsub), codebooks(b, M, dsub)
        assert np.array_equal(ca.view(np.uint32), cbk.view(np.uint32)), "single-thread runs differ: " + tag
        rows, _ = F.read_obj(os.path.join(src, "obj"), dim, np.float32)
        ch = harness(rows, M, dsub, work)
        assert np.array_equal(ca.view(np.uint32), ch.view(np.uint32)), "restatement differs: " + tag
        res[tag] = ca.reshape(M, 16) if dsub == 1 else ca
        import hashlib
        for f in ("ivt", "grp"):
            print(tag, "qg/%s sha256" % f, hashlib.sha256(open(os.path.join(a, "qg", f), "rb").read()).hexdigest())
        print(tag, "M", M, "dsub", dsub, ": two single-thread reference runs and the restatement agree")
    np.savez(os.path.join(HERE, "qg_kmeans_st.npz"), **res)
    shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
