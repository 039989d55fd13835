"""Reference builds of the C1 data at other creation batch sizes.

``ngt create -d 128 -o f -D 2 -b <B>`` (Command.cpp:41, batchSizeForCreation,
used by Index.cpp:1297 to cut the insertion batches) of tests/golden/sift5k.npy
with the reference CLI compiled by oracle/ref.mk (oracle/_ref/ngt).  Writes
``c1_anng_b<B>/{grp,tre}`` for B in 1000, 5000 (one batch holds the whole data
set); the objects are c1_anng's.  Run from the repo root after build()."""
import argparse
import os
import shutil
import subprocess

import numpy as np


def main():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap = argparse.ArgumentParser()
    ap.add_argument("--ngt", default=os.path.join(root, "oracle", "_ref", "ngt"))
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--work", default="/tmp/ngt_batch_goldens")
    ap.add_argument("--batches", default="1000,5000")
    args = ap.parse_args()
    shutil.rmtree(args.work, ignore_errors=True)
    os.makedirs(args.work)
    sift = np.load(os.path.join(args.out, "sift5k.npy"))
    tsv = os.path.join(args.work, "sift5k.tsv")
    with open(tsv, "w") as f:
        for r in sift:
            f.write("\t".join("%d" % v for v in r) + "\n")
    for b in (int(x) for x in args.batches.split(",")):
        name = "c1_anng_b%d" % b
        r = subprocess.run([args.ngt, "create", "-d", "128", "-o", "f", "-D", "2", "-b", str(b), name, tsv],
                           cwd=args.work, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("ngt create -b %d failed:\n%s" % (b, r.stderr[-2000:]))
        dst = os.path.join(args.out, name)
        os.makedirs(dst, exist_ok=True)
        for f in ("grp", "tre", "prf"):
            shutil.copy(os.path.join(args.work, name, f), os.path.join(dst, f))
        print(name, "written")


if __name__ == "__main__":
    main()
