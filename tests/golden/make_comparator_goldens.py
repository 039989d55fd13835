#!/usr/bin/env python3
"""Comparator and normalization fixtures from the reference's own code.

Development container only (never on the GPU box):

    make -f oracle/ref.mk
    python3 tests/golden/make_comparator_goldens.py

Runs oracle/_ref/comparator_harness (tests/golden/comparator_harness.cpp,
compiled against /root/reference's headers with the reference's flags) on
seeded inputs and writes:

* ``pair_sparse_jaccard_f_d<D>.npz`` -- compareSparseJaccardDistance
  (lib/NGT/PrimitiveComparator.h:399-418) on 0-terminated ascending id lists
  stored as float bit patterns (Index::makeSparseObject, Index.cpp:304-320),
  including empty lists and lists that fill the whole row;
* ``pair_<normalized metric>_c_d<D>.npz`` -- the uint8 dot-product family
  (compareDotProduct(const uint8_t*), :479-485, under compareNormalizedL2 /
  compareNormalizedCosineSimilarity / compareNormalizedAngleDistance);
* ``norm_f_d<D>.npz`` -- ObjectSpace::normalize (ObjectSpace.h:251-266) of
  float rows: the stored form of objects and queries of the normalized metrics.

Each pair file holds ``a``, ``b`` (padded rows), ``dist`` (float32 as the
search loop stores it) and ``dim`` / ``dp``.
"""
import argparse
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def harness(bin_, *args):
    subprocess.run([bin_] + [str(a) for a in args], check=True)


def sparse_rows(rng, n, dim):
    """n rows of dim+1 slots (the object space of SparseJaccard has dimension+1,
    Index.cpp:488-490), padded to a multiple of 16: ascending distinct ids in
    [1, 4 * dim], 0-terminated, stored as float bit patterns."""
    dp = ((dim + 1 - 1) // 16 + 1) * 16
    out = np.zeros((n, dp), np.uint32)
    for i in range(n):
        if i % 17 == 0:
            m = 0                    # empty list
        elif i % 17 == 1:
            m = dim                  # full row (dim ids + the terminator)
        else:
            m = int(rng.integers(1, dim + 1))
        ids = np.sort(rng.choice(np.arange(1, 4 * dim + 1), size=m, replace=False)).astype(np.uint32)
        out[i, :m] = ids
    return out.view(np.float32), dp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bin", default=os.path.join(ROOT, "oracle", "_ref", "comparator_harness"))
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--n", type=int, default=2000)
    args = ap.parse_args()
    rng = np.random.default_rng(0x5A4C)
    with tempfile.TemporaryDirectory() as td:
        def run_pairs(metric, ot, a, b, dp):
            fa, fb, fo = (os.path.join(td, x) for x in ("a.bin", "b.bin", "o.bin"))
            a.tofile(fa)
            b.tofile(fb)
            harness(args.bin, "dist", metric, ot, dp, fa, fb, a.shape[0], fo)
            return np.fromfile(fo, np.float32)

        for dim in (31, 100):
            a, dp = sparse_rows(rng, args.n, dim)
            b, _ = sparse_rows(rng, args.n, dim)
            # overlapping lists: half of the b rows share a prefix with their a row
            for i in range(0, args.n, 2):
                ai = a[i].view(np.uint32)
                m = int((ai != 0).sum())
                if m:
                    keep = ai[:m][rng.random(m) < 0.6]
                    extra = rng.choice(np.arange(1, 4 * dim + 1), size=max(0, min(dim, m) - len(keep)), replace=False)
                    ids = np.unique(np.concatenate([keep, extra.astype(np.uint32)]))[:dim]
                    row = np.zeros(dp, np.uint32)
                    row[:len(ids)] = ids
                    b[i] = row.view(np.float32)
            d = run_pairs("sparse_jaccard", "f", a, b, dp)
            np.savez_compressed(os.path.join(args.out, "pair_sparse_jaccard_f_d%d.npz" % dim),
                                a=a, b=b, dist=d, dim=dim, dp=dp)
            print("sparse_jaccard d%d: %d pairs" % (dim, args.n))

        for metric in ("normalized_cosine", "normalized_angle", "normalized_l2"):
            for dim in (100, 128):
                dp = ((dim - 1) // 16 + 1) * 16
                a = np.zeros((args.n, dp), np.uint8)
                b = np.zeros((args.n, dp), np.uint8)
                # small values keep dot products in the range where the metric is defined
                a[:, :dim] = rng.integers(0, 3, size=(args.n, dim))
                b[:, :dim] = rng.integers(0, 3, size=(args.n, dim))
                d = run_pairs(metric, "c", a, b, dp)
                np.savez_compressed(os.path.join(args.out, "pair_%s_c_d%d.npz" % (metric, dim)),
                                    a=a, b=b, dist=d, dim=dim, dp=dp)
                print("%s c d%d: %d pairs" % (metric, dim, args.n))

        for dim in (20, 100, 128, 960):
            x = (rng.random((256, dim), dtype=np.float32) * np.float32(2.0) - np.float32(0.7)).astype(np.float32)
            fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
            x.tofile(fi)
            harness(args.bin, "normalize", dim, fi, x.shape[0], fo)
            y = np.fromfile(fo, np.float32).reshape(x.shape)
            np.savez_compressed(os.path.join(args.out, "norm_f_d%d.npz" % dim), x=x, y=y, dim=dim)
            print("normalize d%d" % dim)


if __name__ == "__main__":
    main()
