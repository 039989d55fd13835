#!/usr/bin/env python3
"""Fixture: the epsilon NGT's Index::AccuracyTable::getEpsilon (Index.h:293-346)
maps expected accuracies to, for the AccuracyTable of the reference-built C1
ONNG (tests/golden/c1_onng/prf), from oracle/_ref/accuracy_harness (built by
`make -f oracle/ref.mk` against the reference's own headers).  Writes
accuracy_c1_onng.json: [[accuracy float bits, epsilon float bits], ...]."""
import argparse
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def accuracies():
    table = open(os.path.join(HERE, "c1_onng", "prf")).read().split("AccuracyTable\t")[1].split("\n")[0]
    pts = [float(t.split(":")[1]) for t in table.split(",")]
    grid = list(np.linspace(0.0, 1.2, 121)) + pts + [p + 1e-4 for p in pts] + [p - 1e-4 for p in pts]
    return sorted({float(np.float32(a)) for a in grid if a > 0.0})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    acc = accuracies()
    exe = os.path.join(ROOT, "oracle", "_ref", "accuracy_harness")
    out = subprocess.check_output([exe, os.path.join(HERE, "c1_onng", "prf")] + [repr(a) for a in acc]).decode()
    pairs = [[int(x) for x in l.split()] for l in out.splitlines()]
    assert len(pairs) == len(acc)
    with open(os.path.join(args.out, "accuracy_c1_onng.json"), "w") as f:
        json.dump({"source": "oracle/_ref/accuracy_harness tests/golden/c1_onng/prf (Index::AccuracyTable::getEpsilon)",
                   "pairs": pairs}, f)


if __name__ == "__main__":
    main()
