#!/usr/bin/env python3
"""Offline: how well cheap per-query features predict a query's search cost
(expansions, from a bench dump: NGT_BENCH_ORDER=1 NGT_BENCH_DUMP=...), and
the makespan of the single launch's list scheduling (S persistent slots pull
queries in order) under each ordering.  CPU only; regenerates the bench's
splitmix64 data and queries.
  order_predictors.py <dump.npz> [slots=4096] [sample=1024]"""
import heapq
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from bench import BASE_SEED, splitmix_uniform  # noqa: E402

dump = np.load(sys.argv[1])
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
S = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
ne = dump["expansions"].astype(np.float64)
NQ = len(ne)
N, D = 1_000_000, 128
X = splitmix_uniform(N, D, BASE_SEED)
Q = splitmix_uniform(NQ, D, BASE_SEED + 1)


def makespan(order, cost):
    h = [0.0] * slots
    heapq.heapify(h)
    end = 0.0
    for i in order:
        t = heapq.heappop(h) + cost[i]
        end = max(end, t)
        heapq.heappush(h, t)
    return end


def spearman(a, b):
    ra = np.argsort(np.argsort(a))
    rb = np.argsort(np.argsort(b))
    return float(np.corrcoef(ra, rb)[0, 1])


rng = np.random.default_rng(1)
samp = X[rng.choice(N, S, replace=False)]
d2 = (Q * Q).sum(1)[:, None] + (samp * samp).sum(1)[None, :] - 2.0 * Q @ samp.T
d = np.sqrt(np.maximum(d2, 0))
mn, mu, sd = d.min(1), d.mean(1), d.std(1)
cen = X.mean(0)
feats = {
    "centroid_dist": np.linalg.norm(Q - cen, axis=1),
    "sample_min": mn,
    "sample_mean": mu,
    "sample_contrast(mean/min)": mu / mn,
    "sample_z(mean-min)/sd": (mu - mn) / sd,
    "sample_cv(sd/mean)": sd / mu,
    "sample_min_over_mean": mn / mu,
}
base = makespan(range(NQ), ne)
ideal = ne.sum() / slots
print("queries %d slots %d: given order makespan %.0f (ideal %.0f, %.3f of it)" % (NQ, slots, base, ideal, ideal / base))
print("oracle LPT: %.3f of given" % (makespan(np.argsort(-ne), ne) / base))
for k, f in feats.items():
    r = spearman(f, ne)
    o = np.argsort(-f) if r > 0 else np.argsort(f)
    print("%-28s spearman %+.3f  makespan %.3f of given" % (k, r, makespan(o, ne) / base))

# moment predictor: squared distance to a random data row has mean mu_q and
# (independent dimensions) variance var_q from the data's per-dimension raw
# moments; the ball (1+eps) r_k holds more rows the larger mu_q / sd_q
m = [np.mean(X.astype(np.float64) ** p, axis=0) for p in (1, 2, 3, 4)]
q = Q.astype(np.float64)
e2 = q * q - 2 * q * m[0] + m[1]
e4 = q ** 4 - 4 * q ** 3 * m[0] + 6 * q * q * m[1] - 4 * q * m[2] + m[3]
mu = e2.sum(1)
var = (e4 - e2 * e2).sum(1)
for k, f in {"moment_mu/sd": mu / np.sqrt(var), "moment_mu": mu, "moment_sd": np.sqrt(var)}.items():
    r = spearman(f, ne)
    o = np.argsort(-f) if r > 0 else np.argsort(f)
    print("%-28s spearman %+.3f  makespan %.3f of given" % (k, r, makespan(o, ne) / base))
# the exploration ball itself (brute force over a row subsample, scaled)
eps = float(dump["epsilon"])
sub = X[::10]
dd = (Q * Q).sum(1)[:, None] + (sub * sub).sum(1)[None, :] - 2.0 * Q @ sub.T
dd = np.sqrt(np.maximum(dd, 0))
rk = np.sort(dd, axis=1)[:, 0]  # ~ the 10th neighbour of the full set
ball = ((dd <= (1 + eps) * rk[:, None]).sum(1)).astype(np.float64)
r = spearman(ball, ne)
print("%-28s spearman %+.3f  makespan %.3f of given" % ("ball((1+eps) r_10)/10", r, makespan(np.argsort(-ball), ne) / base))
