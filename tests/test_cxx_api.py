"""The C++ facade (include/NGT/Index.h, include/NGT/NGTQ/QuantizedGraph.h):
tests/cxx/ngt_sample.cpp, a program in the style of the reference's
samples/cosine-float/cosine-float.cpp:17-100, compiled against include/ and
linked with libngt_amd.so, must reproduce the reference's own results
(tests/golden) -- searches, linear search, graph-only search, NGTQG search,
index construction -- through NGT::Index / NGT::SearchQuery /
NGT::SearchContainer / NGTQG::Index."""
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import ngt_files as F
import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def sample(tmp_path_factory):
    d = tmp_path_factory.mktemp("cxx")
    exe = str(d / "ngt_sample")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                           "-o", exe, os.path.join(ROOT, "tests", "cxx", "ngt_sample.cpp"),
                           "-L", os.path.join(ROOT, "ngt_amd"), "-lngt_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "ngt_amd")])
    q = np.load(os.path.join(GOLD, "queries.npy"))
    qf = str(d / "queries.tsv")
    with open(qf, "w") as f:
        for r in q:
            f.write("\t".join(str(int(x)) for x in r) + "\n")
    return exe, qf, d


def run(exe, *args):
    r = subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True)
    if r.returncode != 0:
        raise AssertionError("ngt_sample %s: %s" % (args, r.stderr))
    return r.stdout


def parse(out, nq, k):
    ids = np.zeros((nq, k), np.int64) - 1
    bits = np.zeros((nq, k), np.uint32)
    nd = {}
    first = {}
    for line in out.splitlines():
        if line.startswith("# "):
            q, v = line[2:].split(" distances=")
            nd[int(q)] = int(v)
            continue
        if line.startswith("@ "):
            q, b = line[2:].split()
            first[int(q)] = int(b, 16)
            continue
        q, rank, i, b = line.split()
        ids[int(q), int(rank) - 1] = int(i)
        bits[int(q), int(rank) - 1] = int(b, 16)
    return ids, bits.view(np.float32), nd, first


def test_sample_compiles_and_reads_accuracy_table(sample):
    """CPU: the facade compiles warning-free against include/, and
    getEpsilonFromExpectedAccuracy restates AccuracyTable::getEpsilon
    (Index.h:316-347) over the prf's table."""
    exe, qf, d = sample
    prop = F.read_prf(os.path.join(GOLD, "c1_onng", "prf"))
    table = [(np.float32(a), float(b)) for a, b in (t.split(":") for t in prop["AccuracyTable"].split(","))]
    for acc in (0.5, 0.8, 0.95, 0.99, 1.2):
        a = min(acc, 1.0)
        i = next((j for j, t in enumerate(table) if t[1] >= a), len(table))
        i = i - 2 if i == len(table) else (i - 1 if i else 0)
        lo, up = table[i], table[i + 1]
        e = np.float32(lo[0] + np.float64(np.float32(up[0] - lo[0])) * (a - lo[1]) / (up[1] - lo[1]))
        got = float(run(exe, "accuracy", os.path.join(GOLD, "c1_onng"), acc))
        assert np.float32(got) == max(e, np.float32(-0.9)), acc


@pytest.mark.gpu
def test_cxx_search_matches_reference(sample):
    """Single-query searches through the C++ facade (the serving grid of the
    latency kernel): ids and distance counts equal the reference's goldens,
    and the distance bits equal the pinned oracle's restatement of
    NeighborhoodGraph::search over the same index (the goldens hold the
    reference CLI's printed distances, 6 significant digits)."""
    exe, qf, d = sample
    ids, ds, nd, first = parse(run(exe, "search", os.path.join(GOLD, "c1_anng"), qf, 10, 0.1), 100, 10)
    g = np.load(os.path.join(GOLD, "search_c1_anng_tw_0.1.npz"))
    name = os.path.join(GOLD, "c1_anng")
    prop = F.read_prf(os.path.join(name, "prf"))
    rows, _ = F.read_obj(os.path.join(name, "obj"), 128, np.float32)
    offs, gids, _ = F.read_grp(os.path.join(name, "grp"))
    tree = F.read_tre(os.path.join(name, "tre"), 128, np.float32)
    es = int(prop["EdgeSizeForSearch"])
    qs = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    for i in range(100):
        ref = g["ids"][i][g["ids"][i] >= 0]
        assert list(ids[i, :len(ref)]) == list(ref), i
        assert ["%g" % x for x in ds[i, :len(ref)]] == ["%g" % x for x in g["dists"][i][:len(ref)]], i
        seeds, _, _ = O.tree_seeds("l2", tree, qs[i], 10, int(prop["SeedSize"]))
        oid, od, _ = O.search("l2", rows, offs, gids, qs[i], seeds, 10, np.float32(0.1), edge_size=es)
        assert list(oid) == list(ref), i
        assert np.array_equal(ds[i, :len(ref)].view(np.uint32), od.view(np.uint32)), i
        # sc.distanceComputationCount of the reference's read-write search
        assert nd[i] == int(g["ndist"][i]), i
        assert first[i] == int(rows[ref[0], 0].view(np.uint32))  # getObjectSpace().getObject


@pytest.mark.gpu
def test_cxx_linear_and_graph_only_match_reference(sample):
    exe, qf, d = sample
    ids, ds, _, _ = parse(run(exe, "linear", os.path.join(GOLD, "c1_anng"), qf, 10), 100, 10)
    g = np.load(os.path.join(GOLD, "search_c1_anng_sr_0.0.npz"))
    for i in range(100):
        assert list(ids[i]) == list(g["ids"][i]), i
    # searchUsingOnlyGraph with the SearchContainer(Object&) form: random seeds
    # from a fresh process's rand() stream, as `ngt search -i g`
    ids, ds, _, _ = parse(run(exe, "search", os.path.join(GOLD, "c1_anng"), qf, 10, 0.1, "graph"), 100, 10)
    g = np.load(os.path.join(GOLD, "search_c1_anng_gw_0.1.npz"))
    for i in range(100):
        ref = g["ids"][i][g["ids"][i] >= 0]
        assert list(ids[i, :len(ref)]) == list(ref), i


@pytest.mark.gpu
def test_cxx_create_matches_reference_build(sample):
    """create -> append -> createIndex(16) -> save through NGT::Index builds the
    reference CLI's C1 index byte for byte (`ngt create -d 128 -o f -D 2`)."""
    exe, qf, d = sample
    data = str(d / "sift5k.tsv")
    rows = np.load(os.path.join(GOLD, "sift5k.npy"))
    with open(data, "w") as f:
        for r in rows:
            f.write("\t".join(str(int(x)) for x in r) + "\n")
    idx = str(d / "c1_cxx")
    out = run(exe, "create", idx, data, 128, "L2", 40)
    assert out.strip() == "objects 5000"
    for f in ("obj", "grp", "tre"):
        assert open(os.path.join(idx, f), "rb").read() == open(os.path.join(GOLD, "c1_anng", f), "rb").read(), f


@pytest.mark.gpu
def test_cxx_cosine_sample_flow(sample):
    """The cosine-float sample's own flow (Cosine, default property): the saved
    index searched through NGT::Index equals the oracle over its files."""
    exe, qf, d = sample
    data = str(d / "sift5k_c.tsv")
    rows = np.load(os.path.join(GOLD, "sift5k.npy"))[:3000].astype(np.float32) * np.float32(0.37) + np.float32(0.013)
    with open(data, "w") as f:
        for r in rows:
            f.write("\t".join("%.9g" % x for x in r) + "\n")
    idx = str(d / "cos_cxx")
    run(exe, "create", idx, data, 128, "Cosine")
    prop = F.read_prf(os.path.join(idx, "prf"))
    srows, _ = F.read_obj(os.path.join(idx, "obj"), 128, np.float32)
    offs, eids, _ = F.read_grp(os.path.join(idx, "grp"))
    tree = F.read_tre(os.path.join(idx, "tre"), 128, np.float32)
    ids, ds, nd, _ = parse(run(exe, "search", idx, qf, 10, 0.1), 100, 10)
    q = np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)
    es = int(prop["EdgeSizeForSearch"])
    for i in range(100):
        seeds, _, _ = O.tree_seeds("cosine", tree, q[i], 10, int(prop["SeedSize"]))
        oid, od, ocnt = O.search("cosine", srows, offs, eids, q[i], seeds, 10, np.float32(0.1), edge_size=es)
        assert list(ids[i, :len(oid)]) == list(oid), i
        assert np.array_equal(ds[i, :len(oid)].view(np.uint32), od.view(np.uint32)), i
        assert nd[i] == int(ocnt[0]) - len(seeds), i


@pytest.mark.gpu
def test_cxx_ngtqg_matches_reference(sample):
    """NGTQG::Index(path) + NGTQG::SearchQuery::setResultExpansion + search on the
    reference's C1 quantizer (tests/golden/c1_qg): the reference's own results."""
    exe, qf, d = sample
    idx = str(d / "c1_qg_cxx")
    shutil.copytree(os.path.join(GOLD, "c1_onng"), idx)
    shutil.copytree(os.path.join(GOLD, "c1_qg", "qg"), os.path.join(idx, "qg"))
    z = np.load(os.path.join(GOLD, "c1_qg", "goldens.npz"))
    qs = z["queries"].astype(np.float32)
    qq = str(d / "qg_queries.tsv")
    with open(qq, "w") as f:
        for r in qs:
            f.write("\t".join("%.9g" % x for x in r) + "\n")
    for key in ("10_0.05_3", "20_0.03_3", "10_0.1_2"):
        k, eps, exp = key.split("_")
        ids, ds, _, _ = parse(run(exe, "qg", idx, qq, k, eps, exp), len(qs), int(k))
        for i in range(len(qs)):
            n = int(z["n_" + key][i])
            assert list(ids[i, :n]) == list(z["ids_" + key][i][:n]), (key, i)
            assert np.array_equal(ds[i, :n].view(np.uint32), z["dist_" + key][i][:n].view(np.uint32)), (key, i)


@pytest.mark.gpu
def test_cxx_ngtq_search_matches_reference(sample):
    """NGTQ::Index(path) + search(object, objs, size, expansion, mode, epsilon)
    through include/NGT/NGTQ/Quantizer.h reproduce the reference's
    NGTQ::Index::search (tests/golden/ngtq_n16, make_ngtq_goldens.py)."""
    exe, qf, d = sample
    idx = str(d / "ngtq_n16")
    shutil.copytree(os.path.join(GOLD, "ngtq_n16"), idx)
    rows, _ = F.read_obj(os.path.join(GOLD, "c1_anng", "obj"), 128, np.float32)
    F.write_array_file(os.path.join(idx, "obj"), rows[:, :128])
    z = np.load(os.path.join(GOLD, "ngtq_n16", "goldens.npz"))
    qtsv = str(d / "ngtq_q.tsv")
    with open(qtsv, "w") as f:
        for r in z["queries"]:
            f.write("\t".join("%.9g" % x for x in r) + "\n")
    for m, size, exp, eps, key in [("l", 10, 4, "0.1", "l_10_4_0p1"), ("r", 20, 8, "0.05", "r_20_8_0p05"),
                                   ("c", 10, 16, "-", "c_10_16_m1")]:
        ids, ds, _, _ = parse(run(exe, "ngtq", idx, qtsv, size, exp, m, eps), len(z["queries"]), size)
        for i in range(len(z["queries"])):
            n = int(z["n_" + key][i])
            assert list(ids[i, :n]) == list(z["ids_" + key][i, :n]), (key, i)
            assert np.array_equal(ds[i, :n].view(np.uint32), z["d_" + key][i, :n].view(np.uint32)), (key, i)
