"""GPU parity of the NGTQG path (qg_kernels.hip through the C ABI) against the
reference's own outputs (tests/golden/*_qg, made by make_qg_goldens.py from
the reference library) and against the CPU restatement (oracle/).

Bar: LUT bytes, scale and totalOffset bit-exact; ADC distances bit-exact;
NGTQG::Index::search ids and float distances identical for every
(k, epsilon, result_expansion) the fixtures hold."""
import json
import os

import numpy as np
import pytest

import ngt_files as F
import oracle_py as O
from ngt_amd.device import SEED_GIVEN, SEED_TREE, DeviceIndex, NativeError

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = {"c1_qg": ("c1_onng", 128, 128), "d20_qg": ("d20_qg", 20, 64)}
_CACHE = {}


def state(name):
    if name not in _CACHE:
        src, dim, maxe = CASES[name]
        offs, ids, _ = F.read_grp(os.path.join(GOLD, src, "grp"))
        qg = F.read_qg(os.path.join(GOLD, name), offs, ids, maxe)
        rows, valid = F.read_obj(os.path.join(GOLD, src, "obj"), dim, np.float32)
        tree = F.read_tre(os.path.join(GOLD, src, "tre"), dim, np.float32)
        prop = F.read_prf(os.path.join(GOLD, src, "prf"))
        z = dict(np.load(os.path.join(GOLD, name, "goldens.npz")))
        meta = json.load(open(os.path.join(GOLD, name, "meta.json")))
        _CACHE[name] = (qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe)
    return _CACHE[name]


def local_codes(qg, nrows):
    """[nrows, M] localID - 1 from qg/ivt (rows without an entry: 0)."""
    lid = qg["local_ids"]
    out = np.zeros((nrows, qg["M"]), np.uint8)
    n = min(nrows, lid.shape[0])
    out[:n] = (lid[:n].astype(np.int32) - 1).clip(0, 15).astype(np.uint8)
    return out


def device_qg(name, build="device"):
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state(name)
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows, valid)
    ix.set_graph(offs, ids)
    ix.set_tree(tree)
    ix.set_search_property(int(prop["EdgeSizeForSearch"]), int(prop["DynamicEdgeSizeBase"]),
                           int(prop["DynamicEdgeSizeRate"]), int(prop["SeedSize"]), 0)
    ix.qg_set_quantizer(qg["global"], qg["local"][:, 1:17, :])
    if build == "device":
        ix.qg_build_graph(local_codes(qg, rows.shape[0]), maxe)
    else:
        ix.qg_set_graph(qg["qoff"], qg["qids"], qg["code_off"], qg["codes"])
    return ix


@pytest.mark.parametrize("name", sorted(CASES))
def test_qg_lut_bit_exact_vs_reference(name):
    qg, *_, z, meta, dim, maxe = state(name)
    ix = device_qg(name)
    qs = z["queries"].astype(np.float32)
    lut, sc, to = ix.qg_lut(qs)
    for qi in range(len(qs)):
        assert np.array_equal(lut[qi], z["lut"][qi]), qi
    assert np.array_equal(sc.view(np.uint32), z["scale"].astype(np.float32).view(np.uint32))
    assert np.array_equal(to.view(np.uint32), z["total_offset"].astype(np.float32).view(np.uint32))
    ix.close()


@pytest.mark.parametrize("build", ["device", "file"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_qg_adc_bit_exact_vs_reference(name, build):
    """Device-built quantized graph (construct) and the host-packed one
    (deserialize) both give the reference's ADC distances."""
    qg, *_, z, meta, dim, maxe = state(name)
    ix = device_qg(name, build)
    nodes = np.asarray(z["nodes"], np.uint32)
    nq = len(z["queries"])
    qidx = np.repeat(np.arange(nq, dtype=np.uint32), len(nodes))
    nn = np.tile(nodes, nq)
    out, n = ix.qg_adc(z["lut"], z["scale"], z["total_offset"], qidx, nn)
    for qi in range(nq):
        got = np.concatenate([out[qi * len(nodes) + j, :n[qi * len(nodes) + j]] for j in range(len(nodes))])
        assert np.array_equal(got.view(np.uint32), z["adc"][qi].view(np.uint32)), qi
    ix.close()


def _params(meta):
    for p in meta["params"]:
        k, eps, exp = p.split(":")
        yield p.replace(":", "_"), int(k), float(eps), float(exp)


@pytest.mark.parametrize("name", sorted(CASES))
def test_qg_search_matches_reference(name):
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state(name)
    ix = device_qg(name)
    qs = z["queries"].astype(np.float32)
    for key, k, eps, exp in _params(meta):
        gi, gd, gn, cnt = ix.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, seed_mode=SEED_TREE)
        for qi in range(len(qs)):
            n = int(z["n_" + key][qi])
            assert int(gn[qi]) == n, (key, qi)
            assert list(gi[qi, :n]) == list(z["ids_" + key][qi][:n]), (key, qi)
            assert np.array_equal(gd[qi, :n].view(np.uint32), z["dist_" + key][qi][:n].view(np.uint32)), (key, qi)
    ix.close()


@pytest.mark.parametrize("name", sorted(CASES))
def test_qg_search_counters_match_oracle(name):
    """Same traversal as the restatement: ADC count, accepted, expansions and
    exact distances agree query by query."""
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state(name)
    ix = device_qg(name)
    qs = z["queries"].astype(np.float32)
    for k, eps, exp in [(10, 0.05, 3.0), (10, 0.1, 0.5)]:
        gi, gd, gn, cnt = ix.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, seed_mode=SEED_TREE)
        for qi, q in enumerate(qs):
            qq = np.zeros(rows.shape[1], np.float32)
            qq[:len(q)] = q
            seeds, _, _ = O.tree_seeds("l2", tree, qq, k, int(prop["SeedSize"]))
            oid, od, ocnt = O.qg_search(qg, rows, qq, seeds, k, np.float32(eps), np.float32(exp))
            assert list(gi[qi, :gn[qi]]) == list(oid), (k, eps, exp, qi)
            assert np.array_equal(gd[qi, :gn[qi]].view(np.uint32), od.view(np.uint32))
            assert [int(x) for x in cnt[qi, :4]] == [int(x) for x in ocnt], (k, eps, exp, qi)
    ix.close()


@pytest.mark.parametrize("ht,cq", [("8", "64"), ("bitmap", "64"), ("9", "1024")])
def test_qg_overflow_paths_exact(monkeypatch, ht, cq):
    """Tiny LDS capacities force the visited hash -> HBM epochs and the
    unchecked array -> HBM spill; results must not change."""
    if ht != "bitmap":
        monkeypatch.setenv("NGT_AMD_HT_LOG2", ht)
    monkeypatch.setenv("NGT_AMD_CQ_CAP", cq)
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state("c1_qg")
    ix = device_qg("c1_qg")
    rng = np.random.default_rng(5)
    qs = z["queries"].astype(np.float32)
    seeds = [rng.choice(np.arange(1, rows.shape[0]), 10, replace=False).astype(np.uint32) for _ in qs]
    for eps, exp in [(0.3, 3.0), (0.6, 2.0)]:
        gi, gd, gn, cnt = ix.qg_search(qs, k=20, epsilon=eps, result_expansion=exp, seed_mode=SEED_GIVEN,
                                       seeds=seeds, visited_hash_log2=-1 if ht == "bitmap" else 0)
        for qi, q in enumerate(qs):
            oid, od, ocnt = O.qg_search(qg, rows, q, seeds[qi], 20, np.float32(eps), np.float32(exp))
            assert list(gi[qi, :gn[qi]]) == list(oid), (eps, qi)
            assert np.array_equal(gd[qi, :gn[qi]].view(np.uint32), od.view(np.uint32))
            assert [int(x) for x in cnt[qi, :4]] == [int(x) for x in ocnt]
    ix.close()


def test_qg_spill_trim_at_capacity(monkeypatch):
    """A full HBM spill first drops its keys beyond the exploration radius
    (they can never be popped) and flags 'spill capacity exceeded' only if
    that frees nothing.  The unchecked set's peak (counter 5) at
    the default capacity sizes the runs: below the peak spill some capacity
    must give the oracle's exact results only after trims (counter 7 > 0),
    i.e. where the untrimmed spill would have overflowed; smaller ones may
    still overflow, and must say so."""
    monkeypatch.setenv("NGT_AMD_CQ_CAP", "64")
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state("c1_qg")
    rng = np.random.default_rng(11)
    qs = z["queries"].astype(np.float32)
    seeds = [rng.choice(np.arange(1, rows.shape[0]), 10, replace=False).astype(np.uint32) for _ in qs]
    outcome = []
    # large result sets (k x expansion = 300): the radius stays unbounded until
    # 300 ids are accepted, so the keys spilled meanwhile are mostly beyond the
    # radius once it forms -- the keys a trim drops
    for k, eps, exp in [(30, 0.0, 10.0), (100, 0.05, 3.0), (60, 0.1, 5.0)]:
        ref = [O.qg_search(qg, rows, q, seeds[qi], k, np.float32(eps), np.float32(exp)) for qi, q in enumerate(qs)]
        monkeypatch.delenv("NGT_AMD_SPILL_CAP", raising=False)
        ix = device_qg("c1_qg")
        _, _, _, cnt = ix.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, seed_mode=SEED_GIVEN, seeds=seeds,
                                    visited_hash_log2=0)
        ix.close()
        peak_spill = int(cnt[:, 5].max()) - 64 - 64  # head and tail capacities
        for f in (0.9, 0.75, 0.6, 0.45, 0.3):
            cap = max(40, int(peak_spill * f))
            monkeypatch.setenv("NGT_AMD_SPILL_CAP", str(cap))
            ix = device_qg("c1_qg")
            try:
                gi, gd, gn, cnt = ix.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, seed_mode=SEED_GIVEN,
                                               seeds=seeds, visited_hash_log2=0)
            except NativeError as e:
                assert "spill capacity" in str(e), e
                outcome.append((k, eps, exp, peak_spill, cap, "overflow"))
                ix.close()
                continue
            ix.close()
            for qi in range(len(qs)):
                oid, od, ocnt = ref[qi]
                assert list(gi[qi, :gn[qi]]) == list(oid), (k, cap, qi)
                assert np.array_equal(gd[qi, :gn[qi]].view(np.uint32), od.view(np.uint32)), (k, cap, qi)
                assert [int(x) for x in cnt[qi, :4]] == [int(x) for x in ocnt], (k, cap, qi)
            outcome.append((k, eps, exp, peak_spill, cap, "exact", int(cnt[:, 7].sum())))
    print(outcome)
    assert any(o[5] == "exact" and o[6] > 0 for o in outcome), outcome


def test_qg_edge_cases():
    """Seeds-only searches, result_expansion < 1 (ADC distances returned),
    a tiny radius and k beyond the reachable set pad like the reference."""
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state("d20_qg")
    ix = device_qg("d20_qg")
    qs = z["queries"].astype(np.float32)[:4]
    seeds = [np.array([1, 2, 3], np.uint32), np.array([], np.uint32), np.array([5], np.uint32),
             np.array([7, 8], np.uint32)]
    for k, eps, exp, rad in [(5, 0.1, 0.5, -1.0), (300, 0.02, 1.0, -1.0), (10, 0.1, 3.0, 0.05),
                             (7, 0.0, 1.5, -1.0)]:
        gi, gd, gn, cnt = ix.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, radius=rad,
                                       seed_mode=SEED_GIVEN, seeds=seeds)
        for qi, q in enumerate(qs):
            r = np.float32(3.402823466e38) if rad < 0 else np.float32(rad)
            oid, od, ocnt = O.qg_search(qg, rows, q, seeds[qi], k, np.float32(eps), np.float32(exp), radius=r)
            assert int(gn[qi]) == len(oid), (k, eps, exp, rad, qi)
            assert list(gi[qi, :gn[qi]]) == list(oid), (k, eps, exp, rad, qi)
            assert np.array_equal(gd[qi, :gn[qi]].view(np.uint32), od.view(np.uint32))
    ix.close()


@pytest.mark.parametrize("with_grp", [False, True])
def test_ngtqg_capi_matches_reference(tmp_path, with_grp):
    """The drop-in ngtqg_open_index / ngtqg_search_index path (NGTQ/Capi.cpp:52-115)
    on the C1 ONNG + its reference-quantized qg/ directory, with the quantized
    graph constructed on open (no qg/grp) or read from a saved qg/grp."""
    import shutil
    from ngt_amd.qg import QuantizedIndex
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state("c1_qg")
    d = tmp_path / "idx"
    d.mkdir()
    for f in ["prf", "obj", "grp", "tre"]:
        os.symlink(os.path.join(GOLD, "c1_onng", f), str(d / f))
    shutil.copytree(os.path.join(GOLD, "c1_qg", "qg"), str(d / "qg"))
    if with_grp:
        with open(str(d / "qg" / "grp"), "wb") as f:
            f.write(F.serialize_qg_grp(qg))
    ix = QuantizedIndex(str(d))
    qs = z["queries"].astype(np.float32)
    for key, k, eps, exp in _params(meta):
        for qi in range(0, len(qs), 7):
            r = ix.search(qs[qi], size=k, epsilon=eps, result_expansion=exp)
            n = int(z["n_" + key][qi])
            assert [i for i, _ in r] == [int(x) - 1 for x in z["ids_" + key][qi][:n]], (key, qi)
            assert np.array_equal(np.array([dd for _, dd in r], np.float32).view(np.uint32),
                                  z["dist_" + key][qi][:n].view(np.uint32)), (key, qi)
        bi, bd, bn = ix.batch_search(qs, size=k, epsilon=eps, result_expansion=exp)
        for qi in range(len(qs)):
            n = int(z["n_" + key][qi])
            assert int(bn[qi]) == n and list(bi[qi, :n]) == list(z["ids_" + key][qi][:n]), (key, qi)
    ix.close()


# ---------------------------------------------------------------------------
# encoder and codebook training (ngt_amd_qg_encode / ngt_amd_qg_train)
# ---------------------------------------------------------------------------
def _l2_sub(r, c):
    """compareL2 of zero-padded subvectors (dsub <= 16), as l2_sub in
    qg_kernels.hip: 16 float lanes, 16->8->4 fold, sqrt in double."""
    diff = (r - c).astype(np.float32)
    v = np.zeros(diff.shape[:-1] + (16,), np.float32)
    v[..., :diff.shape[-1]] = diff
    acc = (v * v).astype(np.float32)
    t4 = (acc[..., 12:16] + acc[..., 4:8]) + (acc[..., 8:12] + acc[..., 0:4])
    s = (t4[..., 0] + t4[..., 1]) + (t4[..., 2] + t4[..., 3])
    return np.sqrt(s.astype(np.float64)).astype(np.float32)


@pytest.mark.parametrize("name", sorted(CASES))
def test_qg_encoder_matches_reference_ivt(name):
    """Every object of the reference-quantized index coded with the
    reference's own codebooks: the device encoder's local ids equal qg/ivt's
    (the reference's insertion search over each 16-centroid codebook index)."""
    qg, rows, valid, *_ = state(name)
    ix = device_qg(name)
    codes = ix.qg_encode()
    ref = local_codes(qg, rows.shape[0])
    have = np.zeros(rows.shape[0], bool)
    have[:min(rows.shape[0], qg["local_ids"].shape[0])] = qg["local_ids"][:rows.shape[0]].min(1) > 0
    have[0] = False
    bad = np.argwhere((codes != ref) & have[:, None])
    assert have.sum() > 0.9 * (rows.shape[0] - 1)
    assert len(bad) == 0, ("mismatches", len(bad), bad[:5].tolist())
    # the codes kept in HBM build the same quantized graph as the ivt codes
    ids_ref, codes_ref = ix.qg_get_graph()
    ix.qg_build_graph(None, CASES[name][2])
    ids_enc, codes_enc = ix.qg_get_graph()
    assert np.array_equal(ids_ref, ids_enc) and np.array_equal(codes_ref, codes_enc)
    ix.close()


def test_qg_train_fixpoint_and_search():
    """Trained codebooks (global = 0, dsub = 1, 1600 samples): every subspace
    that converged is a Lloyd fixpoint -- each centroid is the float mean, in
    sample order, of the samples nearest to it -- and the quantized graph built
    from the device-encoded codes finds the exact neighbours at recall >= 0.9
    (C1 data, k=10, expansion 3)."""
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state("c1_qg")
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows, valid)
    ix.set_graph(offs, ids)
    ix.set_tree(tree)
    ix.set_search_property(int(prop["EdgeSizeForSearch"]), int(prop["DynamicEdgeSizeBase"]),
                           int(prop["DynamicEdgeSizeRate"]), int(prop["SeedSize"]), 0)
    loc, its = ix.qg_train(dim, nsample=1600, max_iter=20)
    assert loc.shape == (dim, 16, 1) and its.max() <= 20
    s = rows[1:1601, :dim].astype(np.float32)
    checked = 0
    for m in range(dim):
        if its[m] >= 20:
            continue
        c = loc[m]                                             # [16, 1]
        d = _l2_sub(s[:, m:m + 1][:, None, :], c[None, :, :])  # [1600, 16]
        a = d.argmin(1)                                        # ties -> lower id
        cnt = np.bincount(a, minlength=16)
        if cnt.min() == 0:
            continue
        for ci in range(16):
            mem = s[a == ci, m]
            mean = np.float32(np.cumsum(mem, dtype=np.float32)[-1]) / np.float32(len(mem))
            assert np.float32(mean).view(np.uint32) == np.float32(c[ci, 0]).view(np.uint32), (m, ci)
        checked += 1
    assert checked > dim // 2
    codes = ix.qg_encode()
    assert codes.max() <= 15
    d = _l2_sub(rows[1:, :dim, None, None], loc[None, :, :, :])  # [n, dim, 16]
    assert np.array_equal(codes[1:], d.argmin(2).astype(np.uint8))
    ix.qg_build_graph(None, maxe)
    qs = queries_c1()[:100]
    gi, gd, gn, _ = ix.qg_search(qs, k=10, epsilon=0.1, result_expansion=3.0, seed_mode=SEED_TREE)
    li, ld, ln = ix.linear_search(qs, k=10)
    rec = np.mean([len(set(gi[i, :10]) & set(li[i, :ln[i]])) / 10.0 for i in range(len(qs))])
    assert rec >= 0.9, rec
    ix.close()


def queries_c1():
    return np.load(os.path.join(GOLD, "queries.npy")).astype(np.float32)


def test_ngtqg_quantize_capi(tmp_path):
    """ngtqg_quantize on the C1 ONNG: the qg/ directory is written in the
    reference's formats -- qg/prf and qg/global/prf byte-identical to the
    reference's, every codebook a complete NGT index (prf/obj/grp/tre), qg/ivt
    holding the device encoder's codes for the codebooks written, qg/grp the
    quantized graph built from them -- ngtqg_open_index reads it back, search
    reaches recall >= 0.9, and a second call leaves it alone."""
    import hashlib
    from ngt_amd.qg import QuantizedIndex, quantize
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state("c1_qg")
    d = tmp_path / "idx"
    d.mkdir()
    for f in ["prf", "obj", "grp", "tre"]:
        os.symlink(os.path.join(GOLD, "c1_onng", f), str(d / f))
    quantize(str(d), 0, 128)
    q = str(d / "qg")
    for f in ["prf", os.path.join("global", "prf")]:
        assert open(os.path.join(q, f), "rb").read() == open(os.path.join(GOLD, "c1_qg", "qg", f), "rb").read(), f
    for sub in ["global", "local-0", "local-127"]:
        assert sorted(os.listdir(os.path.join(q, sub))) == ["grp", "obj", "prf", "tre"], sub
    mine = F.read_qg(str(d), offs, ids, 128)
    # the codebooks: kmeansWithNGT restated over device searches, equal to the
    # reference's own quantize run with one OpenMP thread (make_kmeans_goldens.py)
    st = np.load(os.path.join(GOLD, "qg_kmeans_st.npz"))["c1"]
    assert np.array_equal(mine["local"][:, 1:17, 0].view(np.uint32), st.view(np.uint32))
    # with those codebooks, qg/ivt and qg/grp are the single-thread reference's bytes
    sha = {f: hashlib.sha256(open(os.path.join(q, f), "rb").read()).hexdigest() for f in ("ivt", "grp")}
    print("ngtqg_quantize sha256", sha)
    assert sha["ivt"] == "f4a5c511c370ed63c8f626db456c181558e43b2754ae10e8ebc79c865a97b0db"
    assert sha["grp"] == "45bfcbbe1adc1bda34a1430d545751e538db6b7e0f838afdfe6e594a5e8ef527"
    # the codes in ivt are the encoder's for the written codebooks
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows, valid)
    ix.qg_set_quantizer(mine["global"], mine["local"][:, 1:17, :])
    codes = ix.qg_encode()
    assert np.array_equal(codes[1:], (mine["local_ids"][1:rows.shape[0]].astype(np.int32) - 1).astype(np.uint8))
    ix.close()
    # qg/grp: the quantized graph of those codes (same bytes as read_qg constructs)
    raw = open(os.path.join(q, "grp"), "rb").read()
    assert raw == F.serialize_qg_grp(mine)
    h0 = hashlib.sha256(open(os.path.join(q, "ivt"), "rb").read()).hexdigest()
    quantize(str(d), 0, 128)  # exists: nothing happens
    assert hashlib.sha256(open(os.path.join(q, "ivt"), "rb").read()).hexdigest() == h0
    qi = QuantizedIndex(str(d))
    qs = queries_c1()[:100]
    bi, bd, bn = qi.batch_search(qs, size=10, epsilon=0.1, result_expansion=3.0)
    lx = DeviceIndex("l2", "float", dim)
    lx.set_objects(rows, valid)
    li, ld, ln = lx.linear_search(qs, k=10)
    lx.close()
    rec = np.mean([len(set(bi[i, :bn[i]].tolist()) & set(li[i, :ln[i]].tolist())) / 10.0 for i in range(len(qs))])
    assert rec >= 0.9, rec
    qi.close()


def _synthetic_qg(dim, n, maxe, seed, dups=(), degrees=None):
    """A QG index over n random rows of `dim` floats (dsub 1 => M = dim): a
    kNN graph, random codebooks and nearest-centroid codes, in both the
    oracle's form (read_qg's dict) and the device's.  dups: (dst, src) rows
    copied (equal codes, so equal ADC distances); degrees: per-node list
    lengths (0 = a node without edges), default maxe everywhere."""
    rng = np.random.default_rng(seed)
    dp = F.padded_dim(dim)
    rows = np.zeros((n + 1, dp), np.float32)
    rows[1:, :dim] = rng.random((n, dim), dtype=np.float32)
    for dst, src in dups:
        rows[dst] = rows[src]
    x = rows[1:, :dim].astype(np.float64)
    sq = (x * x).sum(1)
    d2 = sq[:, None] + sq[None, :] - 2.0 * x @ x.T
    np.fill_diagonal(d2, np.inf)
    nn = np.argsort(d2, axis=1, kind="stable")[:, :maxe] + 1
    deg = np.full(n, maxe, np.int64) if degrees is None else np.asarray(degrees, np.int64)
    offs = np.zeros(n + 2, np.uint64)
    offs[2:] = np.cumsum(deg.astype(np.uint64))
    ids = np.concatenate([nn[i, :deg[i]] for i in range(n)]).astype(np.uint32)
    M = dim
    local = np.zeros((M, 17, 1), np.float32)
    local[:, 1:, 0] = rng.random((M, 16), dtype=np.float32)
    codes = np.abs(rows[:, :dim, None] - local[None, :, 1:, 0]).argmin(2).astype(np.uint8)  # [n+1, M]
    me = (M + 1) // 2 * 2
    qoff = np.zeros(n + 2, np.uint64)
    code_off = np.zeros(n + 2, np.uint64)
    blobs = []
    for v in range(n + 1):
        e = ids[int(offs[v]):int(offs[v + 1])]
        qoff[v + 1] = qoff[v] + len(e)
        if len(e) == 0:
            code_off[v + 1] = code_off[v]
            continue
        nb = (len(e) - 1) // 16 + 1
        lc = np.zeros((nb * 16, M), np.uint8)
        lc[:len(e)] = codes[e]
        st = np.zeros((nb, me, 16), np.uint8)
        st[:, :M, :] = lc.reshape(nb, 16, M).transpose(0, 2, 1)
        st = st.reshape(-1)
        c = (st[0::2] | (st[1::2] << 4)).astype(np.uint8).tobytes()
        blobs.append(c)
        code_off[v + 1] = code_off[v] + len(c)
    qg = {"dim": dim, "M": M, "dsub": 1, "global": np.zeros(dp, np.float32), "local": local,
          "qoff": qoff, "qids": ids, "code_off": code_off, "codes": np.frombuffer(b"".join(blobs), np.uint8).copy()}
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows, np.r_[0, np.ones(n, np.uint8)].astype(np.uint8))
    ix.set_graph(offs, ids)
    ix.qg_set_quantizer(np.zeros(dim, np.float32), local[:, 1:17, :])
    ix.qg_build_graph(codes, maxe)
    return qg, rows, ix


@pytest.mark.parametrize("dim", [129, 256, 512])
def test_qg_wide_subspace_counts_exact(dim):
    """Subspace counts past one pair per lane (M = 129: a padded odd subspace
    and idle lanes; 256: two pairs per lane; 512: four) give the oracle's ids,
    float distance bits and work counters -- the i8 matrix-core sum of the ADC
    (table bytes stored as v - 128) is exact for every lane layout."""
    qg, rows, ix = _synthetic_qg(dim, 1200, 40, 7 + dim)
    rng = np.random.default_rng(dim)
    qs = rng.random((6, dim), dtype=np.float32)
    seeds = [np.array([1 + 37 * i, 600 + i], np.uint32) for i in range(len(qs))]
    for k, eps, exp in [(10, 0.1, 3.0), (20, 0.05, 1.0)]:
        gi, gd, gn, cnt = ix.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, seed_mode=SEED_GIVEN,
                                       seeds=seeds)
        for qi, q in enumerate(qs):
            oid, od, ocnt = O.qg_search(qg, rows, q, seeds[qi], k, np.float32(eps), np.float32(exp))
            assert list(gi[qi, :gn[qi]]) == list(oid), (dim, k, qi)
            assert np.array_equal(gd[qi, :gn[qi]].view(np.uint32), od.view(np.uint32)), (dim, k, qi)
            assert [int(x) for x in cnt[qi, :4]] == [int(x) for x in ocnt], (dim, k, qi)
    ix.close()


def test_ngtqg_quantize_codebooks_dsub4(tmp_path):
    """ngtqg_quantize -Q 4 on the 20-d index: the 5 local codebooks (16
    centroids of 4 floats) equal the reference's single-thread quantize."""
    from ngt_amd.qg import quantize
    d = tmp_path / "d20"
    d.mkdir()
    for f in ["prf", "obj", "grp", "tre"]:
        os.symlink(os.path.join(GOLD, "d20_qg", f), str(d / f))
    quantize(str(d), 4, 64)
    st = np.load(os.path.join(GOLD, "qg_kmeans_st.npz"))["d20"]
    for m in range(5):
        rows, _ = F.read_obj(os.path.join(str(d), "qg", "local-%d" % m, "obj"), 4, np.float32)
        assert np.array_equal(rows[1:17, :4].view(np.uint32), st[m].view(np.uint32)), m


def test_qg_train_local_ngt_equals_reference_codebooks():
    """DeviceIndex.qg_train_ngt (ngt_amd_qg_train_local_ngt, the codebook
    training ngtqg_quantize runs, used by bench.py --mode qg) on the C1 objects:
    the reference's single-thread `ngtqg quantize` codebooks bit for bit."""
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state("c1_qg")
    ix = DeviceIndex("l2", "float", dim)
    ix.set_objects(rows, valid)
    local = ix.qg_train_ngt(rows, dsub=1)
    st = np.load(os.path.join(GOLD, "qg_kmeans_st.npz"))["c1"]
    assert np.array_equal(local[:, :, 0].view(np.uint32), st.view(np.uint32))
    ix.close()


@pytest.mark.parametrize("name", sorted(CASES))
def test_qg_packed_layout_equals_fixed(monkeypatch, name):
    """The packed search layout (per node ceil(deg/16) blocks + {id, key word}
    entries, keys carrying the key word; qg_api.cpp qg_pack) and the fixed
    slabs give the same ids, distance bits and work counters, including the
    code-block count; the records take sum(ceil(deg/16) * (8*Me + 128)) bytes
    rounded to their unit."""
    qg, rows, valid, offs, ids, tree, prop, z, meta, dim, maxe = state(name)
    ix = device_qg(name)
    rec = int(ix.L.ngt_amd_qg_record_bytes(ix.h))
    assert rec > 0
    deg = np.diff(qg["qoff"].astype(np.int64))[1:rows.shape[0]]
    nb = np.maximum(1, (deg + 15) // 16)
    me = (qg["M"] + 1) // 2 * 2
    per = nb * (8 * me + 128)
    assert rec >= int(per.sum()) and rec <= int(per.sum()) + 4096 * len(per)
    monkeypatch.setenv("NGT_AMD_QG_PACKED", "0")
    fx = device_qg(name)
    assert int(fx.L.ngt_amd_qg_record_bytes(fx.h)) == 0
    qs = z["queries"].astype(np.float32)
    for k, eps, exp in [(10, 0.05, 3.0), (20, 0.2, 2.0), (10, 0.1, 0.5)]:
        for vis in (-1, 0):
            a = ix.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, seed_mode=SEED_TREE, visited_hash_log2=vis)
            b = fx.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, seed_mode=SEED_TREE, visited_hash_log2=vis)
            assert np.array_equal(a[2], b[2])
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
            assert np.array_equal(a[3][:, :5], b[3][:, :5])
    ix.close()
    fx.close()


def test_qg_packed_layout_ties_and_isolated_nodes():
    """Duplicate rows (equal ADC distances, ordered by id) and nodes without
    edges (one empty block each) through the packed layout: the oracle's ids,
    distance bits and counters."""
    n = 900
    degrees = [(7 * i) % 41 for i in range(n)]  # 0..40 edges, some nodes none
    qg, rows, ix = _synthetic_qg(128, n, 40, 77, dups=[(6, 5), (7, 5), (300, 299)], degrees=degrees)
    assert int(ix.L.ngt_amd_qg_record_bytes(ix.h)) > 0
    rng = np.random.default_rng(9)
    qs = rng.random((8, 128), dtype=np.float32)
    qs[0] = rows[5, :128]
    seeds = [np.array([1 + 91 * i, 450 + i, 5], np.uint32) for i in range(len(qs))]
    for k, eps, exp in [(10, 0.1, 3.0), (20, 0.3, 2.0)]:
        gi, gd, gn, cnt = ix.qg_search(qs, k=k, epsilon=eps, result_expansion=exp, seed_mode=SEED_GIVEN,
                                       seeds=seeds)
        for qi, q in enumerate(qs):
            oid, od, ocnt = O.qg_search(qg, rows, q, seeds[qi], k, np.float32(eps), np.float32(exp))
            assert list(gi[qi, :gn[qi]]) == list(oid), (k, qi)
            assert np.array_equal(gd[qi, :gn[qi]].view(np.uint32), od.view(np.uint32)), (k, qi)
            assert [int(x) for x in cnt[qi, :4]] == [int(x) for x in ocnt], (k, qi)
    ix.close()
