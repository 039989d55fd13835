"""Readers for NGT 1.13.8 index files (test infrastructure).

These parse the reference's on-disk formats into numpy arrays so that the
golden-vector generator and the tests can inspect reference-built indexes:

* ``prf`` -- tab-separated PropertySet (lib/NGT/Common.h:573-666).
* ``obj`` -- Repository<Object>::serialize (lib/NGT/Common.h:1776-1793):
  ``size_t n`` then per slot ``'-'`` or ``'+'`` + ``dim * sizeof(T)`` bytes
  (BaseObject::serialize, lib/NGT/ObjectSpace.h:297-301).
* ``grp`` -- GraphRepository::serialize (lib/NGT/Graph.h:151-154): the node
  Repository (per slot ``'+'`` + ``uint32 n`` + ``n`` packed
  ``{uint32 id, float distance}``, lib/NGT/ObjectSpace.h:29, Common.h:706-712,
  1937-1990) followed by ``prevsize`` (vector<unsigned short>).
* ``tre`` -- DVPTree::serialize (lib/NGT/Tree.h:344-347): leaf Repository then
  internal-node Repository (lib/NGT/Node.h:90-99, 224-251, 451-480).

The product path has its own C++ loader (ngt_amd/csrc/index_io.cpp); this
module is only used by tests/ and the golden generator.
"""
import os
import struct

import numpy as np


def read_prf(path):
    prop = {}
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            k, _, v = line.partition("\t")
            prop[k] = v
    return prop


def padded_dim(dim):
    # ObjectSpace::getPaddedDimension (lib/NGT/ObjectSpace.h:249)
    return ((dim - 1) // 16 + 1) * 16


def read_obj(path, dim, dtype):
    """Returns (rows[n, padded_dim], valid[n]) with row 0 the dummy slot."""
    dtype = np.dtype(dtype)
    raw = open(path, "rb").read()
    n = struct.unpack_from("<Q", raw, 0)[0]
    dp = padded_dim(dim)
    rows = np.zeros((n, dp), dtype=dtype)
    valid = np.zeros(n, dtype=np.uint8)
    off = 8
    nbytes = dim * dtype.itemsize
    for i in range(n):
        t = raw[off:off + 1]
        off += 1
        if t == b"+":
            rows[i, :dim] = np.frombuffer(raw, dtype=dtype, count=dim, offset=off)
            valid[i] = 1
            off += nbytes
        elif t != b"-":
            raise ValueError("corrupt obj file at slot %d" % i)
    return rows, valid


def read_grp(path):
    """Returns (offsets[n+1] uint64, ids uint32, dists float32)."""
    raw = open(path, "rb").read()
    n = struct.unpack_from("<Q", raw, 0)[0]
    off = 8
    offsets = np.zeros(n + 1, dtype=np.uint64)
    chunks_i, chunks_d = [], []
    total = 0
    rec = np.dtype([("id", "<u4"), ("d", "<f4")])
    for i in range(n):
        t = raw[off:off + 1]
        off += 1
        if t == b"+":
            cnt = struct.unpack_from("<I", raw, off)[0]
            off += 4
            e = np.frombuffer(raw, dtype=rec, count=cnt, offset=off)
            off += 8 * cnt
            chunks_i.append(e["id"].copy())
            chunks_d.append(e["d"].copy())
            total += cnt
        elif t != b"-":
            raise ValueError("corrupt grp file at slot %d" % i)
        offsets[i + 1] = total
    ids = np.concatenate(chunks_i) if chunks_i else np.zeros(0, np.uint32)
    dists = np.concatenate(chunks_d) if chunks_d else np.zeros(0, np.float32)
    return offsets, ids, dists


def read_tre(path, dim, dtype):
    """Parses the DVP tree. Returns a dict with numpy arrays:

    leaves: leaf_off (n_leaf_slots+1), leaf_ids (object ids in leaf order),
            leaf_valid; internal: in_pivot [n_in, padded_dim], in_child
            [n_in, 5] (raw Node::ID), in_border [n_in, 4], in_valid; root raw id.
    """
    dtype = np.dtype(dtype)
    raw = open(path, "rb").read()
    dp = padded_dim(dim)
    nbytes = dim * dtype.itemsize
    off = 0
    nleaf = struct.unpack_from("<Q", raw, off)[0]
    off += 8
    leaf_off = np.zeros(nleaf + 1, dtype=np.uint64)
    leaf_ids = []
    leaf_valid = np.zeros(nleaf, dtype=np.uint8)
    total = 0
    for i in range(nleaf):
        t = raw[off:off + 1]
        off += 1
        if t == b"+":
            _id, parent = struct.unpack_from("<II", raw, off)
            off += 8
            cnt = struct.unpack_from("<H", raw, off)[0]
            off += 2
            for _ in range(cnt):
                oid, _d = struct.unpack_from("<If", raw, off)
                off += 8
                leaf_ids.append(oid)
            total += cnt
            if not (parent & 0x7FFFFFFF == 0 and cnt == 0):
                off += nbytes  # pivot object
            leaf_valid[i] = 1
        elif t != b"-":
            raise ValueError("corrupt tre file (leaf %d)" % i)
        leaf_off[i + 1] = total
    nin = struct.unpack_from("<Q", raw, off)[0]
    off += 8
    in_pivot = np.zeros((nin, dp), dtype=dtype)
    in_child = np.zeros((nin, 5), dtype=np.uint32)
    in_border = np.zeros((nin, 4), dtype=np.float32)
    in_valid = np.zeros(nin, dtype=np.uint8)
    for i in range(nin):
        t = raw[off:off + 1]
        off += 1
        if t == b"+":
            off += 8  # id, parent
            in_pivot[i, :dim] = np.frombuffer(raw, dtype=dtype, count=dim, offset=off)
            off += nbytes
            csize = struct.unpack_from("<Q", raw, off)[0]
            off += 8
            if csize != 5:
                raise ValueError("unexpected childrenSize %d" % csize)
            in_child[i] = np.frombuffer(raw, dtype="<u4", count=5, offset=off)
            off += 20
            in_border[i] = np.frombuffer(raw, dtype="<f4", count=4, offset=off)
            off += 16
            in_valid[i] = 1
        elif t != b"-":
            raise ValueError("corrupt tre file (internal %d)" % i)
    if off != len(raw):
        raise ValueError("trailing bytes in tre: %d" % (len(raw) - off))
    # DVPTree::getRootNode (lib/NGT/Tree.h:219-235): internal 1, else leaf 1.
    if nin > 1 and in_valid[1]:
        root = 1
    else:
        root = 0x80000001
    return dict(leaf_off=leaf_off, leaf_ids=np.array(leaf_ids, dtype=np.uint32),
                leaf_valid=leaf_valid, in_pivot=in_pivot, in_child=in_child,
                in_border=in_border, in_valid=in_valid, root=root)


def parse_search_output(text):
    """Parses `ngt search -o e` output into a list of (ids, dists, ndist, nvisit)."""
    out = []
    cur = None
    for line in text.splitlines():
        if line.startswith("# Query No."):
            cur = {"ids": [], "dists": [], "ndist": 0, "nvisit": 0, "time_ms": 0.0}
        elif line.startswith("# Query Time (msec)="):
            cur["time_ms"] = float(line.split("=")[1])
        elif line.startswith("# Distance Computation="):
            cur["ndist"] = int(line.split("=")[1])
        elif line.startswith("# Visit Count="):
            cur["nvisit"] = int(line.split("=")[1])
        elif line.startswith("# End of Search"):
            out.append(cur)
        elif line and not line.startswith("#") and cur is not None:
            parts = line.split("\t")
            if len(parts) == 3:
                cur["ids"].append(int(parts[1]))
                cur["dists"].append(float(parts[2]))
    return out


# ---------------------------------------------------------------------------
# NGTQG quantizer state (index/qg/): prf, global/obj, local-*/obj, ivt, grp
# ---------------------------------------------------------------------------
def read_ivt(path):
    """qg/ivt: Repository<InvertedIndexEntry<uint16_t>> (NGTQ/Quantizer.h:105-132):
    u64 n, then per slot '+'/'-', u32 size, u16 numOfLocalIDs, size x
    {u32 id, u16 localID[nids] padded to 4 B}.  Returns {slot: (ids, localIDs)}."""
    raw = open(path, "rb").read()
    n = struct.unpack_from("<Q", raw, 0)[0]
    off = 8
    ents = {}
    for slot in range(n):
        t = raw[off:off + 1]
        off += 1
        if t == b"-":
            continue
        if t != b"+":
            raise ValueError("corrupt ivt at slot %d" % slot)
        sz, nids = struct.unpack_from("<IH", raw, off)
        off += 6
        es = 4 + ((nids * 2 - 1) // 4 + 1) * 4
        a = np.frombuffer(raw, np.uint8, sz * es, off).reshape(sz, es)
        off += sz * es
        ents[slot] = (a[:, :4].copy().view(np.uint32)[:, 0], a[:, 4:4 + 2 * nids].copy().view(np.uint16))
    if off != len(raw):
        raise ValueError("trailing bytes in ivt")
    return ents


def read_qg(index_dir, graph_offs, graph_ids, max_edges=128):
    """The quantizer state an NGTQG::Index opens (QuantizedGraph.h:170-185) and
    the quantized graph it constructs when qg/grp is absent (:64-115)."""
    qg = os.path.join(index_dir, "qg")
    p = read_prf(os.path.join(qg, "prf"))
    dim, M = int(p["Dimension"]), int(p["LocalDivisionNo"])
    dsub = dim // M
    g, _ = read_obj(os.path.join(qg, "global", "obj"), dim, np.float32)
    local = np.stack([read_obj(os.path.join(qg, "local-%d" % i, "obj"), dsub, np.float32)[0][:, :dsub]
                      for i in range(M)])
    ents = read_ivt(os.path.join(qg, "ivt"))
    last = max(int(ids.max()) for ids, _ in ents.values() if len(ids))
    lid = np.zeros((last + 1, M), np.uint16)
    for gid in sorted(ents):
        if gid == 0:
            continue
        ids, l = ents[gid]
        lid[ids] = l[:, :M]
    n = len(graph_offs) - 1
    me = (M + 1) // 2 * 2
    qoff = np.zeros(n + 1, np.uint64)
    code_off = np.zeros(n + 1, np.uint64)
    qids, blobs = [], []
    for v in range(n):
        e = np.asarray(graph_ids[graph_offs[v]:graph_offs[v + 1]][:max_edges], np.uint32)
        qids.append(e)
        qoff[v + 1] = qoff[v] + len(e)
        if len(e) == 0:
            blobs.append(b"")
            code_off[v + 1] = code_off[v]
            continue
        nb = (len(e) - 1) // 16 + 1
        # stream byte blk*16*Me + 16*m + (i % 16) = localID - 1 (Quantizer.h:1295-1303)
        lc = np.zeros((nb * 16, M), np.uint8)
        lc[:len(e)] = lid[e] - 1
        st = np.zeros((nb, me, 16), np.uint8)
        st[:, :M, :] = lc.reshape(nb, 16, M).transpose(0, 2, 1)
        st = st.reshape(-1)
        c = (st[0::2] | (st[1::2] << 4)).astype(np.uint8).tobytes()  # compressIntoUint4 (:1305-1327)
        blobs.append(c)
        code_off[v + 1] = code_off[v] + len(c)
    return {"dim": dim, "M": M, "dsub": dsub, "global": g[1].copy(), "local": local, "local_ids": lid,
            "qoff": qoff, "qids": np.concatenate(qids) if qids else np.zeros(0, np.uint32),
            "code_off": code_off, "codes": np.frombuffer(b"".join(blobs), np.uint8).copy()}


def serialize_qg_grp(q):
    """QuantizedGraphRepository::serialize (QuantizedGraph.h:117-128)."""
    n = len(q["qoff"]) - 1
    out = [struct.pack("<QQ", q["M"], n)]
    for v in range(n):
        a, b = int(q["qoff"][v]), int(q["qoff"][v + 1])
        out.append(struct.pack("<I", b - a) + q["qids"][a:b].astype(np.uint32).tobytes())
        out.append(q["codes"][int(q["code_off"][v]):int(q["code_off"][v + 1])].tobytes())
    return b"".join(out)


def read_array_file(path, dim, dtype=np.float32):
    """NGTQ object list (ArrayFile<NGT::Object>, lib/NGT/ArrayFile.h:35-46,
    136-145): {u64 recordSize, u64 reserve}, then per record a 16-byte
    {bool deleteFlag, u64 reserve} head and recordSize bytes of the object.
    Returns rows[n, dim] (record 0 is the unused slot)."""
    raw = open(path, "rb").read()
    rs = struct.unpack_from("<Q", raw, 0)[0]
    n = (len(raw) - 16) // (16 + rs)
    a = np.frombuffer(raw, np.uint8, n * (16 + rs), 16).reshape(n, 16 + rs)[:, 16:16 + dim * np.dtype(dtype).itemsize]
    return a.copy().view(dtype).reshape(n, dim)


def write_array_file(path, rows):
    """Inverse of read_array_file (record 0 written as all zeros)."""
    rows = np.ascontiguousarray(rows, dtype=np.float32)
    rs = rows.shape[1] * 4
    with open(path, "wb") as f:
        f.write(struct.pack("<QQ", rs, 0))
        for r in rows:
            f.write(b"\0" * 16)
            f.write(r.tobytes())
