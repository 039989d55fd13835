// ivf_api.cpp -- host side of the NGTQ IVF-ADC entry points of include/ngt_amd.h
// (ngt_amd_ngtq_*): the quantizer state of an NGTQ index in HBM and the
// search orchestration of NGTQ::QuantizerInstance::search
// (lib/NGT/NGTQ/Quantizer.h:2471-2549).
//
// HBM layout (attached to the index that holds the global codebook: its rows,
// graph and DVP tree are the global centroids and their ANNG):
//   local     [N][17][dsub]   local centroids per subspace (slot 0 unused;
//                             a single shared codebook is replicated)
//   list_off  [nlists+1]      inverted lists by global centroid id (CSR)
//   eids      [entries]       object ids in list order
//   elids     [entries][Np]   uint16 local ids (Np = N rounded up to even)
//   orows     [records][row]  the object list (ArrayFile "obj"), padded rows
// Every distance is computed on the device (graph/linear search kernels for
// the global codebook, ivf_kernels.hip for the aggregation); no CPU path.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <cfloat>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/ngt_amd.h"
#include "index_internal.h"
#include "index_io.h"
#include "ngt_kernels.h"

using namespace ngt_amd;

extern "C" int ngt_amd_ngtq_set(ngt_amd_index* ix, const float* local, uint32_t N, uint32_t dsub,
                                const uint64_t* list_off, uint64_t nlists, const uint32_t* eids,
                                const uint16_t* elids, uint64_t nentries, const float* objects,
                                uint64_t object_records) {
  if (!ix || !local || !list_off || N == 0 || dsub == 0 || nlists == 0 || (nentries && (!eids || !elids)) ||
      (object_records && !objects))
    return fail("ngt_amd_ngtq_set: bad arguments");
  if (ix->metric != NGT_AMD_DISTANCE_L2 || ix->otype != NGT_AMD_OBJECT_FLOAT)
    return fail("ngt_amd_ngtq_set: NGTQ needs an L2 float global codebook");
  if ((uint64_t)N * dsub != ix->dim)
    return fail("ngt_amd_ngtq_set: N (%u) x dsub (%u) != dimension (%u)", N, dsub, ix->dim);
  if ((uint64_t)N * 17 * 8 > 32 * 1024) return fail("ngt_amd_ngtq_set: %u subspaces exceed the LDS table", N);
  if (list_off[0] != 0 || list_off[nlists] != nentries) return fail("ngt_amd_ngtq_set: inconsistent list offsets");
  for (uint64_t g = 0; g < nlists; g++)
    if (list_off[g + 1] < list_off[g]) return fail("ngt_amd_ngtq_set: list offsets must be non-decreasing");
  const uint32_t np = (N + 1) / 2 * 2;
  for (uint64_t e = 0; e < nentries; e++) {
    if (eids[e] == 0 || eids[e] >= object_records)
      return fail("ngt_amd_ngtq_set: entry %llu names object %u outside the object list", (unsigned long long)e, eids[e]);
    for (uint32_t li = 0; li < N; li++)
      if (elids[e * N + li] > 16) return fail("ngt_amd_ngtq_set: local id %u > 16", elids[e * N + li]);
  }
  HIP_OK(hipSetDevice(ix->device));
  IvfState& v = ix->ivf;
  std::vector<float> loc((size_t)N * 17 * dsub, 0.0f);
  for (uint32_t li = 0; li < N; li++)
    memcpy(&loc[((size_t)li * 17 + 1) * dsub], local + (size_t)li * 16 * dsub, (size_t)16 * dsub * sizeof(float));
  std::vector<uint16_t> lids((size_t)std::max<uint64_t>(nentries, 1) * np, 0);
  for (uint64_t e = 0; e < nentries; e++) memcpy(&lids[e * np], elids + e * N, (size_t)N * sizeof(uint16_t));
  std::vector<uint8_t> rows((size_t)std::max<uint64_t>(object_records, 1) * ix->row_bytes, 0);
  for (uint64_t r = 0; r < object_records; r++)
    memcpy(&rows[r * ix->row_bytes], objects + r * ix->dim, (size_t)ix->dim * sizeof(float));
  HIP_OK(v.local.upload(loc.data(), loc.size()));
  HIP_OK(v.list_off.upload(list_off, nlists + 1));
  HIP_OK(v.eids.upload(eids, std::max<uint64_t>(nentries, 1)));
  HIP_OK(v.elids.upload(lids.data(), lids.size()));
  HIP_OK(v.orows.upload(rows.data(), rows.size()));
  v.N = N;
  v.dsub = dsub;
  v.lid_stride = np;
  v.nlists = nlists;
  v.nentries = nentries;
  v.object_records = object_records;
  v.ready = true;
  return 0;
}

extern "C" int ngt_amd_ngtq_search_device(ngt_amd_index* ix, const ngt_amd_ngtq_search_params* prm,
                                          const void* d_queries, uint64_t query_bytes, uint32_t nq, uint32_t* d_ids,
                                          float* d_dists, uint32_t* d_n, void* stream) {
  if (!ix || !prm || (!d_queries && nq)) return fail("ngt_amd_ngtq_search_device: bad arguments");
  if (!ix->ivf.ready) return fail("ngt_amd_ngtq_search: the index has no NGTQ quantizer");
  if (nq && query_bytes < ix->row_bytes)
    return fail("ngt_amd_ngtq_search_device: query stride %llu < %llu bytes", (unsigned long long)query_bytes,
                (unsigned long long)ix->row_bytes);
  if (prm->size == 0) return fail("ngt_amd_ngtq_search: size must be > 0");
  int mode;
  switch (prm->mode) {
    case NGT_AMD_NGTQ_APPROXIMATE: mode = kIvfApprox; break;
    case NGT_AMD_NGTQ_LOOKUP_TABLE: mode = kIvfLut; break;
    case NGT_AMD_NGTQ_CACHE: mode = kIvfCache; break;
    case NGT_AMD_NGTQ_REFINE: mode = kIvfRefine; break;
    case NGT_AMD_NGTQ_EXACT: mode = kIvfExact; break;
    default: return fail("ngt_amd_ngtq_search: invalid aggregation mode %d", prm->mode);
  }
  IvfState& v = ix->ivf;
  if ((mode == kIvfCache || mode == kIvfRefine) && v.dsub % 8)
    return fail("ngt_amd_ngtq_search: the cached-distance modes read whole 8-float blocks; subvector dimension %u "
                "is not a multiple of 8", v.dsub);
  if (mode == kIvfRefine && prm->size > 256) return fail("ngt_amd_ngtq_search: refine mode supports size <= 256");
  if (nq == 0) return 0;
  // approximateSearchSize = size * expansion (size_t * float); codebookSearchSize
  // = approximateSearchSize / (objectList.size() / globalCodebook size) + 1
  // (Quantizer.h:2471-2479)
  const uint64_t ass = (uint64_t)((float)prm->size * prm->expansion);
  const uint64_t per = v.object_records / ix->nrows;
  if (per == 0) return fail("ngt_amd_ngtq_search: the object list is smaller than the global codebook");
  const uint64_t cbs64 = ass / per + 1;
  const uint64_t ncent = ix->nrows - 1;
  const uint32_t cbs = (uint32_t)std::min<uint64_t>(cbs64, std::max<uint64_t>(ncent, 1));
  if (cbs64 > 4096 && cbs64 <= ncent) return fail("ngt_amd_ngtq_search: codebook search size %llu too large",
                                                  (unsigned long long)cbs64);
  HIP_OK(hipSetDevice(ix->device));
  hipStream_t s = (hipStream_t)stream;
  SearchCtx* sc = ctx_for(ix, s);  // the centroid lists belong to this index and stream
  if (!sc) return -1;
  HIP_OK(sc->ivf_cid.alloc((size_t)nq * cbs));
  HIP_OK(sc->ivf_cd.alloc((size_t)nq * cbs));
  HIP_OK(sc->ivf_cn.alloc(nq));
  // searchGlobalCodebook (Quantizer.h:2248-2262): linear search when epsilon
  // is FLT_MAX, else the index's search (tree seeds + graph)
  const bool linear = prm->epsilon < 0.0f || prm->epsilon >= FLT_MAX;
  if (linear) {
    if (ngt_amd_linear_search_device(ix, d_queries, query_bytes, nq, cbs, (double)FLT_MAX, sc->ivf_cid.p, sc->ivf_cd.p,
                                     sc->ivf_cn.p, stream))
      return -1;
  } else {
    ngt_amd_search_params p{};
    p.k = cbs;
    p.epsilon = prm->epsilon;
    p.radius = FLT_MAX;
    p.edge_size = -1;
    p.seed_mode = ix->has_tree ? NGT_AMD_SEED_TREE : NGT_AMD_SEED_RANDOM;
    p.visited_hash_log2 = 0;
    if (ngt_amd_search_device(ix, &p, d_queries, query_bytes, nq, nullptr, nullptr, sc->ivf_cid.p, sc->ivf_cd.p, sc->ivf_cn.p,
                              nullptr, stream))
      return -1;
  }
  IvfSearchArgs a{};
  a.queries = static_cast<const uint8_t*>(d_queries);
  a.query_bytes = query_bytes;
  a.nq = nq;
  a.dp = (int)ix->dp;
  a.cent_ids = sc->ivf_cid.p;
  a.cent_d = sc->ivf_cd.p;
  a.cent_n = sc->ivf_cn.p;
  a.cent_stride = cbs;
  a.grows = ix->rows.p;
  a.grow_bytes = ix->row_bytes;
  a.local = v.local.p;
  a.N = v.N;
  a.dsub = v.dsub;
  a.lid_stride = v.lid_stride;
  a.list_off = v.list_off.p;
  a.nlists = (uint32_t)v.nlists;
  a.eids = v.eids.p;
  a.elids = v.elids.p;
  a.orows = v.orows.p;
  a.orow_bytes = ix->row_bytes;
  a.size = prm->size;
  a.ass = ass;
  a.mode = mode;
  a.out_ids = d_ids;
  a.out_dists = d_dists;
  a.out_n = d_n;
  if (ivf_search_lds_bytes(a) > 64 * 1024) return fail("ngt_amd_ngtq_search: size %u needs too much LDS", prm->size);
  HIP_OK(launch_ivf_search(a, s));
  return 0;
}

extern "C" int ngt_amd_ngtq_search(ngt_amd_index* ix, const ngt_amd_ngtq_search_params* prm, const float* queries,
                                   uint32_t nq, uint32_t* ids, float* dists, uint32_t* n) {
  if (!ix || !prm || (!queries && nq) || !ids || !dists || !n) return fail("ngt_amd_ngtq_search: bad arguments");
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(ix->device));
  CallGuard g(ix);
  CallCtx* cc = g.c;
  if (!cc) return -1;
  hipStream_t s = cc->stream;
  if (clear_device_error(ix, s)) return -1;
  if (upload_queries(ix, queries, nq, cc->raw, cc->prep, s)) return -1;
  HIP_OK(cc->ids.alloc((size_t)nq * prm->size));
  HIP_OK(cc->dists.alloc((size_t)nq * prm->size));
  HIP_OK(cc->n.alloc(nq));
  if (ngt_amd_ngtq_search_device(ix, prm, cc->prep.p, ix->row_bytes, nq, cc->ids.p, cc->dists.p, cc->n.p, s))
    return -1;
  HIP_OK(hipMemcpyAsync(ids, cc->ids.p, (size_t)nq * prm->size * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(dists, cc->dists.p, (size_t)nq * prm->size * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(n, cc->n.p, (size_t)nq * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  int flag = 0;
  if (take_device_error(ix, s, &flag)) return -1;
  if (flag) return fail("ngt_amd_ngtq_search: device error flag %d (%s)", flag, device_error_text(flag).c_str());
  return 0;
}

// ---------------------------------------------------------------------------
// Opening an NGTQ index directory (NGTQ::Index(path), Quantizer.h:1520-1570).
// ---------------------------------------------------------------------------
namespace {

struct Reader {
  std::ifstream f;
  bool ok = true;
  bool open(const std::string& p) {
    f.open(p, std::ios::binary);
    return (bool)f;
  }
  template <typename T>
  T get() {
    T v{};
    f.read(reinterpret_cast<char*>(&v), sizeof(T));
    if (!f) ok = false;
    return v;
  }
  void bytes(void* p, size_t n) {
    f.read(static_cast<char*>(p), (std::streamsize)n);
    if (!f) ok = false;
  }
};

// Repository<Object>::serialize of a local codebook (obj): slots 1..16 = centroids
std::string read_local(const std::string& path, uint32_t dsub, std::vector<float>& out16) {
  Reader r;
  if (!r.open(path)) return "cannot open " + path;
  const uint64_t n = r.get<uint64_t>();
  out16.assign((size_t)16 * dsub, 0.0f);
  std::vector<float> row(dsub);
  for (uint64_t i = 0; i < n && r.ok; i++) {
    const char t = r.get<char>();
    if (t == '-') continue;
    if (t != '+') return "corrupt " + path;
    r.bytes(row.data(), (size_t)dsub * 4);
    if (i >= 1 && i <= 16) memcpy(&out16[(i - 1) * dsub], row.data(), (size_t)dsub * 4);
  }
  if (!r.ok) return "truncated " + path;
  if (n < 2) return path + " holds no centroids";
  return "";
}

}  // namespace

extern "C" int ngt_amd_ngtq_open(const char* path, int device, ngt_amd_index** out) {
  if (!path || !out) return fail("ngt_amd_ngtq_open: bad arguments");
  *out = nullptr;
  const std::string dir = path;
  HostProperty qp;
  std::string e = read_prf(dir + "/prf", qp);
  if (!e.empty()) return fail("ngt_amd_ngtq_open: %s", e.c_str());
  auto geti = [&](const char* k, long dflt) {
    auto it = qp.kv.find(k);
    return it == qp.kv.end() ? dflt : atol(it->second.c_str());
  };
  const uint32_t dim = (uint32_t)geti("Dimension", 0);
  const uint32_t N = (uint32_t)geti("LocalDivisionNo", 0);
  const long dtype = geti("DataType", 1), dist = geti("DistanceType", 2), lidb = geti("LocalIDByteSize", 2);
  const bool single = geti("SingleLocalCodebook", 0) != 0;
  if (dim == 0 || N == 0 || dim % N) return fail("ngt_amd_ngtq_open: bad Dimension/LocalDivisionNo in %s/prf", path);
  if (dtype != 1) return fail("ngt_amd_ngtq_open: only float NGTQ indexes are supported (DataType %ld)", dtype);
  if (dist != 2) return fail("ngt_amd_ngtq_open: only L2 NGTQ indexes are supported (DistanceType %ld)", dist);
  if (lidb != 2) return fail("ngt_amd_ngtq_open: only 2-byte local ids are supported (LocalIDByteSize %ld)", lidb);
  const uint32_t dsub = dim / N;
  HostIndex g;
  e = load_index(dir + "/global", g);
  if (!e.empty()) return fail("ngt_amd_ngtq_open: %s", e.c_str());
  if (g.prop.dimension != (int32_t)dim || g.prop.object_type != 2 || g.prop.distance_type != 1)
    return fail("ngt_amd_ngtq_open: the global codebook is not a %u-d float L2 index", dim);
  // local codebooks
  std::vector<float> local((size_t)N * 16 * dsub);
  for (uint32_t li = 0; li < N; li++) {
    std::vector<float> c;
    e = read_local(dir + "/local-" + std::to_string(single ? 0 : li) + "/obj", dsub, c);
    if (!e.empty()) return fail("ngt_amd_ngtq_open: %s", e.c_str());
    memcpy(&local[(size_t)li * 16 * dsub], c.data(), c.size() * sizeof(float));
  }
  // ivt: Repository<InvertedIndexEntry<uint16_t>> (Quantizer.h:72-143)
  std::vector<uint64_t> list_off;
  std::vector<uint32_t> eids;
  std::vector<uint16_t> elids;
  {
    Reader r;
    if (!r.open(dir + "/ivt")) return fail("ngt_amd_ngtq_open: cannot open %s/ivt", path);
    const uint64_t n = r.get<uint64_t>();
    list_off.assign(n + 1, 0);
    std::vector<uint8_t> buf;
    for (uint64_t slot = 0; slot < n && r.ok; slot++) {
      const char t = r.get<char>();
      list_off[slot + 1] = list_off[slot];
      if (t == '-') continue;
      if (t != '+') return fail("ngt_amd_ngtq_open: corrupt ivt at slot %llu", (unsigned long long)slot);
      const uint32_t sz = r.get<uint32_t>();
      const uint16_t nids = r.get<uint16_t>();
      if (nids != N) return fail("ngt_amd_ngtq_open: ivt entries hold %u local ids, expected %u", nids, N);
      const size_t es = 4 + ((size_t)(nids * 2 - 1) / 4 + 1) * 4;
      buf.resize((size_t)sz * es);
      r.bytes(buf.data(), buf.size());
      for (uint32_t j = 0; j < sz; j++) {
        uint32_t id;
        memcpy(&id, &buf[j * es], 4);
        eids.push_back(id);
        const size_t b = elids.size();
        elids.resize(b + N);
        memcpy(&elids[b], &buf[j * es + 4], (size_t)N * 2);
      }
      list_off[slot + 1] = eids.size();
    }
    if (!r.ok) return fail("ngt_amd_ngtq_open: truncated ivt");
  }
  // object list: ArrayFile<NGT::Object> (lib/NGT/ArrayFile.h:35-46, 136-145)
  std::vector<float> objects;
  uint64_t records = 0;
  {
    Reader r;
    if (!r.open(dir + "/obj")) return fail("ngt_amd_ngtq_open: cannot open %s/obj", path);
    r.f.seekg(0, std::ios::end);
    const uint64_t fsz = (uint64_t)r.f.tellg();
    r.f.seekg(0);
    const uint64_t rs = r.get<uint64_t>();
    (void)r.get<uint64_t>();
    if (rs < (uint64_t)dim * 4) return fail("ngt_amd_ngtq_open: object records of %llu bytes < %u floats",
                                            (unsigned long long)rs, dim);
    records = (fsz - 16) / (16 + rs);
    objects.assign((size_t)records * dim, 0.0f);
    std::vector<uint8_t> rec(16 + rs);
    for (uint64_t i = 0; i < records && r.ok; i++) {
      r.bytes(rec.data(), rec.size());
      memcpy(&objects[(size_t)i * dim], &rec[16], (size_t)dim * 4);
    }
    if (!r.ok) return fail("ngt_amd_ngtq_open: truncated object list");
  }
  ngt_amd_index* ix = nullptr;
  if (ngt_amd_index_create(&ix, device, NGT_AMD_DISTANCE_L2, NGT_AMD_OBJECT_FLOAT, dim)) return -1;
  auto bail = [&]() {
    ngt_amd_index_destroy(ix);
    return -1;
  };
  if (ngt_amd_index_set_objects(ix, g.rows.data(), g.nrows, g.valid.data())) return bail();
  if (g.edge_off.size() == g.nrows + 1 && !g.edges.empty() &&
      ngt_amd_index_set_graph(ix, g.edge_off.data(), g.edges.data(), g.edges.size()))
    return bail();
  if (g.tree.present && g.prop.index_type == 0) {
    const HostTree& t = g.tree;
    if (ngt_amd_index_set_tree(ix, t.in_pivot.data(), t.n_internal(), t.in_child.data(), t.in_border.data(), 5, t.root,
                               t.leaf_off.data(), t.n_leaf(), t.leaf_ids.data(), t.leaf_ids.size()))
      return bail();
  }
  ngt_amd_index_set_search_property(ix, g.prop.edge_size_for_search, g.prop.dynamic_edge_size_base,
                                    g.prop.dynamic_edge_size_rate, g.prop.seed_size, g.prop.seed_type);
  const uint64_t nlists = std::min<uint64_t>(list_off.size() - 1, g.nrows);
  list_off.resize(nlists + 1);
  const uint64_t ne = list_off[nlists];
  eids.resize(ne);
  elids.resize((size_t)ne * N);
  if (ngt_amd_ngtq_set(ix, local.data(), N, dsub, list_off.data(), nlists, eids.data(), elids.data(), ne,
                       objects.data(), records))
    return bail();
  *out = ix;
  return 0;
}
