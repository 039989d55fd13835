// qg_capi.cpp -- the reference's `ngtqg_*` C API (lib/NGT/NGTQ/Capi.cpp:40-131)
// on the MI355X path.  An NGTQGIndex is the NGT index (prf/obj/grp/tre) plus
// its <index>/qg quantizer, loaded straight into HBM: exact rows, graph and
// DVP tree through ngt_amd_index_*, codebooks and the quantized graph through
// ngt_amd_qg_* (constructed on the device from qg/ivt unless qg/grp was
// saved, as NGTQG::Index's constructor does, QuantizedGraph.h:170-185).
// Search = NGTQG::Index::search(SearchQuery&) (:354-372) as one device batch.
#include <float.h>
#include <stdlib.h>
#include <sys/stat.h>

#include <algorithm>
#include <fstream>

#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/NGT/Capi.h"
#include "../../include/NGT/NGTQ/Capi.h"
#include "../../include/ngt_amd.h"
#include "coalesce.h"
#include "index_internal.h"
#include "index_io.h"
#include "kmeans_ngt.h"

namespace {

struct QgCapiIndex {
  ngt_amd::HostIndex host;
  ngt_amd::HostQuantizer quant;
  ngt_amd_index* dev = nullptr;
  std::unique_ptr<ngt_amd::Coalescer> co;  // concurrent ngtqg_search_index callers
  ~QgCapiIndex() {
    if (dev) ngt_amd_index_destroy(dev);
  }
};

typedef std::vector<NGTObjectDistance> Results;  // NGTObjectDistances of capi.cpp

void report(NGTError error, const std::string& msg) {
  if (error != NULL) *static_cast<std::string*>(error) = msg;
  else std::cerr << msg << std::endl;
}

std::string amd_err() { return std::string(ngt_amd_last_error()); }

std::string open_device(QgCapiIndex* ix, uint32_t max_edges) {
  using ngt_amd::HostIndex;
  HostIndex& h = ix->host;
  if (h.prop.distance_type != NGT_AMD_DISTANCE_L2 || h.prop.object_type != NGT_AMD_OBJECT_FLOAT)
    return "NGTQG supports L2 float indexes only";
  int dev = 0;
  if (const char* env = getenv("NGT_AMD_DEVICE")) dev = atoi(env);
  if (ngt_amd_index_create(&ix->dev, dev, h.prop.distance_type, h.prop.object_type, (uint32_t)h.prop.dimension))
    return amd_err();
  if (ngt_amd_index_set_objects(ix->dev, h.rows.data(), h.nrows, h.valid.data())) return amd_err();
  if (ngt_amd_index_set_graph(ix->dev, h.edge_off.data(), h.edges.data(), h.edges.size())) return amd_err();
  if (h.tree.present) {
    const ngt_amd::HostTree& t = h.tree;
    if (ngt_amd_index_set_tree(ix->dev, t.in_pivot.data(), t.n_internal(), t.in_child.data(), t.in_border.data(), 5,
                               t.root, t.leaf_off.data(), t.n_leaf(), t.leaf_ids.data(), t.leaf_ids.size()))
      return amd_err();
  }
  ngt_amd_index_set_search_property(ix->dev, h.prop.edge_size_for_search, h.prop.dynamic_edge_size_base,
                                    h.prop.dynamic_edge_size_rate, h.prop.seed_size, h.prop.seed_type);
  const ngt_amd::HostQuantizer& q = ix->quant;
  if (ngt_amd_qg_set_quantizer(ix->dev, q.global.data(), q.local.data(), q.M, q.dsub)) return amd_err();
  if (q.has_grp) {
    if (q.qoff.size() != h.nrows + 1) return "qg/grp node count differs from the graph";
    if (ngt_amd_qg_set_graph(ix->dev, q.qoff.data(), q.qids.data(), q.code_off.data(), q.qcodes.data()))
      return amd_err();
  } else {
    // QuantizedGraphRepository::construct with maxNoOfEdges (default 128, QuantizedGraph.h:170)
    if (ngt_amd_qg_build_graph(ix->dev, q.codes.data(), max_edges)) return amd_err();
  }
  return "";
}

// One device batch of queries; per query up to `size` results.
std::string run(QgCapiIndex* ix, const float* queries, uint32_t nq, size_t size, float epsilon, float expansion,
                float radius, std::vector<uint32_t>& ids, std::vector<float>& dists, std::vector<uint32_t>& n) {
  n.assign(nq, 0);
  if (size == 0 || nq == 0) return "";  // sc.size == 0 returns nothing (QuantizedGraph.h:331-334)
  ngt_amd_qg_search_params p{};
  p.k = (uint32_t)size;
  p.epsilon = epsilon;
  p.result_expansion = expansion;
  p.radius = radius < 0.0f ? FLT_MAX : radius;
  p.seed_mode = ix->host.tree.present ? NGT_AMD_SEED_TREE : NGT_AMD_SEED_RANDOM;
  ids.resize((size_t)nq * size);
  dists.resize((size_t)nq * size);
  if (ngt_amd_qg_search(ix->dev, &p, queries, nq, nullptr, nullptr, ids.data(), dists.data(), n.data(), nullptr))
    return amd_err();
  return "";
}

// One NGT index (a codebook) of `n` float rows of `d` dimensions: created,
// built and saved through this library's ngt_* API (obj/prf/grp/tre).
std::string write_codebook(const std::string& dir, const float* rows, uint32_t n, uint32_t d, int edge_create,
                           int edge_search) {
  NGTError er = ngt_create_error_object();
  NGTProperty prop = ngt_create_property(er);
  std::string e;
  NGTIndex cb = NULL;
  if (!ngt_set_property_dimension(prop, (int32_t)d, er) || !ngt_set_property_object_type_float(prop, er) ||
      !ngt_set_property_distance_type_l2(prop, er) ||
      !ngt_set_property_edge_size_for_creation(prop, (int16_t)edge_create, er) ||
      !ngt_set_property_edge_size_for_search(prop, (int16_t)edge_search, er))
    e = ngt_get_error_string(er);
  if (e.empty() && !(cb = ngt_create_graph_and_tree(dir.c_str(), prop, er))) e = ngt_get_error_string(er);
  for (uint32_t i = 0; e.empty() && i < n; i++)
    if (ngt_insert_index_as_float(cb, const_cast<float*>(rows + (size_t)i * d), d, er) == 0)
      e = ngt_get_error_string(er);
  if (e.empty() && !ngt_create_index(cb, 16, er)) e = ngt_get_error_string(er);
  if (e.empty() && !ngt_save_index(cb, dir.c_str(), er)) e = ngt_get_error_string(er);
  if (cb) ngt_close_index(cb);
  ngt_destroy_property(prop);
  ngt_destroy_error_object(er);
  return e;
}

std::string write_quantizer(const std::string& qd, const ngt_amd::HostIndex& h, uint32_t dim, uint32_t M,
                            uint32_t dsub, const std::vector<float>& local, const std::vector<uint8_t>& codes,
                            uint32_t stride, uint64_t cstride, const std::vector<uint32_t>& qids,
                            const std::vector<uint8_t>& qcodes) {
  if (mkdir(qd.c_str(), 0755) != 0) return "cannot create " + qd;
  {
    // NGTQ::Property::save (lib/NGT/NGTQ/Quantizer.h:218-240), the frame of
    // constructQuantizedGraphFrame (QuantizedGraph.h:423-454)
    std::ofstream f(qd + "/prf");
    f << "BatchSize\t1000\nCentroidCreationMode\t1\nDataSize\t" << (uint64_t)dim * 4 << "\nDataType\t1\n"
      << "Dimension\t" << dim << "\nDistanceType\t2\nGlobalCentroidLimit\t1\nGlobalRange\t0\n"
      << "LocalCentroidCreationMode\t2\nLocalCentroidLimit\t16\nLocalCodebookState\t1\n"
      << "LocalDivisionNo\t" << M << "\nLocalIDByteSize\t2\nLocalRange\t0\nLocalSampleCoefficient\t100\n"
      << "SingleLocalCodebook\t0\nThreadSize\t24\n";
    if (!f) return "cannot write " + qd + "/prf";
  }
  // global codebook: the zero vector (QuantizedGraph.h:397-399), edge sizes 10 / 40
  std::vector<float> zero(dim, 0.0f);
  std::string e = write_codebook(qd + "/global", zero.data(), 1, dim, 10, 40);
  if (!e.empty()) return e;
  for (uint32_t m = 0; m < M && e.empty(); m++)
    e = write_codebook(qd + "/local-" + std::to_string(m), local.data() + (size_t)m * 16 * dsub, 16, dsub, 10, 40);
  if (!e.empty()) return e;
  {
    // ivt: every valid object under global centroid 1, local ids 1..16 padded to 4 B
    std::ofstream f(qd + "/ivt", std::ios::binary);
    const uint64_t n = 2;
    f.write(reinterpret_cast<const char*>(&n), 8);
    f.put('-');
    f.put('+');
    uint32_t cnt = 0;
    for (uint64_t i = 1; i < h.nrows; i++) cnt += h.valid[i] ? 1 : 0;
    const uint16_t nids = (uint16_t)M;
    f.write(reinterpret_cast<const char*>(&cnt), 4);
    f.write(reinterpret_cast<const char*>(&nids), 2);
    const size_t pad = ((size_t)(nids * 2 - 1) / 4 + 1) * 4;
    std::vector<uint16_t> lid(pad / 2, 0);
    for (uint64_t i = 1; i < h.nrows; i++) {
      if (!h.valid[i]) continue;
      const uint32_t id = (uint32_t)i;
      for (uint32_t m = 0; m < M; m++) lid[m] = (uint16_t)(codes[i * M + m] + 1);
      f.write(reinterpret_cast<const char*>(&id), 4);
      f.write(reinterpret_cast<const char*>(lid.data()), pad);
    }
    if (!f) return "cannot write " + qd + "/ivt";
  }
  if (stride) {
    std::ofstream f(qd + "/grp", std::ios::binary);
    const uint64_t hdr[2] = {M, h.nrows};
    f.write(reinterpret_cast<const char*>(hdr), 16);
    const uint64_t me = (M + 1) / 2 * 2;
    for (uint64_t v = 0; v < h.nrows; v++) {
      const uint32_t* r = qids.data() + v * stride;
      uint32_t deg = 0;
      while (deg < stride && r[deg] != 0) deg++;
      f.write(reinterpret_cast<const char*>(&deg), 4);
      f.write(reinterpret_cast<const char*>(r), (size_t)deg * 4);
      const uint64_t nb = deg == 0 ? 0 : (deg - 1) / 16 + 1;
      f.write(reinterpret_cast<const char*>(qcodes.data() + v * cstride), (std::streamsize)(nb * 8 * me));
    }
    if (!f) return "cannot write " + qd + "/grp";
  }
  return "";
}

}  // namespace

extern "C" {

void ngtqg_initialize_query(NGTQGQuery* query) {
  query->query = 0;
  query->size = 20;
  query->epsilon = 0.03;
  query->result_expansion = 3.0;
  query->radius = FLT_MAX;
}

void ngtqg_initialize_quantization_parameters(NGTQGQuantizationParameters* parameters) {
  parameters->dimension_of_subvector = 0;
  parameters->max_number_of_edges = 128;
}

static NGTQGIndex open_qg(const char* func, const char* index_path, uint32_t max_edges, NGTError error) {
  auto* ix = new QgCapiIndex();
  std::string e;
  if (!index_path) e = "null index path";
  if (e.empty()) e = ngt_amd::load_index(index_path, ix->host);
  if (e.empty()) e = ngt_amd::load_qg(index_path, ix->host.nrows, ix->quant);
  if (e.empty() && (int64_t)ix->quant.dim != ix->host.prop.dimension) e = "qg/prf dimension differs from the index";
  if (e.empty() && max_edges == 0) e = "max_edges must be > 0";
  if (e.empty()) e = open_device(ix, max_edges);
  if (!e.empty()) {
    report(error, std::string("Capi : ") + func + "() : Error: " + e);
    delete ix;
    return NULL;
  }
  ix->co.reset(new ngt_amd::Coalescer((uint32_t)ix->host.prop.dimension));
  return static_cast<NGTQGIndex>(ix);
}

NGTQGIndex ngtqg_open_index(const char* index_path, NGTError error) {
  return open_qg(__FUNCTION__, index_path, 128, error);
}

NGTQGIndex ngtqg_open_index_with_max_edges(const char* index_path, uint32_t max_edges, NGTError error) {
  return open_qg(__FUNCTION__, index_path, max_edges, error);
}

void ngtqg_close_index(NGTQGIndex index) {
  if (index == NULL) return;
  delete static_cast<QgCapiIndex*>(index);
}

// The local codebooks of NGTQG::Index::quantize: NGTQ's dynamic k-means
// (Quantizer.h:1802-1858) inserts the residuals (object - global centroid, the
// zero vector for a quantized graph, QuantizedGraph.h:396-400) of the first
// localCentroidLimit x localClusteringSampleCoefficient = 16 x 100 objects
// into each local codebook index (ANNG, edge sizes 10/40, batch 200,
// insertion coefficient 1.1: the local prf the reference writes), then runs
// NGT::Clustering::kmeansWithNGT on it (kmeans_ngt.h).  Here each sample
// index is built by this library's device construction (ngt_create_index)
// and every assignment search is a device graph search (ngt_batch_search_index,
// tree seeds); the clustering logic is the restatement in kmeans_ngt.h.  The
// reference parallelises those searches with OpenMP while its tree-seed
// thinning draws from the process-wide rand() (Index.h:1555-1559), so its own
// codebooks differ from run to run; run with one OpenMP thread it is
// deterministic, and that is what this reproduces (tests/golden/c1_qg_st).
static std::string train_local_kmeans_ngt(const ngt_amd::HostIndex& h, uint32_t M, uint32_t dsub,
                                          std::vector<float>& local) {
  std::vector<uint64_t> sample;
  for (uint64_t i = 1; i < h.nrows && sample.size() < 16 * 100; i++)
    if (h.valid[i]) sample.push_back(i);
  const uint32_t n = (uint32_t)sample.size();
  local.assign((size_t)M * 16 * dsub, 0.0f);
  for (uint32_t m = 0; m < M; m++) {
    std::vector<std::vector<float>> vectors(n, std::vector<float>(dsub));
    std::vector<float> flat((size_t)n * dsub);
    for (uint32_t i = 0; i < n; i++) {
      const float* r = reinterpret_cast<const float*>(h.rows.data() + sample[i] * h.row_bytes);
      for (uint32_t j = 0; j < dsub; j++) vectors[i][j] = flat[(size_t)i * dsub + j] = r[(size_t)m * dsub + j];
    }
    NGTError err = ngt_create_error_object();
    NGTProperty prop = ngt_create_property(err);
    std::string e;
    NGTIndex idx = nullptr;
    if (!prop || !ngt_set_property_dimension(prop, (int32_t)dsub, err) ||
        !ngt_set_property_edge_size_for_creation(prop, 10, err) ||
        !ngt_set_property_edge_size_for_search(prop, 40, err) || !ngt_set_property_object_type_float(prop, err) ||
        !ngt_set_property_distance_type_l2(prop, err) || !(idx = ngt_create_graph_and_tree_in_memory(prop, err)) ||
        !ngt_batch_append_index(idx, flat.data(), n, err) || !ngt_create_index(idx, 24, err))
      e = ngt_get_error_string(err);
    if (e.empty()) {
      ngt_amd::kmeans::SearchFn search = [&](const std::vector<std::vector<float>>& qs, size_t size, float eps,
                                             std::vector<std::vector<std::pair<uint32_t, float>>>& out) {
        const uint32_t nq = (uint32_t)qs.size();
        std::vector<float> q((size_t)nq * dsub);
        for (uint32_t i = 0; i < nq; i++) std::copy(qs[i].begin(), qs[i].end(), q.begin() + (size_t)i * dsub);
        std::vector<uint32_t> ids((size_t)nq * size), cnt(nq);
        std::vector<float> ds((size_t)nq * size);
        if (!ngt_batch_search_index(idx, q.data(), nq, (int32_t)dsub, size, eps, -1.0f, -1, ids.data(), ds.data(),
                                    cnt.data(), err))
          return false;
        out.assign(nq, {});
        for (uint32_t i = 0; i < nq; i++)
          for (uint32_t r = 0; r < cnt[i]; r++) out[i].push_back({ids[(size_t)i * size + r], ds[(size_t)i * size + r]});
        return true;
      };
      std::vector<std::vector<float>> cents;
      ngt_amd::kmeans::Params prm;
      if (ngt_amd::kmeans::kmeans_with_ngt(search, vectors, 16, prm, cents, e) < 0.0 && e == "search failed")
        e = ngt_get_error_string(err);
      for (size_t c = 0; c < cents.size() && c < 16; c++)
        for (uint32_t j = 0; j < dsub; j++) local[((size_t)m * 16 + c) * dsub + j] = cents[c][j];
    }
    if (idx) ngt_close_index(idx);
    if (prop) ngt_destroy_property(prop);
    ngt_destroy_error_object(err);
    if (!e.empty()) return "local codebook " + std::to_string(m) + ": " + e;
  }
  return "";
}

// The local codebooks ngtqg_quantize trains (train_local_kmeans_ngt: the
// kmeansWithNGT restatement over the first 1,600 objects, Quantizer.h:1802-1858,
// Clustering.h:648-760), for callers that hold the objects themselves:
// rows = [nrows][dim] floats, row 0 the dummy slot; local = [M][16][dsub].
extern "C" int ngt_amd_qg_train_local_ngt(const float* rows, uint64_t nrows, uint32_t dim, uint32_t dsub,
                                          float* local_out) {
  if (!rows || !local_out || dim == 0 || dsub == 0 || dim % dsub != 0 || nrows < 17)
    return ngt_amd::fail("ngt_amd_qg_train_local_ngt: bad arguments");
  ngt_amd::HostIndex h;
  h.prop.dimension = (int32_t)dim;
  h.prop.object_type = NGT_AMD_OBJECT_FLOAT;
  h.prop.distance_type = NGT_AMD_DISTANCE_L2;
  h.init_layout();
  const uint64_t n = std::min<uint64_t>(nrows, 1601);  // the sample is the first 1,600 objects
  h.nrows = n;
  h.rows.assign((size_t)n * h.row_bytes, 0);
  h.valid.assign(n, 1);
  h.valid[0] = 0;
  for (uint64_t i = 1; i < n; i++) memcpy(h.rows.data() + i * h.row_bytes, rows + i * dim, (size_t)dim * 4);
  std::vector<float> local;
  const uint32_t M = dim / dsub;
  std::string e = train_local_kmeans_ngt(h, M, dsub, local);
  if (!e.empty()) return ngt_amd::fail("ngt_amd_qg_train_local_ngt: %s", e.c_str());
  std::copy(local.begin(), local.end(), local_out);
  return 0;
}

// NGTQG::Index::quantize (lib/NGT/NGTQ/QuantizedGraph.h:456-475) on the device:
// nothing when <index>/qg exists; else the quantizer frame (:423-454), the
// codebooks, every object's local codes (:392-421) and the quantized graph
// (:387-390), written in the reference's file formats: qg/prf (NGTQ::Property),
// qg/global and qg/local-<m> as NGT indexes (built by this library's ANNG
// construction), qg/ivt (Repository<InvertedIndexEntry<uint16_t>>) and qg/grp
// (QuantizedGraphRepository::serialize, :117-128).  The local codebooks come
// from the kmeansWithNGT restatement above (train_local_kmeans_ngt).
bool ngtqg_quantize(const char* indexPath, NGTQGQuantizationParameters parameters, NGTError error) {
  auto err = [&](const std::string& e) {
    report(error, std::string("Capi : ") + __FUNCTION__ + "() : Error: " + e);
    return false;
  };
  if (!indexPath) return err("null index path");
  const std::string qd = std::string(indexPath) + "/qg";
  struct stat st;
  if (stat(qd.c_str(), &st) == 0) return true;
  ngt_amd::HostIndex h;
  std::string e = ngt_amd::load_index(indexPath, h);
  if (!e.empty()) return err(e);
  if (h.prop.distance_type != NGT_AMD_DISTANCE_L2 || h.prop.object_type != NGT_AMD_OBJECT_FLOAT)
    return err("NGTQG supports L2 float indexes only");
  const uint32_t dim = (uint32_t)h.prop.dimension;
  // NGTQG::Index::getNumberOfSubvectors (:374-385)
  size_t dsub = (size_t)parameters.dimension_of_subvector;
  if (dsub == 0) {
    dsub = dim > 400 ? 2 : 1;
    dsub = dim % dsub == 0 ? dsub : 1;
  }
  if (dim % dsub != 0) return err("dimensionOfSubvector is invalid. " + std::to_string(dim) + " : " +
                                  std::to_string(dsub));
  const uint32_t M = (uint32_t)(dim / dsub);
  uint64_t nvalid = 0;
  for (uint64_t i = 1; i < h.nrows; i++) nvalid += h.valid[i] ? 1 : 0;
  if (nvalid < 16) return err("at least 16 objects are needed to train 16 centroids per subspace");
  QgCapiIndex ix;
  int dev = 0;
  if (const char* env = getenv("NGT_AMD_DEVICE")) dev = atoi(env);
  if (ngt_amd_index_create(&ix.dev, dev, h.prop.distance_type, h.prop.object_type, dim)) return err(amd_err());
  if (ngt_amd_index_set_objects(ix.dev, h.rows.data(), h.nrows, h.valid.data())) return err(amd_err());
  std::vector<float> local;
  e = train_local_kmeans_ngt(h, M, (uint32_t)dsub, local);
  if (!e.empty()) return err(e);
  {
    // the encoder below takes the codebooks from the device quantizer
    std::vector<float> zero(dim, 0.0f);
    if (ngt_amd_qg_set_quantizer(ix.dev, zero.data(), local.data(), M, (uint32_t)dsub)) return err(amd_err());
  }
  std::vector<uint8_t> codes((size_t)h.nrows * M);
  if (ngt_amd_qg_encode(ix.dev, codes.data())) return err(amd_err());
  const uint32_t max_edges = (uint32_t)parameters.max_number_of_edges;
  std::vector<uint32_t> qids;
  std::vector<uint8_t> qcodes;
  uint32_t stride = 0;
  uint64_t cstride = 0;
  if (max_edges != 0) {
    if (ngt_amd_index_set_graph(ix.dev, h.edge_off.data(), h.edges.data(), h.edges.size())) return err(amd_err());
    if (ngt_amd_qg_build_graph(ix.dev, nullptr, max_edges)) return err(amd_err());
    stride = ngt_amd_qg_max_degree(ix.dev);
    cstride = ngt_amd_qg_code_stride(ix.dev);
    qids.resize((size_t)h.nrows * stride);
    qcodes.resize((size_t)h.nrows * cstride);
    if (ngt_amd_qg_get_graph(ix.dev, qids.data(), qcodes.data())) return err(amd_err());
  }
  e = write_quantizer(qd, h, dim, M, (uint32_t)dsub, local, codes, stride, cstride, qids, qcodes);
  if (!e.empty()) return err(e);
  return true;
}

bool ngtqg_search_index(NGTQGIndex index, NGTQGQuery query, NGTObjectDistances results, NGTError error) {
  if (index == NULL || query.query == NULL || results == NULL) {
    std::stringstream ss;
    ss << "Capi : " << __FUNCTION__ << "() : parametor error: index = " << index << " query = " << query.query
       << " results = " << results;
    report(error, ss.str());
    return false;
  }
  auto* ix = static_cast<QgCapiIndex*>(index);
  if (query.radius < 0.0) query.radius = FLT_MAX;
  std::vector<uint32_t> ids;
  std::vector<float> dists;
  uint32_t nres = 0;
  std::string e;
  if (!ngt_amd::coalesce_enabled()) {
    std::vector<uint32_t> n;
    e = run(ix, query.query, 1, query.size, query.epsilon, query.result_expansion, query.radius, ids, dists, n);
    nres = n.empty() ? 0 : n[0];
  } else {
    // concurrent callers with equal parameters share one launch (coalesce.h)
    ngt_amd::CoalesceReq r;
    r.key.kind = 2;
    r.key.size = (uint32_t)query.size;
    r.key.epsilon = query.epsilon;
    r.key.radius = query.radius;
    r.key.expansion = query.result_expansion;
    r.query = query.query;
    ix->co->submit(&r, [ix](const ngt_amd::CoalesceKey& k, const float* qs, uint32_t nq,
                            std::vector<ngt_amd::CoalesceReq*>& batch) {
      std::vector<uint32_t> vi, vn;
      std::vector<float> vd;
      std::string err = run(ix, qs, nq, k.size, k.epsilon, k.expansion, k.radius, vi, vd, vn);
      for (uint32_t i = 0; i < nq; i++) {
        batch[i]->err = err;
        if (!err.empty()) continue;
        batch[i]->n = vn[i];
        batch[i]->ids.assign(vi.begin() + (size_t)i * k.size, vi.begin() + (size_t)i * k.size + vn[i]);
        batch[i]->dists.assign(vd.begin() + (size_t)i * k.size, vd.begin() + (size_t)i * k.size + vn[i]);
      }
    });
    e = r.err;
    ids.swap(r.ids);
    dists.swap(r.dists);
    nres = r.n;
  }
  if (!e.empty()) {
    report(error, std::string("Capi : ") + __FUNCTION__ + "() : Error: " + e);
    return false;
  }
  Results* r = static_cast<Results*>(results);
  r->clear();  // moveFrom overwrites the result set
  for (uint32_t i = 0; i < nres; i++) r->push_back(NGTObjectDistance{ids[i], dists[i]});
  return true;
}

bool ngtqg_batch_search_index(NGTQGIndex index, const float* queries, uint32_t nq, int32_t dim, size_t size,
                              float epsilon, float result_expansion, float radius, uint32_t* ids, float* dists,
                              uint32_t* n, NGTError error) {
  if (index == NULL || (queries == NULL && nq) || ids == NULL || dists == NULL || n == NULL) {
    std::stringstream ss;
    ss << "Capi : " << __FUNCTION__ << "() : parametor error: index = " << index << " queries = " << queries;
    report(error, ss.str());
    return false;
  }
  auto* ix = static_cast<QgCapiIndex*>(index);
  if (dim != ix->host.prop.dimension) {
    report(error, std::string("Capi : ") + __FUNCTION__ + "() : Error: dimension mismatch");
    return false;
  }
  std::vector<uint32_t> vi, vn;
  std::vector<float> vd;
  std::string e = run(ix, queries, nq, size, epsilon, result_expansion, radius, vi, vd, vn);
  if (!e.empty()) {
    report(error, std::string("Capi : ") + __FUNCTION__ + "() : Error: " + e);
    return false;
  }
  std::copy(vn.begin(), vn.end(), n);
  if (size) {
    std::copy(vi.begin(), vi.end(), ids);
    std::copy(vd.begin(), vd.end(), dists);
  }
  return true;
}

}  // extern "C"
