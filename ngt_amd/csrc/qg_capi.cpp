// qg_capi.cpp -- the reference's `ngtqg_*` C API (lib/NGT/NGTQ/Capi.cpp:40-131)
// on the MI355X path.  An NGTQGIndex is the NGT index (prf/obj/grp/tre) plus
// its <index>/qg quantizer, loaded straight into HBM: exact rows, graph and
// DVP tree through ngt_amd_index_*, codebooks and the quantized graph through
// ngt_amd_qg_* (constructed on the device from qg/ivt unless qg/grp was
// saved, as NGTQG::Index's constructor does, QuantizedGraph.h:170-185).
// Search = NGTQG::Index::search(SearchQuery&) (:354-372) as one device batch.
#include <float.h>
#include <stdlib.h>

#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/NGT/Capi.h"
#include "../../include/NGT/NGTQ/Capi.h"
#include "../../include/ngt_amd.h"
#include "index_io.h"

namespace {

struct QgCapiIndex {
  ngt_amd::HostIndex host;
  ngt_amd::HostQuantizer quant;
  ngt_amd_index* dev = nullptr;
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

std::string open_device(QgCapiIndex* ix) {
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
    // QuantizedGraphRepository::construct with the default maxNoOfEdges (QuantizedGraph.h:170)
    if (ngt_amd_qg_build_graph(ix->dev, q.codes.data(), 128)) return amd_err();
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

NGTQGIndex ngtqg_open_index(const char* index_path, NGTError error) {
  auto* ix = new QgCapiIndex();
  std::string e;
  if (!index_path) e = "null index path";
  if (e.empty()) e = ngt_amd::load_index(index_path, ix->host);
  if (e.empty()) e = ngt_amd::load_qg(index_path, ix->host.nrows, ix->quant);
  if (e.empty() && (int64_t)ix->quant.dim != ix->host.prop.dimension) e = "qg/prf dimension differs from the index";
  if (e.empty()) e = open_device(ix);
  if (!e.empty()) {
    report(error, std::string("Capi : ") + __FUNCTION__ + "() : Error: " + e);
    delete ix;
    return NULL;
  }
  return static_cast<NGTQGIndex>(ix);
}

void ngtqg_close_index(NGTQGIndex index) {
  if (index == NULL) return;
  delete static_cast<QgCapiIndex*>(index);
}

bool ngtqg_quantize(const char* indexPath, NGTQGQuantizationParameters parameters, NGTError error) {
  (void)indexPath;
  (void)parameters;
  report(error, std::string("Capi : ") + __FUNCTION__ +
                    "() : Error: quantization (codebook training) is not available in this build; "
                    "quantize with the reference's `ngtqg quantize` and open the index here");
  return false;
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
  std::vector<uint32_t> ids, n;
  std::vector<float> dists;
  std::string e = run(ix, query.query, 1, query.size, query.epsilon, query.result_expansion, query.radius, ids,
                      dists, n);
  if (!e.empty()) {
    report(error, std::string("Capi : ") + __FUNCTION__ + "() : Error: " + e);
    return false;
  }
  Results* r = static_cast<Results*>(results);
  r->clear();  // moveFrom overwrites the result set
  for (uint32_t i = 0; i < n[0]; i++) r->push_back(NGTObjectDistance{ids[i], dists[i]});
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
