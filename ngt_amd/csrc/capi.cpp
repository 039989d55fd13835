// capi.cpp -- the reference's `ngt_*` C API (lib/NGT/Capi.cpp) served by the
// MI355X path.  An NGTIndex is a host mirror of the index files (needed for
// ngt_get_object_as_float's borrowed pointers, Capi.cpp:750-765, and for
// ngt_save_index) plus a device-resident ngt_amd_index that every search and
// linear search runs on.  Error convention of Capi.cpp:25-38.
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <iostream>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/NGT/Capi.h"
#include "../../include/ngt_amd.h"
#include "coalesce.h"
#include "index_io.h"

using ngt_amd::HostIndex;
using ngt_amd::HostProperty;

namespace {

struct CapiIndex {
  HostIndex host;
  ngt_amd_index* dev = nullptr;
  bool device_stale = true;
  // Searches hold `rw` shared from the device check to the end of their
  // device call; appends/inserts, construction and the device rebuild hold it
  // exclusively, so a rebuild never frees rows a running batch still reads.
  std::shared_mutex rw;
  std::mutex mu;                           // the coalescer's lazy creation
  std::unique_ptr<ngt_amd::Coalescer> co;  // concurrent single-query callers
  ~CapiIndex() {
    if (dev) ngt_amd_index_destroy(dev);
  }
};

// The last search's counters are per calling thread: concurrent callers of
// one handle each read their own (ngt_get_last_search_counters).
thread_local uint64_t t_last_counters[3] = {0, 0, 0};

typedef std::vector<NGTObjectDistance> Results;

bool set_error(NGTError error, const char* func, const std::string& what) {
  std::stringstream ss;
  ss << "Capi : " << func << "() : Error: " << what;
  if (error != NULL) {
    *static_cast<std::string*>(error) = ss.str();
  } else {
    std::cerr << ss.str() << std::endl;
  }
  return true;
}

bool param_error(NGTError error, const char* func, const std::string& what) {
  std::stringstream ss;
  ss << "Capi : " << func << "() : parametor error: " << what;
  if (error != NULL) {
    *static_cast<std::string*>(error) = ss.str();
  } else {
    std::cerr << ss.str() << std::endl;
  }
  return true;
}

std::string amd_err() { return std::string(ngt_amd_last_error()); }

// Build / refresh the device index from the host mirror (caller holds `rw`
// exclusively).
std::string rebuild_device(CapiIndex* ix) {
  if (!ix->device_stale && ix->dev) return "";
  HostIndex& h = ix->host;
  if (h.nrows < 2) return "the index is empty";
  if (!ix->dev) {
    int dev = 0;
    const char* env = getenv("NGT_AMD_DEVICE");
    if (env) dev = atoi(env);
    if (ngt_amd_index_create(&ix->dev, dev, h.prop.distance_type, h.prop.object_type,
                             (uint32_t)h.prop.object_dimension()))
      return amd_err();
  }
  if (ngt_amd_index_set_objects(ix->dev, h.rows.data(), h.nrows, h.valid.data())) return amd_err();
  if (h.edge_off.size() == h.nrows + 1 && !h.edges.empty()) {
    if (ngt_amd_index_set_graph(ix->dev, h.edge_off.data(), h.edges.data(), h.edges.size()))
      return amd_err();
  }
  if (h.tree.present) {
    const ngt_amd::HostTree& t = h.tree;
    if (ngt_amd_index_set_tree(ix->dev, t.in_pivot.data(), t.n_internal(), t.in_child.data(),
                               t.in_border.data(), 5, t.root, t.leaf_off.data(), t.n_leaf(),
                               t.leaf_ids.data(), t.leaf_ids.size()))
      return amd_err();
  }
  ngt_amd_index_set_search_property(ix->dev, h.prop.edge_size_for_search, h.prop.dynamic_edge_size_base,
                                    h.prop.dynamic_edge_size_rate, h.prop.seed_size, h.prop.seed_type);
  ix->device_stale = false;
  return "";
}

// A current device copy, with `rd` holding `rw` shared on success: the copy
// cannot be rebuilt under the caller until `rd` is released.
std::string sync_device(CapiIndex* ix, std::shared_lock<std::shared_mutex>& rd) {
  for (;;) {
    rd = std::shared_lock<std::shared_mutex>(ix->rw);
    if (!ix->device_stale && ix->dev) return "";
    rd.unlock();
    std::unique_lock<std::shared_mutex> wl(ix->rw);
    std::string e = rebuild_device(ix);
    if (!e.empty()) return e;
  }
}

bool use_tree(CapiIndex* ix) { return ix->host.prop.index_type == 0 && ix->host.tree.present; }

// One batched search: the single-query API is a batch of one.
std::string run_search(CapiIndex* ix, const float* queries, uint32_t nq, size_t size, float epsilon,
                       float radius, int64_t edge_size, int seed_mode, std::vector<uint32_t>& ids,
                       std::vector<float>& dists, std::vector<uint32_t>& n,
                       std::vector<uint64_t>* per_query = nullptr) {
  std::shared_lock<std::shared_mutex> rd;
  std::string e = sync_device(ix, rd);
  if (!e.empty()) return e;
  if (size == 0) {
    // GraphIndex::search with sc.size == 0 returns nothing (Index.h:1141-1144)
    n.assign(nq, 0);
    return "";
  }
  ngt_amd_search_params p{};
  p.k = (uint32_t)size;
  p.epsilon = epsilon;
  p.radius = radius < 0.0f ? FLT_MAX : radius;
  p.edge_size = edge_size;
  p.seed_mode = seed_mode;
  p.all_leaf_nodes = 0;
  // large indexes: visited epochs in HBM from the start (behind the LDS
  // filter) instead of an LDS hash that would spill after a few thousand ids;
  // identical results and distance counts either way
  p.visited_hash_log2 = ix->host.nrows >= (1u << 18) ? -1 : 0;
  ids.resize((size_t)nq * size);
  dists.resize((size_t)nq * size);
  n.resize(nq);
  std::vector<uint64_t> cnt((size_t)nq * NGT_AMD_COUNTERS_PER_QUERY);
  if (ngt_amd_search(ix->dev, &p, queries, nq, nullptr, nullptr, ids.data(), dists.data(), n.data(),
                     cnt.data()))
    return amd_err();
  // the reference's SearchContainer counters of a read-write search
  // (NeighborhoodGraph::search, Graph.cpp:588-604): distanceComputationCount
  // counts neighbour distances (seed distances only under
  // NGT_DISTANCE_COMPUTATION_COUNT, off by default, :287), visitCount every
  // scanned edge; then expansions
  t_last_counters[0] = t_last_counters[1] = t_last_counters[2] = 0;
  for (uint32_t q = 0; q < nq; q++) {
    const uint64_t* c = cnt.data() + (size_t)q * NGT_AMD_COUNTERS_PER_QUERY;
    t_last_counters[0] += c[1];
    t_last_counters[1] += c[4];
    t_last_counters[2] += c[2];
  }
  if (per_query) *per_query = std::move(cnt);
  return "";
}

std::string run_linear(CapiIndex* ix, const float* queries, uint32_t nq, size_t size,
                       std::vector<uint32_t>& ids, std::vector<float>& dists, std::vector<uint32_t>& n,
                       double radius = (double)FLT_MAX) {
  std::shared_lock<std::shared_mutex> rd;
  std::string e = sync_device(ix, rd);
  if (!e.empty()) return e;
  if (size == 0) {
    n.assign(nq, 0);
    return "";
  }
  ids.resize((size_t)nq * size);
  dists.resize((size_t)nq * size);
  n.resize(nq);
  // sc.radius stays FLT_MAX in ngt_linear_search_index_ (Capi.cpp:441-456);
  // ngtpy passes its default radius (ngtpy.cpp:238)
  if (ngt_amd_linear_search(ix->dev, queries, nq, (uint32_t)size, radius, ids.data(),
                            dists.data(), n.data()))
    return amd_err();
  return "";
}

void fill_results(NGTObjectDistances results, const std::vector<uint32_t>& ids,
                  const std::vector<float>& dists, uint32_t n) {
  Results* r = static_cast<Results*>(results);
  r->clear();
  for (uint32_t i = 0; i < n; i++) r->push_back(NGTObjectDistance{ids[i], dists[i]});
}

HostProperty* prop_of(NGTProperty p) { return static_cast<HostProperty*>(p); }

std::string create_empty(CapiIndex* ix, const HostProperty& prop) {
  ix->host = HostIndex();
  ix->host.prop = prop;
  if (prop.dimension <= 0) return "dimension is not specified";
  ix->host.init_layout();
  ix->host.nrows = 1;  // dummy slot 0 (ObjectRepository.h:37-40)
  ix->host.rows.assign(ix->host.row_bytes, 0);
  ix->host.valid.assign(1, 0);
  ix->host.edge_off.assign(2, 0);
  ix->device_stale = true;
  return "";
}

// ObjectSpace::normalize (ObjectSpace.h:251-266) of one stored object, with
// the arithmetic of the device query preparation (prep_kernels.hip: 16 FMA
// lanes over the unpadded dimension, 8/4/2/1 fold, FMA tail, sqrtf, divide),
// so an inserted object and the same vector given as a query normalize to
// the same bits.
template <typename T>
std::string normalize_row(T* data, uint32_t dim) {
  float acc[16] = {0};
  const uint32_t main = dim & ~15u;
  for (uint32_t i = 0; i < main; i++) acc[i & 15] = fmaf((float)data[i], (float)data[i], acc[i & 15]);
  for (int w = 8; w >= 1; w >>= 1)
    for (int l = 0; l < w; l++) acc[l] = acc[l + w] + acc[l];
  float sum = acc[0];
  for (uint32_t i = main; i < dim; i++) sum = fmaf((float)data[i], (float)data[i], sum);
  if (sum == 0.0f)
    return "ObjectSpace::normalize: Error! the object is an invalid zero vector for the cosine similarity or "
           "normalized distances.";
  const float scale = sqrtf(sum);
  for (uint32_t i = 0; i < dim; i++) data[i] = static_cast<T>((float)data[i] / scale);
  return "";
}

// Append one object to the host mirror, converting like
// ObjectRepository::allocateObject (ObjectRepository.h:222-253) and, for the
// normalized metrics, normalizing like allocateNormalizedObject
// (ObjectSpaceRepository.h:560-566).
template <typename T>
std::string append_object(CapiIndex* ix, const T* obj, uint32_t dim, uint32_t& id) {
  std::unique_lock<std::shared_mutex> wl(ix->rw);
  HostIndex& h = ix->host;
  const bool sparse = h.prop.distance_type == 8;
  // a sparse object (0-terminated id list, Index::makeSparseObject) may be
  // shorter than the object dimension (ObjectRepository.h:222-233)
  if (sparse ? (int32_t)dim > h.prop.object_dimension() : (int32_t)dim != h.prop.dimension)
    return "the specified dimension is invalid";
  const int m = h.prop.distance_type;
  const bool normalized = m == 5 || m == 6 || m == 9;
  std::vector<uint8_t> row(h.row_bytes, 0);
  if (h.prop.object_type == 2) {
    float* f = reinterpret_cast<float*>(row.data());
    for (uint32_t i = 0; i < dim; i++) f[i] = static_cast<float>(obj[i]);
    if (normalized) {
      std::string e = normalize_row(f, dim);
      if (!e.empty()) return e;
    }
  } else {
    for (uint32_t i = 0; i < dim; i++) row[i] = static_cast<uint8_t>(obj[i]);
    if (normalized) {
      std::string e = normalize_row(row.data(), dim);
      if (!e.empty()) return e;
    }
  }
  id = (uint32_t)h.nrows;
  h.rows.insert(h.rows.end(), row.begin(), row.end());
  h.valid.push_back(1);
  h.nrows++;
  h.edge_off.push_back(h.edge_off.back());
  ix->device_stale = true;
  return "";
}

// GraphAndTreeIndex::createIndex for the objects appended since the last
// build: ANNG with the tree, on the device; the host mirror receives the
// graph (CSR + distances) and the DVP tree for ngt_save_index and searches.
std::string build_anng(CapiIndex* ix) {
  std::unique_lock<std::shared_mutex> wl(ix->rw);
  HostIndex& h = ix->host;
  if (h.prop.edge_size_for_creation == 0) return "";  // createIndex returns at once (Index.cpp:1162-1164)
  if (h.prop.graph_type != 1) return "index construction supports graphType ANNG only";
  if (h.prop.index_type != 0) return "index construction supports GraphAndTree indexes only";
  bool has_graph = false;
  for (uint64_t v = 0; v < h.nrows && v + 1 < h.edge_off.size() && !has_graph; v++)
    has_graph = h.edge_off[v + 1] != h.edge_off[v];
  if (has_graph && !h.tree.present) return "the index has a graph but no DVP tree";
  if (h.nrows < 2) return "";
  std::string e = rebuild_device(ix);
  if (!e.empty()) return e;
  ngt_amd_build_params p{};
  p.edge_size_for_creation = h.prop.edge_size_for_creation;
  p.edge_size_for_search = h.prop.edge_size_for_search;
  p.batch_size_for_creation = h.prop.batch_size_for_creation;
  p.seed_size = h.prop.seed_size;
  p.epsilon_for_creation = (float)h.prop.epsilon_for_creation;
  if (ngt_amd_build_begin(ix->dev, &p)) return amd_err();
  if (has_graph) {
    // incremental: the objects without a node join the existing graph and tree
    const ngt_amd::HostTree& t = h.tree;
    const uint32_t nl = (uint32_t)t.leaf_parent.size(), ni = (uint32_t)t.in_parent.size();
    if (h.edge_off.size() < h.nrows + 1 || h.edge_dists.size() != h.edges.size())
      return "graph arrays inconsistent with the repository";
    if (ngt_amd_build_set_graph(ix->dev, h.edge_off.data(), h.edges.data(), h.edge_dists.data(), h.nrows) ||
        ngt_amd_build_set_tree(ix->dev, t.leaf_parent.data(), t.leaf_off.data(), t.leaf_ids.data(),
                               t.leaf_dists.data(), t.leaf_has_pivot.data(), t.leaf_pivot.data(), nl,
                               t.in_parent.data(), t.in_pivot.data(), t.in_child.data(), t.in_border.data(),
                               ni < 1 ? 1u : ni, t.root))
      return amd_err();
  }
  if (ngt_amd_build_insert(ix->dev, 1, h.nrows)) return amd_err();
  uint64_t gsize = 0, ne = 0;
  if (ngt_amd_build_graph_size(ix->dev, &gsize, &ne)) return amd_err();
  std::vector<uint64_t> off(gsize + 1);
  h.edges.resize(ne);
  h.edge_dists.resize(ne);
  if (ngt_amd_build_get_graph(ix->dev, off.data(), h.edges.data(), h.edge_dists.data())) return amd_err();
  h.edge_off.assign(h.nrows + 1, ne);
  for (uint64_t v = 0; v <= h.nrows && v <= gsize; v++) h.edge_off[v] = off[v];
  h.prevsize.assign(h.nrows, 0);
  uint32_t nl = 0, ni = 0;
  uint64_t nli = 0;
  if (ngt_amd_build_tree_size(ix->dev, &nl, &ni, &nli)) return amd_err();
  ngt_amd::HostTree& t = h.tree;
  t = ngt_amd::HostTree();
  t.leaf_parent.resize(nl);
  t.leaf_off.resize((size_t)nl + 1);
  t.leaf_ids.resize(nli);
  t.leaf_dists.resize(nli);
  t.leaf_has_pivot.resize(nl);
  t.leaf_pivot.resize((size_t)nl * h.row_bytes);
  t.in_parent.resize(ni);
  t.in_pivot.resize((size_t)ni * h.row_bytes);
  t.in_child.resize((size_t)ni * 5);
  t.in_border.resize((size_t)ni * 4);
  if (ngt_amd_build_get_tree(ix->dev, t.leaf_parent.data(), t.leaf_off.data(), t.leaf_ids.data(),
                             t.leaf_dists.data(), t.leaf_has_pivot.data(), t.leaf_pivot.data(), t.in_parent.data(),
                             t.in_pivot.data(), t.in_child.data(), t.in_border.data()))
    return amd_err();
  t.leaf_valid.assign(nl, 1);
  t.leaf_valid[0] = 0;
  t.in_valid.assign(ni, 1);
  if (ni) t.in_valid[0] = 0;
  for (uint32_t i = 1; i < nl; i++)  // LeafNode::serialize writes the pivot unless the leaf is an empty root
    t.leaf_has_pivot[i] = !((t.leaf_parent[i] & 0x7fffffffu) == 0 && t.leaf_off[i + 1] == t.leaf_off[i]);
  t.root = ni > 1 ? 1u : 0x80000001u;
  t.present = nl > 1;
  ix->device_stale = true;
  return "";
}

const char* kNotImplemented =
    "not implemented in the MI355X build yet (index construction / graph maintenance, SURVEY.md 8(f))";

}  // namespace

extern "C" {

NGTIndex ngt_open_index(const char* index_path, NGTError error) {
  try {
    CapiIndex* ix = new CapiIndex();
    // the device copy is built lazily on the first search (sync_device)
    std::string e = ngt_amd::load_index(index_path, ix->host);
    if (!e.empty()) {
      delete ix;
      set_error(error, __FUNCTION__, e);
      return NULL;
    }
    return static_cast<NGTIndex>(ix);
  } catch (std::exception& err) {
    set_error(error, __FUNCTION__, err.what());
    return NULL;
  }
}

NGTIndex ngt_create_graph_and_tree(const char* database, NGTProperty prop, NGTError error) {
  if (database == NULL || prop == NULL) {
    param_error(error, __FUNCTION__, "database or prop is null");
    return NULL;
  }
  CapiIndex* ix = new CapiIndex();
  std::string e = create_empty(ix, *prop_of(prop));
  if (e.empty()) {
    mkdir(database, 0755);
    e = ngt_amd::save_index(database, ix->host);
  }
  if (!e.empty()) {
    delete ix;
    set_error(error, __FUNCTION__, e);
    return NULL;
  }
  return static_cast<NGTIndex>(ix);
}

NGTIndex ngt_create_graph_and_tree_in_memory(NGTProperty prop, NGTError error) {
  if (prop == NULL) {
    param_error(error, __FUNCTION__, "prop is null");
    return NULL;
  }
  CapiIndex* ix = new CapiIndex();
  std::string e = create_empty(ix, *prop_of(prop));
  if (!e.empty()) {
    delete ix;
    set_error(error, __FUNCTION__, e);
    return NULL;
  }
  return static_cast<NGTIndex>(ix);
}

NGTProperty ngt_create_property(NGTError error) {
  try {
    HostProperty* p = new HostProperty();
    p->set_defaults();
    return static_cast<NGTProperty>(p);
  } catch (std::exception& err) {
    set_error(error, __FUNCTION__, err.what());
    return NULL;
  }
}

bool ngt_save_index(const NGTIndex index, const char* database, NGTError error) {
  if (index == NULL || database == NULL) {
    param_error(error, __FUNCTION__, "index or database is null");
    return false;
  }
  mkdir(database, 0755);
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  std::shared_lock<std::shared_mutex> rd(ix->rw);  // no append/insert/build while the mirror is written out
  std::string e = ngt_amd::save_index(database, ix->host);
  if (!e.empty()) {
    set_error(error, __FUNCTION__, e);
    return false;
  }
  return true;
}

bool ngt_get_property(NGTIndex index, NGTProperty prop, NGTError error) {
  if (index == NULL || prop == NULL) {
    std::stringstream ss;
    ss << "index = " << index << " prop = " << prop;
    param_error(error, __FUNCTION__, ss.str());
    return false;
  }
  *prop_of(prop) = static_cast<CapiIndex*>(index)->host.prop;
  return true;
}

#define PROP_GUARD(RET)                                        \
  if (prop == NULL) {                                          \
    std::stringstream ss;                                      \
    ss << "prop = " << prop;                                   \
    param_error(error, __FUNCTION__, ss.str());                \
    return RET;                                                \
  }

int32_t ngt_get_property_dimension(NGTProperty prop, NGTError error) {
  PROP_GUARD(-1);
  return prop_of(prop)->dimension;
}
bool ngt_set_property_dimension(NGTProperty prop, int32_t value, NGTError error) {
  PROP_GUARD(false);
  prop_of(prop)->dimension = value;
  return true;
}
bool ngt_set_property_edge_size_for_creation(NGTProperty prop, int16_t value, NGTError error) {
  PROP_GUARD(false);
  prop_of(prop)->edge_size_for_creation = value;
  return true;
}
bool ngt_set_property_edge_size_for_search(NGTProperty prop, int16_t value, NGTError error) {
  PROP_GUARD(false);
  prop_of(prop)->edge_size_for_search = value;
  return true;
}
int32_t ngt_get_property_object_type(NGTProperty prop, NGTError error) {
  PROP_GUARD(-1);
  return prop_of(prop)->object_type;
}
bool ngt_is_property_object_type_float(int32_t object_type) { return object_type == 2; }
bool ngt_is_property_object_type_integer(int32_t object_type) { return object_type == 1; }
bool ngt_set_property_object_type_float(NGTProperty prop, NGTError error) {
  PROP_GUARD(false);
  prop_of(prop)->object_type = 2;
  return true;
}
bool ngt_set_property_object_type_integer(NGTProperty prop, NGTError error) {
  PROP_GUARD(false);
  prop_of(prop)->object_type = 1;
  return true;
}
#define SET_DIST(FN, VAL)                       \
  bool FN(NGTProperty prop, NGTError error) {   \
    PROP_GUARD(false);                          \
    prop_of(prop)->distance_type = VAL;         \
    return true;                                \
  }
SET_DIST(ngt_set_property_distance_type_l1, 0)
SET_DIST(ngt_set_property_distance_type_l2, 1)
SET_DIST(ngt_set_property_distance_type_angle, 3)
SET_DIST(ngt_set_property_distance_type_hamming, 2)
SET_DIST(ngt_set_property_distance_type_jaccard, 7)
SET_DIST(ngt_set_property_distance_type_cosine, 4)
SET_DIST(ngt_set_property_distance_type_normalized_angle, 5)
SET_DIST(ngt_set_property_distance_type_normalized_cosine, 6)
SET_DIST(ngt_set_property_distance_type_normalized_l2, 9)
SET_DIST(ngt_set_property_distance_type_sparse_jaccard, 8)
#undef SET_DIST

int16_t ngt_get_property_edge_size_for_creation(NGTProperty prop, NGTError error) {
  PROP_GUARD(-1);
  return (int16_t)prop_of(prop)->edge_size_for_creation;
}
int16_t ngt_get_property_edge_size_for_search(NGTProperty prop, NGTError error) {
  PROP_GUARD(-1);
  return (int16_t)prop_of(prop)->edge_size_for_search;
}
int32_t ngt_get_property_distance_type(NGTProperty prop, NGTError error) {
  PROP_GUARD(-1);
  return prop_of(prop)->distance_type;
}

NGTObjectDistances ngt_create_empty_results(NGTError error) {
  try {
    return static_cast<NGTObjectDistances>(new Results());
  } catch (std::exception& err) {
    set_error(error, __FUNCTION__, err.what());
    return NULL;
  }
}

static ngt_amd::Coalescer* coalescer_of(CapiIndex* ix) {
  std::lock_guard<std::mutex> lk(ix->mu);
  if (!ix->co) ix->co.reset(new ngt_amd::Coalescer((uint32_t)ix->host.prop.object_dimension()));
  return ix->co.get();
}

// The query as the device takes it: object_dimension floats (a sparse query
// shorter than that is zero-padded; other metrics need the exact dimension).
static bool query_of(CapiIndex* ix, const float* q, int32_t qdim, std::vector<float>& out) {
  const HostProperty& p = ix->host.prop;
  if (p.distance_type == 8 ? (qdim > p.object_dimension()) : (qdim != p.dimension)) return false;
  out.assign(q, q + qdim);
  out.resize(p.object_dimension(), 0.0f);
  return true;
}

enum { kGraphSearch = 0, kLinearSearch = 1 };

// One single-query call: joins the batch of concurrent callers with the same
// parameters (coalesce.h), or runs alone when coalescing is off.
static std::string single_query(CapiIndex* ix, int kind, const float* q, size_t size, float epsilon, float radius,
                                int64_t edge_size, int seed_mode, std::vector<uint32_t>& ids,
                                std::vector<float>& dists, uint32_t& n) {
  // graph searches first try the resident serving grid (serve.cpp): answered
  // as soon as this query finishes, without a launch or a batch to wait for
  if (kind == kGraphSearch && size > 0 && size <= 64) {
    std::shared_lock<std::shared_mutex> rd;
    std::string e = sync_device(ix, rd);
    if (!e.empty()) return e;
    ngt_amd_search_params p{};
    p.k = (uint32_t)size;
    p.epsilon = epsilon;
    p.radius = radius < 0.0f ? FLT_MAX : radius;
    p.edge_size = edge_size;
    p.seed_mode = seed_mode;
    ids.resize(size);
    dists.resize(size);
    uint64_t c[NGT_AMD_COUNTERS_PER_QUERY];
    const int r = ngt_amd_search_served(ix->dev, &p, q, ids.data(), dists.data(), &n, c);
    if (r < 0) return amd_err();
    if (r == 0) {
      // the counters run_search reports (NeighborhoodGraph::search)
      t_last_counters[0] = c[1];
      t_last_counters[1] = c[4];
      t_last_counters[2] = c[2];
      return "";
    }
  }
  if (!ngt_amd::coalesce_enabled()) {
    std::vector<uint32_t> vn;
    std::string e = kind == kGraphSearch
                        ? run_search(ix, q, 1, size, epsilon, radius, edge_size, seed_mode, ids, dists, vn)
                        : run_linear(ix, q, 1, size, ids, dists, vn);
    n = vn.empty() ? 0 : vn[0];
    return e;
  }
  ngt_amd::CoalesceReq r;
  r.key.kind = kind;
  r.key.size = (uint32_t)size;
  r.key.epsilon = epsilon;
  r.key.radius = radius;
  r.key.edge_size = edge_size;
  r.key.seed_mode = seed_mode;
  r.query = q;
  coalescer_of(ix)->submit(&r, [ix](const ngt_amd::CoalesceKey& k, const float* qs, uint32_t nq,
                                    std::vector<ngt_amd::CoalesceReq*>& batch) {
    std::vector<uint32_t> vi, vn;
    std::vector<float> vd;
    std::vector<uint64_t> cnt;
    std::string e = k.kind == kGraphSearch
                        ? run_search(ix, qs, nq, k.size, k.epsilon, k.radius, k.edge_size, k.seed_mode, vi, vd, vn,
                                     &cnt)
                        : run_linear(ix, qs, nq, k.size, vi, vd, vn);
    for (uint32_t i = 0; i < nq; i++) {
      ngt_amd::CoalesceReq* b = batch[i];
      b->err = e;
      if (!e.empty()) continue;
      b->n = vn[i];
      b->ids.assign(vi.begin() + (size_t)i * k.size, vi.begin() + (size_t)i * k.size + vn[i]);
      b->dists.assign(vd.begin() + (size_t)i * k.size, vd.begin() + (size_t)i * k.size + vn[i]);
      if (!cnt.empty()) {
        const uint64_t* c = cnt.data() + (size_t)i * NGT_AMD_COUNTERS_PER_QUERY;
        b->counters[0] = c[1];
        b->counters[1] = c[4];
        b->counters[2] = c[2];
      }
    }
  });
  if (r.err.empty()) {
    ids.swap(r.ids);
    dists.swap(r.dists);
    n = r.n;
    if (kind == kGraphSearch) memcpy(t_last_counters, r.counters, sizeof r.counters);
  }
  return r.err;
}

static bool search_one(const char* func, NGTIndex index, const float* q, size_t size, float epsilon,
                       float radius, int64_t edge_size, NGTObjectDistances results, NGTError error) {
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  std::vector<uint32_t> ids;
  std::vector<float> dists;
  uint32_t n = 0;
  if (radius < 0.0f) radius = FLT_MAX;  // Capi.cpp:357-359
  std::string e = single_query(ix, kGraphSearch, q, size, epsilon, radius, edge_size,
                               use_tree(ix) ? NGT_AMD_SEED_TREE : NGT_AMD_SEED_RANDOM, ids, dists, n);
  if (!e.empty()) {
    set_error(error, func, e);
    return false;
  }
  fill_results(results, ids, dists, n);
  return true;
}

bool ngt_search_index(NGTIndex index, double* query, int32_t query_dim, size_t size, float epsilon,
                      float radius, NGTObjectDistances results, NGTError error) {
  if (index == NULL || query == NULL || results == NULL || query_dim <= 0) {
    std::stringstream ss;
    ss << "index = " << index << " query = " << query << " results = " << results << " query_dim = " << query_dim;
    param_error(error, __FUNCTION__, ss.str());
    return false;
  }
  std::vector<float> qf(query, query + query_dim), q;
  if (!query_of(static_cast<CapiIndex*>(index), qf.data(), query_dim, q)) {
    set_error(error, __FUNCTION__, "the specified dimension is invalid");
    return false;
  }
  return search_one(__FUNCTION__, index, q.data(), size, epsilon, radius, -1, results, error);
}

bool ngt_search_index_as_float(NGTIndex index, float* query, int32_t query_dim, size_t size, float epsilon,
                               float radius, NGTObjectDistances results, NGTError error) {
  if (index == NULL || query == NULL || results == NULL || query_dim <= 0) {
    std::stringstream ss;
    ss << "index = " << index << " query = " << query << " results = " << results << " query_dim = " << query_dim;
    param_error(error, __FUNCTION__, ss.str());
    return false;
  }
  std::vector<float> q;
  if (!query_of(static_cast<CapiIndex*>(index), query, query_dim, q)) {
    set_error(error, __FUNCTION__, "the specified dimension is invalid");
    return false;
  }
  return search_one(__FUNCTION__, index, q.data(), size, epsilon, radius, -1, results, error);
}

bool ngt_search_index_with_query(NGTIndex index, NGTQuery query, NGTObjectDistances results, NGTError error) {
  if (index == NULL || query.query == NULL || results == NULL) {
    std::stringstream ss;
    ss << "index = " << index << " query = " << query.query << " results = " << results;
    param_error(error, __FUNCTION__, ss.str());
    return false;
  }
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  std::vector<float> q;
  query_of(ix, query.query, ix->host.prop.dimension, q);  // NGTQuery carries no dimension: the index's
  return search_one(__FUNCTION__, index, q.data(), query.size, query.epsilon, query.radius,
                    (int64_t)(int)query.edge_size, results, error);
}

static bool linear_one(const char* func, NGTIndex index, const float* q, size_t size,
                       NGTObjectDistances results, NGTError error) {
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  std::vector<uint32_t> ids;
  std::vector<float> dists;
  uint32_t n = 0;
  std::string e = single_query(ix, kLinearSearch, q, size, 0.f, FLT_MAX, 0, 0, ids, dists, n);
  if (!e.empty()) {
    set_error(error, func, e);
    return false;
  }
  fill_results(results, ids, dists, n);
  return true;
}

bool ngt_linear_search_index(NGTIndex index, double* query, int32_t query_dim, size_t size,
                             NGTObjectDistances results, NGTError error) {
  if (index == NULL || query == NULL || results == NULL || query_dim <= 0) {
    std::stringstream ss;
    ss << "index = " << index << " query = " << query << " results = " << results << " query_dim = " << query_dim;
    param_error(error, __FUNCTION__, ss.str());
    return false;
  }
  std::vector<float> qf(query, query + query_dim), q;
  if (!query_of(static_cast<CapiIndex*>(index), qf.data(), query_dim, q)) {
    set_error(error, __FUNCTION__, "the specified dimension is invalid");
    return false;
  }
  return linear_one(__FUNCTION__, index, q.data(), size, results, error);
}

bool ngt_linear_search_index_as_float(NGTIndex index, float* query, int32_t query_dim, size_t size,
                                      NGTObjectDistances results, NGTError error) {
  if (index == NULL || query == NULL || results == NULL || query_dim <= 0) {
    std::stringstream ss;
    ss << "index = " << index << " query = " << query << " results = " << results << " query_dim = " << query_dim;
    param_error(error, __FUNCTION__, ss.str());
    return false;
  }
  std::vector<float> q;
  if (!query_of(static_cast<CapiIndex*>(index), query, query_dim, q)) {
    set_error(error, __FUNCTION__, "the specified dimension is invalid");
    return false;
  }
  return linear_one(__FUNCTION__, index, q.data(), size, results, error);
}

bool ngt_linear_search_index_with_query(NGTIndex index, NGTQuery query, NGTObjectDistances results,
                                        NGTError error) {
  if (index == NULL || query.query == NULL || results == NULL) {
    std::stringstream ss;
    ss << "index = " << index << " query = " << query.query << " results = " << results;
    param_error(error, __FUNCTION__, ss.str());
    return false;
  }
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  std::vector<float> q;
  query_of(ix, query.query, ix->host.prop.dimension, q);
  return linear_one(__FUNCTION__, index, q.data(), query.size, results, error);
}

int32_t ngt_get_size(NGTObjectDistances results, NGTError error) {
  if (results == NULL) {
    param_error(error, __FUNCTION__, "results = 0");
    return -1;
  }
  return (int32_t) static_cast<Results*>(results)->size();
}

uint32_t ngt_get_result_size(NGTObjectDistances results, NGTError error) {
  if (results == NULL) {
    param_error(error, __FUNCTION__, "results = 0");
    return 0;
  }
  return (uint32_t) static_cast<Results*>(results)->size();
}

NGTObjectDistance ngt_get_result(const NGTObjectDistances results, const uint32_t i, NGTError error) {
  Results* r = static_cast<Results*>(results);
  if (r == NULL || i >= r->size()) {
    set_error(error, __FUNCTION__, "index out of range");
    NGTObjectDistance err_val = {0, 0.0f};
    return err_val;
  }
  return (*r)[i];
}

ObjectID ngt_insert_index(NGTIndex index, double* obj, uint32_t obj_dim, NGTError error) {
  if (index == NULL || obj == NULL || obj_dim == 0) {
    param_error(error, __FUNCTION__, "index or obj is null");
    return 0;
  }
  uint32_t id = 0;
  std::string e = append_object(static_cast<CapiIndex*>(index), obj, obj_dim, id);
  if (!e.empty()) {
    set_error(error, __FUNCTION__, e);
    return 0;
  }
  return id;
}
ObjectID ngt_append_index(NGTIndex index, double* obj, uint32_t obj_dim, NGTError error) {
  return ngt_insert_index(index, obj, obj_dim, error);
}
ObjectID ngt_insert_index_as_float(NGTIndex index, float* obj, uint32_t obj_dim, NGTError error) {
  if (index == NULL || obj == NULL || obj_dim == 0) {
    param_error(error, __FUNCTION__, "index or obj is null");
    return 0;
  }
  uint32_t id = 0;
  std::string e = append_object(static_cast<CapiIndex*>(index), obj, obj_dim, id);
  if (!e.empty()) {
    set_error(error, __FUNCTION__, e);
    return 0;
  }
  return id;
}
ObjectID ngt_append_index_as_float(NGTIndex index, float* obj, uint32_t obj_dim, NGTError error) {
  return ngt_insert_index_as_float(index, obj, obj_dim, error);
}
bool ngt_batch_append_index(NGTIndex index, float* obj, uint32_t data_count, NGTError error) {
  if (index == NULL || obj == NULL) {
    param_error(error, __FUNCTION__, "index or obj is null");
    return false;
  }
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  uint32_t dim = (uint32_t)ix->host.prop.object_dimension(), id;
  for (uint32_t i = 0; i < data_count; i++) {
    std::string e = append_object(ix, obj + (size_t)i * dim, dim, id);
    if (!e.empty()) {
      set_error(error, __FUNCTION__, e);
      return false;
    }
  }
  return true;
}
bool ngt_batch_insert_index(NGTIndex index, float* obj, uint32_t num_obj, uint32_t* obj_ids, NGTError error) {
  if (!ngt_batch_append_index(index, obj, num_obj, error)) return false;
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  if (obj_ids)
    for (uint32_t i = 0; i < num_obj; i++) obj_ids[i] = (uint32_t)(ix->host.nrows - num_obj + i);
  return ngt_create_index(index, 0, error);
}
bool ngt_create_index(NGTIndex index, uint32_t pool_size, NGTError error) {
  // NGT::Index::createIndex(threadPoolSize) -> GraphAndTreeIndex::createIndex
  // (Index.cpp:1158-1257), built on the device (ngt_amd_build_*, build.cpp).
  // pool_size only sets the reference's host thread count: the result does
  // not depend on it.
  (void)pool_size;
  if (index == NULL) {
    param_error(error, __FUNCTION__, "index = 0");
    return false;
  }
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  HostIndex& h = ix->host;
  std::string e = build_anng(ix);
  if (!e.empty()) {
    set_error(error, __FUNCTION__, e);
    return false;
  }
  (void)h;
  return true;
}
bool ngt_remove_index(NGTIndex index, ObjectID id, NGTError error) {
  (void)id;
  if (index == NULL) {
    param_error(error, __FUNCTION__, "index = 0");
    return false;
  }
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}

NGTObjectSpace ngt_get_object_space(NGTIndex index, NGTError error) {
  if (index == NULL) {
    param_error(error, __FUNCTION__, "index = 0");
    return NULL;
  }
  return static_cast<NGTObjectSpace>(index);
}

float* ngt_get_object_as_float(NGTObjectSpace object_space, ObjectID id, NGTError error) {
  CapiIndex* ix = static_cast<CapiIndex*>(object_space);
  if (ix == NULL) {
    param_error(error, __FUNCTION__, "object_space = 0");
    return NULL;
  }
  HostIndex& h = ix->host;
  if (id == 0 || id >= h.nrows || !h.valid[id]) {
    std::stringstream ss;
    ss << "NGT::ObjectSpaceRepository: The specified ID is out of the range. The object ID should be greater than zero. "
       << id << ":" << h.nrows << ".";
    set_error(error, __FUNCTION__, ss.str());
    return NULL;
  }
  if (h.prop.object_type != 2) {
    set_error(error, __FUNCTION__, "the object type is not float");
    return NULL;
  }
  return reinterpret_cast<float*>(h.rows.data() + (size_t)id * h.row_bytes);
}

uint8_t* ngt_get_object_as_integer(NGTObjectSpace object_space, ObjectID id, NGTError error) {
  CapiIndex* ix = static_cast<CapiIndex*>(object_space);
  if (ix == NULL) {
    param_error(error, __FUNCTION__, "object_space = 0");
    return NULL;
  }
  HostIndex& h = ix->host;
  if (id == 0 || id >= h.nrows || !h.valid[id]) {
    set_error(error, __FUNCTION__, "the specified ID is out of the range");
    return NULL;
  }
  if (h.prop.object_type != 1) {
    set_error(error, __FUNCTION__, "the object type is not integer");
    return NULL;
  }
  return h.rows.data() + (size_t)id * h.row_bytes;
}

void ngt_destroy_results(NGTObjectDistances results) { delete static_cast<Results*>(results); }
void ngt_destroy_property(NGTProperty prop) { delete prop_of(prop); }
void ngt_close_index(NGTIndex index) { delete static_cast<CapiIndex*>(index); }

NGTError ngt_create_error_object() {
  try {
    return static_cast<NGTError>(new std::string());
  } catch (std::exception& err) {
    std::cerr << "Capi : " << __FUNCTION__ << "() : Error: " << err.what();
    return NULL;
  }
}
const char* ngt_get_error_string(const NGTError error) {
  return static_cast<std::string*>(error)->c_str();
}
void ngt_clear_error_string(NGTError error) { *static_cast<std::string*>(error) = ""; }
void ngt_destroy_error_object(NGTError error) { delete static_cast<std::string*>(error); }

NGTOptimizer ngt_create_optimizer(bool, NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return NULL;
}
bool ngt_optimizer_adjust_search_coefficients(NGTOptimizer, const char*, NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}
bool ngt_optimizer_execute(NGTOptimizer, const char*, const char*, NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}
bool ngt_optimizer_set(NGTOptimizer, int, int, int, float, float, float, float, double, double,
                       NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}
bool ngt_optimizer_set_minimum(NGTOptimizer, int, int, int, int, NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}
bool ngt_optimizer_set_extension(NGTOptimizer, float, float, float, float, double, double, NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}
bool ngt_optimizer_set_processing_modes(NGTOptimizer, bool, bool, bool, NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}
void ngt_destroy_optimizer(NGTOptimizer) {}
bool ngt_refine_anng(NGTIndex, float, float, int, int, size_t, NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}

bool ngt_get_edges(NGTIndex index, ObjectID id, NGTObjectDistances edges, NGTError error) {
  if (index == NULL || edges == NULL) {
    param_error(error, __FUNCTION__, "index or edges is null");
    return false;
  }
  HostIndex& h = static_cast<CapiIndex*>(index)->host;
  if (id == 0 || id >= h.nrows) {
    set_error(error, __FUNCTION__, "the specified ID is out of the range");
    return false;
  }
  Results* r = static_cast<Results*>(edges);
  r->clear();
  for (uint64_t j = h.edge_off[id]; j < h.edge_off[id + 1]; j++)
    r->push_back(NGTObjectDistance{h.edges[j], j < h.edge_dists.size() ? h.edge_dists[j] : 0.f});
  return true;
}

uint32_t ngt_get_object_repository_size(NGTIndex index, NGTError error) {
  if (index == NULL) {
    param_error(error, __FUNCTION__, "index = 0");
    return 0;
  }
  return (uint32_t) static_cast<CapiIndex*>(index)->host.nrows;
}

NGTAnngEdgeOptimizationParameter ngt_get_anng_edge_optimization_parameter() {
  NGTAnngEdgeOptimizationParameter p;
  p.no_of_queries = 200;
  p.no_of_results = 50;
  p.no_of_threads = 16;
  p.target_accuracy = 0.9f;
  p.target_no_of_objects = 0;
  p.no_of_sample_objects = 100000;
  p.max_of_no_of_edges = 100;
  p.log = false;
  return p;
}
bool ngt_optimize_number_of_edges(const char*, NGTAnngEdgeOptimizationParameter, NGTError error) {
  set_error(error, __FUNCTION__, kNotImplemented);
  return false;
}

// ---- extensions --------------------------------------------------------------
static bool batch_search(const char* func, NGTIndex index, const float* queries, uint32_t nq, int32_t dim,
                         size_t size, float epsilon, float radius, int64_t edge_size, int seed_mode,
                         uint32_t* ids, float* dists, uint32_t* n, NGTError error) {
  if (index == NULL || queries == NULL || ids == NULL || dists == NULL || n == NULL) {
    param_error(error, func, "null argument");
    return false;
  }
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  if (dim != ix->host.prop.object_dimension()) {  // batches are [nq][object dimension]
    set_error(error, func, "the specified dimension is invalid");
    return false;
  }
  std::vector<uint32_t> vi, vn;
  std::vector<float> vd;
  std::string e = run_search(ix, queries, nq, size, epsilon, radius, edge_size, seed_mode, vi, vd, vn);
  if (!e.empty()) {
    set_error(error, func, e);
    return false;
  }
  memcpy(ids, vi.data(), vi.size() * sizeof(uint32_t));
  memcpy(dists, vd.data(), vd.size() * sizeof(float));
  memcpy(n, vn.data(), vn.size() * sizeof(uint32_t));
  return true;
}

bool ngt_batch_search_index(NGTIndex index, const float* queries, uint32_t nq, int32_t dim, size_t size,
                            float epsilon, float radius, int64_t edge_size, uint32_t* ids, float* dists,
                            uint32_t* n, NGTError error) {
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  int mode = ix && use_tree(ix) ? NGT_AMD_SEED_TREE : NGT_AMD_SEED_RANDOM;
  return batch_search(__FUNCTION__, index, queries, nq, dim, size, epsilon, radius, edge_size, mode, ids,
                      dists, n, error);
}

bool ngt_batch_search_index_using_only_graph(NGTIndex index, const float* queries, uint32_t nq, int32_t dim,
                                             size_t size, float epsilon, float radius, int64_t edge_size,
                                             uint32_t* ids, float* dists, uint32_t* n, NGTError error) {
  return batch_search(__FUNCTION__, index, queries, nq, dim, size, epsilon, radius, edge_size,
                      NGT_AMD_SEED_RANDOM, ids, dists, n, error);
}

bool ngt_batch_linear_search_index(NGTIndex index, const float* queries, uint32_t nq, int32_t dim, size_t size,
                                   uint32_t* ids, float* dists, uint32_t* n, NGTError error) {
  return ngt_batch_linear_search_index_with_radius(index, queries, nq, dim, size, FLT_MAX, ids, dists, n, error);
}

bool ngt_batch_linear_search_index_with_radius(NGTIndex index, const float* queries, uint32_t nq, int32_t dim,
                                               size_t size, float radius, uint32_t* ids, float* dists, uint32_t* n,
                                               NGTError error) {
  if (index == NULL || queries == NULL || ids == NULL || dists == NULL || n == NULL) {
    param_error(error, __FUNCTION__, "null argument");
    return false;
  }
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  if (dim != ix->host.prop.object_dimension()) {
    set_error(error, __FUNCTION__, "the specified dimension is invalid");
    return false;
  }
  std::vector<uint32_t> vi, vn;
  std::vector<float> vd;
  std::string e = run_linear(ix, queries, nq, size, vi, vd, vn, radius < 0.0f ? -1.0 : (double)radius);
  if (!e.empty()) {
    set_error(error, __FUNCTION__, e);
    return false;
  }
  memcpy(ids, vi.data(), vi.size() * sizeof(uint32_t));
  memcpy(dists, vd.data(), vd.size() * sizeof(float));
  memcpy(n, vn.data(), vn.size() * sizeof(uint32_t));
  return true;
}

bool ngt_get_last_search_counters(NGTIndex index, uint64_t* counters3, NGTError error) {
  if (index == NULL || counters3 == NULL) {
    param_error(error, __FUNCTION__, "null argument");
    return false;
  }
  memcpy(counters3, t_last_counters, 3 * sizeof(uint64_t));
  return true;
}

bool ngt_set_property_value(NGTProperty prop, const char* key, const char* value, NGTError error) {
  if (prop == NULL || key == NULL || value == NULL) {
    param_error(error, __FUNCTION__, "null argument");
    return false;
  }
  HostProperty* p = prop_of(prop);
  p->to_kv();
  p->kv[key] = value;
  p->from_kv();
  return true;
}

int32_t ngt_get_property_value(NGTProperty prop, const char* key, char* buf, size_t len, NGTError error) {
  if (prop == NULL || key == NULL) {
    param_error(error, __FUNCTION__, "null argument");
    return -1;
  }
  HostProperty* p = prop_of(prop);
  p->to_kv();
  auto it = p->kv.find(key);
  if (it == p->kv.end()) {
    set_error(error, __FUNCTION__, std::string("no property ") + key);
    return -1;
  }
  if (buf && len) {
    strncpy(buf, it->second.c_str(), len - 1);
    buf[len - 1] = 0;
  }
  return (int32_t)it->second.size();
}

bool ngt_get_coalesce_stats(NGTIndex index, uint64_t* batches, uint64_t* served, NGTError error) {
  if (index == NULL || batches == NULL || served == NULL) {
    param_error(error, __FUNCTION__, "null argument");
    return false;
  }
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  coalescer_of(ix)->stats(batches, served);
  // calls the resident serving grid answered count as served, its launches as batches
  uint64_t s = 0, l = 0;
  if (ix->dev && ngt_amd_serve_stats(ix->dev, &s, &l) == 0) {
    *batches += l;
    *served += s;
  }
  return true;
}

void* ngt_get_device_index(NGTIndex index, NGTError error) {
  if (index == NULL) {
    param_error(error, __FUNCTION__, "null index");
    return NULL;
  }
  CapiIndex* ix = static_cast<CapiIndex*>(index);
  std::shared_lock<std::shared_mutex> rd;
  std::string e = sync_device(ix, rd);
  if (!e.empty()) {
    set_error(error, __FUNCTION__, e);
    return NULL;
  }
  return ix->dev;
}

}  // extern "C"
