// index_io.h -- NGT 1.13.8 on-disk index formats, read straight into the
// layouts the device path uses (padded row-major object slab, CSR adjacency,
// flattened DVP tree).  Formats:
//   prf : tab-separated PropertySet (lib/NGT/Common.h:573-666, Index.h:105-261,
//         Graph.h:423-489)
//   obj : Repository<Object>::serialize (Common.h:1776-1793) -- size_t n, then
//         per slot '-' | '+' + dim*sizeof(T) bytes (ObjectSpace.h:297-301)
//   grp : GraphRepository::serialize (Graph.h:151-154) -- node repository of
//         {uint32 n, n x packed {uint32 id, float distance}} + prevsize vector
//   tre : DVPTree::serialize (Tree.h:344-347) -- leaf then internal repositories
//         (Node.h:90-99, 224-251, 451-480)
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

namespace ngt_amd {

struct HostProperty {
  std::map<std::string, std::string> kv;
  int32_t dimension = 0;
  int32_t object_type = 2;        // 1 Uint8 ("Integer-1"), 2 Float ("Float-4")
  int32_t distance_type = 1;      // ObjectSpace::DistanceType
  int32_t edge_size_for_creation = 10;
  int32_t edge_size_for_search = 40;
  int32_t dynamic_edge_size_base = 30;
  int32_t dynamic_edge_size_rate = 20;
  int32_t seed_size = 10;
  int32_t seed_type = 0;          // SeedTypeNone
  int32_t graph_type = 1;         // ANNG
  int32_t index_type = 0;         // 0 GraphAndTree, 1 Graph
  double epsilon_for_creation = 0.1;
  int32_t batch_size_for_creation = 200;
  int32_t prefetch_offset = 0, prefetch_size = 0;
  void set_defaults();            // NGT::Property defaults (Index.h:45-104, Graph.h:386-402)
  // the object space's dimension: SparseJaccard keeps one more slot for the
  // 0 terminator (GraphIndex::constructObjectSpace, Index.cpp:484-490)
  int32_t object_dimension() const { return dimension + (distance_type == 8 ? 1 : 0); }
  void from_kv();
  void to_kv();
};

struct HostTree {
  bool present = false;
  uint32_t root = 0;
  uint32_t children = 5;
  std::vector<uint8_t> in_pivot;      // [n_internal][row_bytes]
  std::vector<uint32_t> in_child;     // [n_internal][children]
  std::vector<float> in_border;       // [n_internal][children-1]
  std::vector<uint8_t> in_valid;
  std::vector<uint64_t> leaf_off;     // [n_leaf+1]
  std::vector<uint32_t> leaf_ids;
  std::vector<float> leaf_dists;      // ObjectDistance::distance stored with the ids
  std::vector<uint8_t> leaf_valid;
  std::vector<uint32_t> leaf_parent;  // raw parent ids (for save)
  std::vector<uint8_t> leaf_pivot;    // [n_leaf][row_bytes]
  std::vector<uint8_t> leaf_has_pivot;
  std::vector<uint32_t> in_parent;
  uint32_t n_internal() const { return (uint32_t)in_valid.size(); }
  uint32_t n_leaf() const { return (uint32_t)leaf_valid.size(); }
};

struct HostIndex {
  HostProperty prop;
  uint32_t dp = 0;                    // padded dimension
  uint32_t esize = 4;
  uint64_t row_bytes = 0;
  uint64_t nrows = 0;                 // repository size incl. dummy slot 0
  std::vector<uint8_t> rows;          // [nrows][row_bytes], zero padded
  std::vector<uint8_t> valid;         // [nrows]
  std::vector<uint64_t> edge_off;     // [nrows+1]
  std::vector<uint32_t> edges;
  std::vector<float> edge_dists;
  std::vector<uint16_t> prevsize;
  HostTree tree;
  void init_layout();
};

// NGTQG quantizer of <index>/qg (NGTQ::Index, lib/NGT/NGTQ/Quantizer.h) and,
// when saved, its quantized graph qg/grp (QuantizedGraph.h:117-150).
struct HostQuantizer {
  uint32_t dim = 0, M = 0, dsub = 0;
  std::vector<float> global;          // [dim] global centroid 1
  std::vector<float> local;           // [M][16][dsub] local centroids 1..16
  std::vector<uint8_t> codes;         // [nrows][M] localID - 1 (qg/ivt)
  bool has_grp = false;
  std::vector<uint64_t> qoff, code_off;
  std::vector<uint32_t> qids;
  std::vector<uint8_t> qcodes;
};

// All return an empty string on success, else an error message.
std::string read_prf(const std::string& path, HostProperty& p);
std::string write_prf(const std::string& path, HostProperty& p);
std::string load_index(const std::string& dir, HostIndex& ix);
std::string save_index(const std::string& dir, HostIndex& ix);
std::string load_qg(const std::string& dir, uint64_t nrows, HostQuantizer& q);

}  // namespace ngt_amd
