// index_io.cpp -- NGT 1.13.8 index files <-> host staging of the HBM layouts.
// See index_io.h for the format citations.
#include "index_io.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <fstream>
#include <sstream>

namespace ngt_amd {

namespace {

const char* kDistanceNames[][2] = {
    {"L1", "0"}, {"L2", "1"}, {"Hamming", "2"}, {"Angle", "3"}, {"Cosine", "4"},
    {"NormalizedAngle", "5"}, {"NormalizedCosine", "6"}, {"Jaccard", "7"},
    {"SparseJaccard", "8"}, {"NormalizedL2", "9"}, {"Poincare", "100"}, {"Lorentz", "101"}};

const char* kSeedTypes[] = {"None", "RandomNodes", "FixedNodes", "FirstNode", "AllLeafNodes"};
const char* kGraphTypes[] = {"None", "ANNG", "KNNG", "BKNNG", "ONNG", "IANNG", "DNNG"};

long getl(const std::map<std::string, std::string>& kv, const char* k, long dflt) {
  auto it = kv.find(k);
  if (it == kv.end() || it->second.empty()) return dflt;
  return strtol(it->second.c_str(), nullptr, 10);
}
double getf(const std::map<std::string, std::string>& kv, const char* k, double dflt) {
  auto it = kv.find(k);
  if (it == kv.end() || it->second.empty()) return dflt;
  return strtod(it->second.c_str(), nullptr);
}

struct Reader {
  std::vector<char> buf;
  size_t off = 0;
  bool ok = true;
  bool open(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    f.seekg(0, std::ios::end);
    buf.resize((size_t)f.tellg());
    f.seekg(0);
    f.read(buf.data(), (std::streamsize)buf.size());
    return (bool)f;
  }
  template <typename T>
  T get() {
    T v{};
    if (off + sizeof(T) > buf.size()) {
      ok = false;
      return v;
    }
    memcpy(&v, buf.data() + off, sizeof(T));
    off += sizeof(T);
    return v;
  }
  bool bytes(void* dst, size_t n) {
    if (off + n > buf.size()) return ok = false;
    memcpy(dst, buf.data() + off, n);
    off += n;
    return true;
  }
  bool skip(size_t n) {
    if (off + n > buf.size()) return ok = false;
    off += n;
    return true;
  }
};

struct Writer {
  std::ofstream f;
  explicit Writer(const std::string& p) : f(p, std::ios::binary) {}
  template <typename T>
  void put(const T& v) { f.write(reinterpret_cast<const char*>(&v), sizeof(T)); }
  void bytes(const void* p, size_t n) { f.write(static_cast<const char*>(p), (std::streamsize)n); }
};

}  // namespace

void HostProperty::set_defaults() {
  kv.clear();
  dimension = 0;
  object_type = 2;
  distance_type = 1;
  index_type = 0;
  edge_size_for_creation = 10;   // NGT_CREATION_EDGE_SIZE (defines.h.in:32)
  edge_size_for_search = 0;      // Graph.h:389
  dynamic_edge_size_base = 30;   // Graph.h:397
  dynamic_edge_size_rate = 20;   // Graph.h:398
  seed_size = 10;                // NGT_SEED_SIZE
  seed_type = 0;
  graph_type = 1;
  epsilon_for_creation = 0.1;
  batch_size_for_creation = 200;
  prefetch_offset = prefetch_size = 0;
}

void HostProperty::from_kv() {
  dimension = (int32_t)getl(kv, "Dimension", 0);
  auto it = kv.find("ObjectType");
  if (it != kv.end()) object_type = it->second == "Integer-1" ? 1 : 2;
  it = kv.find("DistanceType");
  if (it != kv.end())
    for (auto& d : kDistanceNames)
      if (it->second == d[0]) distance_type = atoi(d[1]);
  it = kv.find("IndexType");
  if (it != kv.end()) index_type = it->second == "Graph" ? 1 : 0;
  edge_size_for_creation = (int32_t)getl(kv, "EdgeSizeForCreation", edge_size_for_creation);
  edge_size_for_search = (int32_t)getl(kv, "EdgeSizeForSearch", edge_size_for_search);
  dynamic_edge_size_base = (int32_t)getl(kv, "DynamicEdgeSizeBase", dynamic_edge_size_base);
  dynamic_edge_size_rate = (int32_t)getl(kv, "DynamicEdgeSizeRate", dynamic_edge_size_rate);
  seed_size = (int32_t)getl(kv, "SeedSize", seed_size);
  batch_size_for_creation = (int32_t)getl(kv, "BatchSizeForCreation", batch_size_for_creation);
  epsilon_for_creation = getf(kv, "EpsilonForCreation", epsilon_for_creation);
  prefetch_offset = (int32_t)getl(kv, "PrefetchOffset", 0);
  prefetch_size = (int32_t)getl(kv, "PrefetchSize", 0);
  it = kv.find("SeedType");
  if (it != kv.end())
    for (int i = 0; i < 5; i++)
      if (it->second == kSeedTypes[i]) seed_type = i;
  it = kv.find("GraphType");
  if (it != kv.end())
    for (int i = 0; i < 7; i++)
      if (it->second == kGraphTypes[i]) graph_type = i;
}

void HostProperty::to_kv() {
  kv["Dimension"] = std::to_string(dimension);
  kv["ObjectType"] = object_type == 1 ? "Integer-1" : "Float-4";
  for (auto& d : kDistanceNames)
    if (atoi(d[1]) == distance_type) kv["DistanceType"] = d[0];
  kv["IndexType"] = index_type == 1 ? "Graph" : "GraphAndTree";
  if (!kv.count("DatabaseType")) kv["DatabaseType"] = "Memory";
  if (!kv.count("ObjectAlignment")) kv["ObjectAlignment"] = "False";
  kv["EdgeSizeForCreation"] = std::to_string(edge_size_for_creation);
  kv["EdgeSizeForSearch"] = std::to_string(edge_size_for_search);
  kv["DynamicEdgeSizeBase"] = std::to_string(dynamic_edge_size_base);
  kv["DynamicEdgeSizeRate"] = std::to_string(dynamic_edge_size_rate);
  kv["SeedSize"] = std::to_string(seed_size);
  kv["SeedType"] = kSeedTypes[seed_type >= 0 && seed_type < 5 ? seed_type : 0];
  kv["GraphType"] = kGraphTypes[graph_type >= 0 && graph_type < 7 ? graph_type : 1];
  kv["BatchSizeForCreation"] = std::to_string(batch_size_for_creation);
  {
    std::ostringstream os;
    os << epsilon_for_creation;
    kv["EpsilonForCreation"] = os.str();
  }
  // 0 = the object space's runtime values, which save() exports
  // (ObjectSpace::setPrefetchOffset/Size, lib/NGT/ObjectSpace.h:268-283)
  const int pdim = ((dimension - 1) / 16 + 1) * 16;
  kv["PrefetchOffset"] = std::to_string(prefetch_offset ? prefetch_offset
                                                        : (int)floor(300.0 / ((float)pdim + 30.0) + 1.0));
  kv["PrefetchSize"] = std::to_string(prefetch_size ? prefetch_size : dimension * (object_type == 1 ? 1 : 4));
  // keys a fresh NGT::Property writes (Index.h:60-75, 150-170; Graph.h:386-402, 430-450)
  static const char* kMore[][2] = {{"AccuracyTable", ""},
                                   {"BuildTimeLimit", "0"},
                                   {"EdgeSizeLimitForCreation", "5"},
                                   {"IncomingEdge", "80"},
                                   {"IncrimentalEdgeSizeLimitForTruncation", "0"},
                                   {"OutgoingEdge", "10"},
                                   {"PathAdjustmentInterval", "0"},
                                   {"ThreadPoolSize", "32"},
                                   {"TruncationThreadPoolSize", "8"}};
  for (auto& m : kMore)
    if (!kv.count(m[0])) kv[m[0]] = m[1];
}

void HostIndex::init_layout() {
  dp = (uint32_t)(((prop.object_dimension() - 1) / 16 + 1) * 16);
  esize = prop.object_type == 1 ? 1 : 4;
  row_bytes = (uint64_t)dp * esize;
}

std::string read_prf(const std::string& path, HostProperty& p) {
  std::ifstream f(path);
  if (!f) return "cannot open " + path;
  p.set_defaults();
  std::string line;
  while (std::getline(f, line)) {
    size_t t = line.find('\t');
    if (t == std::string::npos) continue;
    p.kv[line.substr(0, t)] = line.substr(t + 1);
  }
  p.from_kv();
  if (p.dimension <= 0) return "invalid Dimension in " + path;
  return "";
}

std::string write_prf(const std::string& path, HostProperty& p) {
  p.to_kv();
  std::ofstream f(path);
  if (!f) return "cannot write " + path;
  for (auto& kv : p.kv) f << kv.first << "\t" << kv.second << "\n";
  return "";
}

std::string load_index(const std::string& dir, HostIndex& ix) {
  std::string e = read_prf(dir + "/prf", ix.prop);
  if (!e.empty()) return e;
  ix.init_layout();
  const size_t obytes = (size_t)ix.prop.object_dimension() * ix.esize;
  // ---- obj
  {
    Reader r;
    if (!r.open(dir + "/obj")) return "cannot open " + dir + "/obj";
    uint64_t n = r.get<uint64_t>();
    ix.nrows = n;
    ix.rows.assign(n * ix.row_bytes, 0);
    ix.valid.assign(n, 0);
    for (uint64_t i = 0; i < n && r.ok; i++) {
      char t = r.get<char>();
      if (t == '+') {
        r.bytes(ix.rows.data() + i * ix.row_bytes, obytes);
        ix.valid[i] = 1;
      } else if (t != '-') {
        return "corrupt obj file";
      }
    }
    if (!r.ok) return "truncated obj file";
  }
  // ---- grp
  {
    Reader r;
    if (!r.open(dir + "/grp")) return "cannot open " + dir + "/grp";
    uint64_t n = r.get<uint64_t>();
    if (n > ix.nrows) {
      // graph may be larger if objects were removed at the tail; pad objects
      ix.rows.resize(n * ix.row_bytes, 0);
      ix.valid.resize(n, 0);
      ix.nrows = n;
    }
    ix.edge_off.assign(ix.nrows + 1, 0);
    ix.edges.clear();
    ix.edge_dists.clear();
    for (uint64_t i = 0; i < n && r.ok; i++) {
      char t = r.get<char>();
      if (t == '+') {
        uint32_t cnt = r.get<uint32_t>();
        for (uint32_t j = 0; j < cnt && r.ok; j++) {
          uint32_t id = r.get<uint32_t>();
          float d = r.get<float>();
          ix.edges.push_back(id);
          ix.edge_dists.push_back(d);
        }
      } else if (t != '-') {
        return "corrupt grp file";
      }
      ix.edge_off[i + 1] = ix.edges.size();
    }
    for (uint64_t i = n; i < ix.nrows; i++) ix.edge_off[i + 1] = ix.edges.size();
    uint32_t ps = r.get<uint32_t>();
    ix.prevsize.resize(ps);
    for (uint32_t i = 0; i < ps && r.ok; i++) ix.prevsize[i] = r.get<uint16_t>();
    if (!r.ok) return "truncated grp file";
  }
  // ---- tre (GraphAndTree indexes)
  ix.tree = HostTree();
  {
    Reader r;
    if (r.open(dir + "/tre")) {
      HostTree& t = ix.tree;
      uint64_t nl = r.get<uint64_t>();
      t.leaf_off.assign(nl + 1, 0);
      t.leaf_valid.assign(nl, 0);
      t.leaf_parent.assign(nl, 0);
      t.leaf_pivot.assign(nl * ix.row_bytes, 0);
      t.leaf_has_pivot.assign(nl, 0);
      for (uint64_t i = 0; i < nl && r.ok; i++) {
        char c = r.get<char>();
        if (c == '+') {
          (void)r.get<uint32_t>();  // id
          uint32_t parent = r.get<uint32_t>();
          uint16_t cnt = r.get<uint16_t>();
          for (uint16_t j = 0; j < cnt; j++) {
            t.leaf_ids.push_back(r.get<uint32_t>());
            t.leaf_dists.push_back(r.get<float>());
          }
          t.leaf_parent[i] = parent;
          if (!((parent & 0x7fffffffu) == 0 && cnt == 0)) {
            r.bytes(t.leaf_pivot.data() + i * ix.row_bytes, obytes);
            t.leaf_has_pivot[i] = 1;
          }
          t.leaf_valid[i] = 1;
        } else if (c != '-') {
          return "corrupt tre file (leaf)";
        }
        t.leaf_off[i + 1] = t.leaf_ids.size();
      }
      uint64_t ni = r.get<uint64_t>();
      t.in_valid.assign(ni, 0);
      t.in_parent.assign(ni, 0);
      t.in_pivot.assign(ni * ix.row_bytes, 0);
      t.in_child.assign(ni * 5, 0);
      t.in_border.assign(ni * 4, 0.f);
      for (uint64_t i = 0; i < ni && r.ok; i++) {
        char c = r.get<char>();
        if (c == '+') {
          (void)r.get<uint32_t>();
          t.in_parent[i] = r.get<uint32_t>();
          r.bytes(t.in_pivot.data() + i * ix.row_bytes, obytes);
          uint64_t cs = r.get<uint64_t>();
          if (cs != 5) return "unsupported DVP tree fan-out";
          for (int j = 0; j < 5; j++) t.in_child[i * 5 + j] = r.get<uint32_t>();
          for (int j = 0; j < 4; j++) t.in_border[i * 4 + j] = r.get<float>();
          t.in_valid[i] = 1;
        } else if (c != '-') {
          return "corrupt tre file (internal)";
        }
      }
      if (!r.ok) return "truncated tre file";
      // DVPTree::getRootNode (Tree.h:219-235)
      t.root = (ni > 1 && t.in_valid[1]) ? 1u : 0x80000001u;
      t.present = nl > 1;
    }
  }
  return "";
}

std::string save_index(const std::string& dir, HostIndex& ix) {
  std::string e = write_prf(dir + "/prf", ix.prop);
  if (!e.empty()) return e;
  const size_t obytes = (size_t)ix.prop.object_dimension() * ix.esize;
  {
    Writer w(dir + "/obj");
    if (!w.f) return "cannot write obj";
    w.put<uint64_t>(ix.nrows);
    for (uint64_t i = 0; i < ix.nrows; i++) {
      if (ix.valid[i]) {
        w.put<char>('+');
        w.bytes(ix.rows.data() + i * ix.row_bytes, obytes);
      } else {
        w.put<char>('-');
      }
    }
  }
  {
    Writer w(dir + "/grp");
    if (!w.f) return "cannot write grp";
    w.put<uint64_t>(ix.nrows);
    for (uint64_t i = 0; i < ix.nrows; i++) {
      uint64_t b = ix.edge_off[i], en = ix.edge_off[i + 1];
      if (i == 0 || (!ix.valid[i] && b == en)) {
        w.put<char>('-');
        continue;
      }
      w.put<char>('+');
      w.put<uint32_t>((uint32_t)(en - b));
      for (uint64_t j = b; j < en; j++) {
        w.put<uint32_t>(ix.edges[j]);
        w.put<float>(j < ix.edge_dists.size() ? ix.edge_dists[j] : 0.f);
      }
    }
    w.put<uint32_t>((uint32_t)ix.prevsize.size());
    for (uint16_t v : ix.prevsize) w.put<uint16_t>(v);
  }
  if (ix.tree.present) {
    HostTree& t = ix.tree;
    Writer w(dir + "/tre");
    if (!w.f) return "cannot write tre";
    w.put<uint64_t>(t.n_leaf());
    for (uint32_t i = 0; i < t.n_leaf(); i++) {
      if (!t.leaf_valid[i]) {
        w.put<char>('-');
        continue;
      }
      w.put<char>('+');
      w.put<uint32_t>(0x80000000u | i);
      w.put<uint32_t>(t.leaf_parent[i]);
      uint16_t cnt = (uint16_t)(t.leaf_off[i + 1] - t.leaf_off[i]);
      w.put<uint16_t>(cnt);
      for (uint64_t j = t.leaf_off[i]; j < t.leaf_off[i + 1]; j++) {
        w.put<uint32_t>(t.leaf_ids[j]);
        w.put<float>(t.leaf_dists[j]);
      }
      if (t.leaf_has_pivot[i]) w.bytes(t.leaf_pivot.data() + (size_t)i * ix.row_bytes, obytes);
    }
    w.put<uint64_t>(t.n_internal());
    for (uint32_t i = 0; i < t.n_internal(); i++) {
      if (!t.in_valid[i]) {
        w.put<char>('-');
        continue;
      }
      w.put<char>('+');
      w.put<uint32_t>(i);
      w.put<uint32_t>(t.in_parent[i]);
      w.bytes(t.in_pivot.data() + (size_t)i * ix.row_bytes, obytes);
      w.put<uint64_t>(5);
      for (int j = 0; j < 5; j++) w.put<uint32_t>(t.in_child[(size_t)i * 5 + j]);
      for (int j = 0; j < 4; j++) w.put<float>(t.in_border[(size_t)i * 4 + j]);
    }
  }
  return "";
}

}  // namespace ngt_amd

namespace ngt_amd {

// obj file of 32-bit float rows of `dim` elements (slot 0 = dummy).
static std::string read_float_obj(const std::string& path, uint32_t dim, std::vector<float>& rows,
                                  uint64_t& n) {
  Reader r;
  if (!r.open(path)) return "cannot open " + path;
  n = r.get<uint64_t>();
  rows.assign(n * dim, 0.f);
  for (uint64_t i = 0; i < n && r.ok; i++) {
    char t = r.get<char>();
    if (t == '+') r.bytes(rows.data() + i * dim, (size_t)dim * 4);
    else if (t != '-') return "corrupt obj file " + path;
  }
  if (!r.ok) return "truncated obj file " + path;
  return "";
}

std::string load_qg(const std::string& dir, uint64_t nrows, HostQuantizer& q) {
  const std::string qd = dir + "/qg";
  HostProperty p;
  {
    std::ifstream f(qd + "/prf");
    if (!f) return "cannot open " + qd + "/prf (not an NGTQG index: run ngtqg quantize)";
    std::string line;
    while (std::getline(f, line)) {
      size_t t = line.find('\t');
      if (t != std::string::npos) p.kv[line.substr(0, t)] = line.substr(t + 1);
    }
  }
  const long dim = getl(p.kv, "Dimension", 0), M = getl(p.kv, "LocalDivisionNo", 0);
  if (dim <= 0 || M <= 0 || dim % M != 0) return "invalid Dimension/LocalDivisionNo in " + qd + "/prf";
  if (getl(p.kv, "LocalIDByteSize", 2) != 2) return "unsupported LocalIDByteSize in " + qd + "/prf";
  q.dim = (uint32_t)dim;
  q.M = (uint32_t)M;
  q.dsub = (uint32_t)(dim / M);
  // global codebook: centroid 1 (QuantizedGraph.h:397-399 inserts the zero vector)
  {
    std::vector<float> rows;
    uint64_t n = 0;
    std::string e = read_float_obj(qd + "/global/obj", q.dim, rows, n);
    if (!e.empty()) return e;
    if (n < 2) return "empty global codebook";
    q.global.assign(rows.begin() + q.dim, rows.begin() + 2 * q.dim);
  }
  // local codebooks: local-m/obj, ids 1..16
  q.local.assign((size_t)q.M * 16 * q.dsub, 0.f);
  for (uint32_t m = 0; m < q.M; m++) {
    std::vector<float> rows;
    uint64_t n = 0;
    std::string e = read_float_obj(qd + "/local-" + std::to_string(m) + "/obj", q.dsub, rows, n);
    if (!e.empty()) return e;
    for (uint64_t c = 1; c < n && c <= 16; c++)
      std::copy(rows.begin() + c * q.dsub, rows.begin() + (c + 1) * q.dsub,
                q.local.begin() + ((size_t)m * 16 + c - 1) * q.dsub);
  }
  // ivt: Repository<InvertedIndexEntry<uint16_t>> (NGTQ/Quantizer.h:105-132) ->
  // per object the M local ids (1..16); stored as localID - 1
  q.codes.assign(nrows * q.M, 0);
  {
    Reader r;
    if (!r.open(qd + "/ivt")) return "cannot open " + qd + "/ivt";
    uint64_t n = r.get<uint64_t>();
    for (uint64_t s = 0; s < n && r.ok; s++) {
      char t = r.get<char>();
      if (t == '-') continue;
      if (t != '+') return "corrupt ivt";
      uint32_t sz = r.get<uint32_t>();
      uint16_t nids = r.get<uint16_t>();
      const size_t pad = ((size_t)(nids * 2 - 1) / 4 + 1) * 4;
      std::vector<uint16_t> lid(pad / 2);
      for (uint32_t i = 0; i < sz && r.ok; i++) {
        uint32_t id = r.get<uint32_t>();
        r.bytes(lid.data(), pad);
        if (id >= nrows) return "ivt object id out of range";
        for (uint32_t m = 0; m < q.M && m < nids; m++) {
          if (lid[m] < 1 || lid[m] > 16) return "invalid local centroid id in ivt";
          q.codes[(size_t)id * q.M + m] = (uint8_t)(lid[m] - 1);
        }
      }
    }
    if (!r.ok) return "truncated ivt";
  }
  // qg/grp, if saved (QuantizedGraphRepository::deserialize, QuantizedGraph.h:130-150)
  q.has_grp = false;
  {
    Reader r;
    if (r.open(qd + "/grp")) {
      const uint64_t Mfile = r.get<uint64_t>(), n = r.get<uint64_t>();
      if (Mfile != q.M) return "qg/grp subspace count differs from qg/prf";
      const uint64_t me = (q.M + 1) / 2 * 2;
      q.qoff.assign(n + 1, 0);
      q.code_off.assign(n + 1, 0);
      q.qids.clear();
      q.qcodes.clear();
      for (uint64_t v = 0; v < n && r.ok; v++) {
        uint32_t cnt = r.get<uint32_t>();
        for (uint32_t i = 0; i < cnt && r.ok; i++) q.qids.push_back(r.get<uint32_t>());
        const uint64_t nb = cnt == 0 ? 0 : (cnt - 1) / 16 + 1;
        const size_t bytes = (size_t)(nb * 8 * me);
        const size_t at = q.qcodes.size();
        q.qcodes.resize(at + bytes);
        r.bytes(q.qcodes.data() + at, bytes);
        q.qoff[v + 1] = q.qids.size();
        q.code_off[v + 1] = q.qcodes.size();
      }
      if (!r.ok) return "truncated qg/grp";
      q.has_grp = true;
    }
  }
  return "";
}

}  // namespace ngt_amd
