// index_internal.h -- the device-resident index object behind the C ABI of
// include/ngt_amd.h, shared by ngt_amd_api.cpp (exact path) and qg_api.cpp
// (NGTQG path).  Not part of the public boundary.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ngt_amd.h"
#include "ngt_kernels.h"

namespace ngt_amd {

int fail(const char* fmt, ...);

#define HIP_OK(expr)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return ngt_amd::fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  bool owned = true;
  ~DevBuf() { release(); }
  void release() {
    if (p && owned) (void)hipFree(p);
    p = nullptr;
    n = 0;
    owned = true;
  }
  hipError_t alloc(size_t count) {
    if (p && owned && n >= count) return hipSuccess;
    release();
    n = count;
    return hipMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T));
  }
  hipError_t upload_async(const T* h, size_t count, hipStream_t s) {
    hipError_t e = alloc(count);
    if (e != hipSuccess) return e;
    if (count) e = hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s);
    return e;
  }
  hipError_t upload(const T* h, size_t count) {
    hipError_t e = alloc(count);
    if (e != hipSuccess) return e;
    if (count) e = hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice);
    return e;
  }
};

// quantized graph of an index (NGTQG), see qg_api.cpp
struct QgState {
  bool ready = false;
  uint32_t M = 0, dsub = 0, Me = 0;
  DevBuf<float> global;     // [dim]
  DevBuf<float> local;      // [M][16][dsub]
  DevBuf<uint32_t> qids;    // [nrows][id_stride]
  DevBuf<uint8_t> qcodes;   // [nrows][code_stride]
  DevBuf<uint8_t> codes;    // [nrows][M] local codes of the last ngt_amd_qg_encode
  bool has_codes = false;
  uint32_t id_stride = 0;
  uint64_t code_stride = 0;
  bool has_graph = false;
  // the search layout (qg_pack): one record per node in id order, its code
  // blocks then 16 entries {id, key word} per block; a node's key word is
  // (record unit << 3) | (blocks - 1), so a popped key names the record and
  // its length and both load in one round trip (qg_api.cpp, qg_kernels.hip)
  DevBuf<uint8_t> recs;     // sum over nodes of blocks * (8*Me + 128) bytes, rounded to 1 << rec_shift
  DevBuf<uint32_t> qkw;     // [nrows] key word of every node (0 for the dummy)
  uint32_t rec_shift = 0;
  uint64_t rec_bytes = 0;
  bool packed = false;
};

// NGTQ IVF-ADC quantizer attached to a global-codebook index (ivf_api.cpp)
struct IvfState {
  bool ready = false;
  uint32_t N = 0, dsub = 0, lid_stride = 0;
  uint64_t nlists = 0, nentries = 0;
  uint64_t object_records = 0;   // ObjectList::size() (records incl. slot 0)
  DevBuf<float> local;           // [N][17][dsub]
  DevBuf<uint64_t> list_off;     // [nlists + 1]
  DevBuf<uint32_t> eids;         // [nentries]
  DevBuf<uint16_t> elids;        // [nentries][lid_stride]
  DevBuf<uint8_t> orows;         // [object_records][row_bytes]
};

// Scratch owned by one in-flight search launch.  One context per HIP stream
// a caller searches on, so consecutive batches on different streams run
// concurrently (the next batch's waves fill the CUs the previous batch's
// tail leaves idle) without sharing visited arrays or work counters.
struct SearchCtx {
  hipStream_t stream = nullptr;
  DevBuf<uint32_t> work, seeds, seed_count, slot_epoch;
  DevBuf<uint64_t> seed_off, spill;
  DevBuf<uint8_t> vis;           // [slots][vis_stride] visited epochs
  uint32_t slots = 0;
  uint32_t launch_slots = 0;     // workgroups (resident waves) of the last launch
  bool launch_filtered = false;  // the last graph-search launch read the filter copy
  int launch_la = -1;            // the last graph-search launch's lookahead form (-1: none)
  uint64_t vis_stride = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the search kernel
  DevBuf<uint8_t> lut;           // NGTQG: [nq][Me*16]
  DevBuf<float> scale, toff;
  DevBuf<uint64_t> partial;      // linear search: [nq][nslices][k] slice top-k
  DevBuf<uint16_t> sqh, sql;     // matrix-core scan: queries in fragment order
  DevBuf<float> shb;             // matrix-core scan: per-query filter base
  DevBuf<uint64_t> gthr;         // matrix-core scan: per-query k-th key shared by the parts
  DevBuf<uint32_t> ivf_cid, ivf_cn;  // NGTQ: global-codebook search results [nq][cbs], [nq]
  DevBuf<float> ivf_cd;
  DevBuf<int> err;               // device error flag of the launches on this stream
  // launch schedule ("probe and resume", ngt_amd_api.cpp run_search): the
  // paused queries' states, flags, predictions and the resume order; the
  // mean expansions per query of earlier launches of the same configuration
  // (a pinned copy of the device sums, read once the launch has finished)
  DevBuf<uint8_t> qstate;
  DevBuf<uint32_t> qflag, order;
  DevBuf<float> prio;
  DevBuf<unsigned long long> stat;
  unsigned long long* h_stat = nullptr;
  hipEvent_t ev_stat = nullptr;
  bool stat_pending = false;
  uint64_t stat_key = 0;
  std::vector<std::pair<uint64_t, double>> sched_mean;
  uint32_t launch_budget = 0;
  ~SearchCtx() {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (ev_stat) (void)hipEventDestroy(ev_stat);
    if (h_stat) (void)hipHostFree(h_stat);
  }
};

// Buffers of one synchronous host-API call (ngt_amd_search, _linear_search,
// _qg_search, ...): its own HIP stream, so concurrent callers run concurrent
// launches, and device/pinned buffers kept across calls, so a call costs no
// hipMalloc once warm.  Taken from and returned to the index's pool.
struct CallCtx {
  hipStream_t stream = nullptr;
  DevBuf<float> raw;             // host float queries as uploaded
  DevBuf<uint8_t> prep;          // prepared (converted, padded, normalized) rows
  DevBuf<uint32_t> ids, n, seeds;
  DevBuf<float> dists;
  DevBuf<uint64_t> cnt, seed_off;
  ~CallCtx() {
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// glibc random(3) TYPE_3 (random_r), host side: the rand() stream of a fresh
// process (srand(1)), for getRandomSeeds during construction.
struct GlibcRandHost {
  uint32_t s[31];
  int f = 3, r = 0;
  void seed(uint32_t sd) {
    int32_t word = (int32_t)(sd == 0 ? 1u : sd);
    s[0] = (uint32_t)word;
    for (int i = 1; i < 31; i++) {
      int32_t hi = word / 127773, lo = word % 127773;
      word = 16807 * lo - 2836 * hi;
      if (word < 0) word += 2147483647;
      s[i] = (uint32_t)word;
    }
    f = 3;
    r = 0;
    for (int i = 0; i < 310; i++) next();
  }
  int next() {
    s[f] += s[r];
    int res = (int)((s[f] >> 1) & 0x7fffffff);
    f = f == 30 ? 0 : f + 1;
    r = r == 30 ? 0 : r + 1;
    return res;
  }
};

// ANNG construction state (build.cpp): the graph being built (host, sorted
// edge lists), the DVP tree being built (HBM, fixed-capacity node arrays) and
// the padded search adjacency the insertion searches read (HBM).
struct Server;  // serve.cpp

struct BuildState {
  int32_t edge_size_for_creation = 10, edge_size_for_search = 40, batch_size = 200, seed_size = 10;
  float epsilon_for_creation = 0.1f;
  std::vector<std::vector<std::pair<uint32_t, float>>> graph;  // graph repository, slot = object id
  std::vector<uint8_t> in_graph;
  uint64_t graph_size = 0;       // GraphRepository::size() (max inserted id + 1, 0 when empty)
  // tree (leaf ids and internal ids start at 1; leaf 1 is the initial root)
  DevBuf<uint32_t> lf_parent, lf_count, lf_ids, in_parent, in_child, counts;
  DevBuf<uint8_t> lf_has_pivot, lf_pivot, in_pivot;
  DevBuf<float> lf_dist, in_border;
  uint32_t leaf_cap_nodes = 0, in_cap_nodes = 0;
  uint32_t n_leaf = 2, n_internal = 1;  // next ids
  uint32_t root = 0x80000001u;
  GlibcRandHost rnd;
  uint64_t adj_stride = 0;
};

}  // namespace ngt_amd

struct ngt_amd_index {
  using QgState = ngt_amd::QgState;
  template <typename T> using DevBuf = ngt_amd::DevBuf<T>;
  int device = 0;
  int metric = 1;
  int otype = 2;
  uint32_t dim = 0;
  uint32_t dp = 0;
  uint32_t esize = 4;
  uint64_t row_bytes = 0;
  uint64_t nrows = 0;
  DevBuf<uint8_t> rows, valid;
  uint64_t rows_version = 0;     // bumped whenever rows / valid change
  struct {                       // matrix-core scan image of the rows (scan_mfma.hip)
    DevBuf<uint16_t> rh, rl;
    DevBuf<uint32_t> xmax;
    uint64_t version = ~0ull;
    int passes = 0;
  } scan;
  struct {                       // 1-byte filter copy of L2 float rows (filter_kernels.hip)
    DevBuf<uint8_t> codes;
    DevBuf<uint32_t> st;
    DevBuf<float> params;        // {a, b, E, X, valid}
    uint64_t stride = 0;         // bytes per code row
    uint64_t version = ~0ull;
  } filt;
  std::vector<uint8_t> h_valid;
  std::vector<uint64_t> h_degree_nonzero;  // for isEmpty in getRandomSeeds
  DevBuf<uint64_t> edge_off;
  DevBuf<uint32_t> edges;
  uint64_t nedges = 0;
  DevBuf<uint32_t> adj;          // padded fixed-stride copy of the adjacency
  uint64_t adj_stride = 0;
  uint64_t max_degree = 0;       // widest adjacency list
  uint64_t adj_version = 0;      // bumped whenever adj changes

  bool has_graph = false;
  std::vector<uint8_t> h_graph_empty;
  // tree
  bool has_tree = false;
  DevBuf<uint8_t> in_pivot;
  DevBuf<uint32_t> in_child, leaf_ids;
  DevBuf<float> in_border;
  DevBuf<uint64_t> leaf_off;
  uint32_t children = 5, root = 0;
  uint64_t tree_version = 0;     // bumped whenever the tree changes
  // property
  int32_t edge_size_for_search = 0;
  int32_t dyn_base = 30, dyn_rate = 20;
  int32_t seed_size = 10, seed_type = 0;
  // scratch
  std::mutex mu;                           // guards ctxs, calls, rand() seeds
  std::vector<ngt_amd::SearchCtx*> ctxs;   // per launch stream
  std::atomic<ngt_amd::SearchCtx*> last_ctx{nullptr};  // context of the latest search
  std::vector<ngt_amd::CallCtx*> calls;    // idle host-API call contexts
  DevBuf<int> error;
  uint32_t spill_cap = 1u << 16;
  hipStream_t stream = nullptr;
  ngt_amd::BuildState* build = nullptr;    // ANNG construction (build.cpp)
  std::atomic<ngt_amd::Server*> serve{nullptr};  // resident single-query serving grid (serve.cpp)
  // serving-grid exclusion (serve.cpp): a mutator holds the index from before
  // it touches a buffer until the change is complete; served calls register
  // only if no hold began since they read the index's buffers
  std::mutex serve_mu;
  int serve_hold = 0;        // under serve_mu: mutations in progress
  int serve_inflight = 0;    // under serve_mu: served calls past registration
  uint64_t serve_gen = 0;    // under serve_mu: holds begun so far
  ~ngt_amd_index() {
    for (auto* c : ctxs) delete c;
    for (auto* c : calls) delete c;
    delete build;
  }
  int cu_count = 256;
  size_t lds_per_cu = 160 * 1024;
  size_t lds_per_block = 64 * 1024;  // hipDeviceProp_t::sharedMemPerBlock
  QgState qg;                      // NGTQG quantized graph (qg_api.cpp)
  ngt_amd::IvfState ivf;           // NGTQ IVF-ADC quantizer (ivf_api.cpp)
};

namespace ngt_amd {

constexpr uint32_t kTreeSeedStride = 128;  // max seeds per query from a tree leaf

// the launch context of stream s (created on first use), or null on failure
SearchCtx* ctx_for(ngt_amd_index* ix, hipStream_t s);
// per-slot visited scratch for a launch of nq queries (slots = resident waves)
int ensure_vis_scratch(ngt_amd_index* ix, SearchCtx* c, size_t lds_per_slot, uint32_t nq, hipStream_t s);
// device error flag of stream s's launches: read (synchronising s), clear, return
int take_device_error(ngt_amd_index* ix, hipStream_t s, int* flag);
// zero stream s's error word, ordered on s (the start of a host-API call)
int clear_device_error(ngt_amd_index* ix, hipStream_t s);
// the names of the bits set in a device error word ("1: ...; 32: ...")
std::string device_error_text(int flag);
// host-API call contexts (own stream + persistent buffers), pooled per index
CallCtx* acquire_call(ngt_amd_index* ix);
void release_call(ngt_amd_index* ix, CallCtx* c);
struct CallGuard {
  ngt_amd_index* ix;
  CallCtx* c;
  explicit CallGuard(ngt_amd_index* i) : ix(i), c(acquire_call(i)) {}
  ~CallGuard() {
    if (c) release_call(ix, c);
  }
};
int run_tree_seeds(ngt_amd_index* ix, SearchCtx* c, const void* d_queries, uint64_t query_bytes, uint32_t nq,
                   uint32_t k, int all_leaf_nodes, hipStream_t s);
float coef_of(float epsilon);
// the padded adjacency copy holding `need` edges per list (grown on demand;
// caller holds ix->mu), and the edges a search of resolved edge size es reads
int build_padded_adjacency(ngt_amd_index* ix, uint64_t need);
uint64_t adjacency_need(const ngt_amd_index* ix, uint64_t es);
// stop and free the serving grid (serve.cpp); no-op without one
void serve_destroy(ngt_amd_index* ix);
// stop the serving grid before the index's buffers change: new served calls
// take the launch path, the calls in flight finish, the grid leaves; the hold
// lasts until serve_resume (ServeHold does both)
void serve_quiesce(ngt_amd_index* ix);
void serve_resume(ngt_amd_index* ix);
struct ServeHold {
  ngt_amd_index* ix;
  explicit ServeHold(ngt_amd_index* i) : ix(i) { serve_quiesce(ix); }
  ~ServeHold() { serve_resume(ix); }
  ServeHold(const ServeHold&) = delete;
  ServeHold& operator=(const ServeHold&) = delete;
};
// GraphIndex::getRandomSeeds (Index.h:775-801) over the library's rand() stream
// (a fresh process's glibc sequence, ngt_amd_srand)
std::vector<uint32_t> random_seed_lists(ngt_amd_index* ix, uint32_t nq, std::vector<uint64_t>& off);
// host float queries [nq][dim] -> prepared device rows (Index::allocateObject)
int upload_queries(ngt_amd_index* ix, const void* queries, uint32_t nq, DevBuf<float>& raw,
                   DevBuf<uint8_t>& prep, hipStream_t s);

}  // namespace ngt_amd
