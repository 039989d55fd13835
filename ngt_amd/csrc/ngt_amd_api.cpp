// ngt_amd_api.cpp -- host side of the C ABI declared in include/ngt_amd.h.
//
// Owns the HBM layout of an index (padded row-major object slab, CSR
// adjacency, flattened DVP tree, per-slot search scratch) and enqueues the
// gfx950 kernels of search_kernels.hip / prep_kernels.hip.  There is no CPU
// compute path: every distance is evaluated on the device.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cfloat>
#include <string>
#include <vector>

#include "../../include/ngt_amd.h"
#include "index_internal.h"
#include "ngt_kernels.h"
#include "prep_kernels.h"

using namespace ngt_amd;

static thread_local std::string g_err;

int ngt_amd::fail(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return -1;
}

extern "C" const char* ngt_amd_last_error(void) { return g_err.c_str(); }

extern "C" int ngt_amd_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static bool valid_metric(int m) {
  return (m >= 0 && m <= 9) || m == 100 || m == 101;
}

extern "C" int ngt_amd_index_create(ngt_amd_index** out, int device, int distance_type,
                                    int object_type, uint32_t dimension) {
  if (!out) return fail("ngt_amd_index_create: out is null");
  *out = nullptr;
  if (!valid_metric(distance_type)) return fail("ngt_amd_index_create: invalid distance type %d", distance_type);
  if (object_type != 1 && object_type != 2) return fail("ngt_amd_index_create: invalid object type %d", object_type);
  if (dimension == 0) return fail("ngt_amd_index_create: dimension is 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail("ngt_amd_index_create: no HIP device available (the MI355X path has no CPU fallback)");
  if (device < 0 || device >= ndev) return fail("ngt_amd_index_create: device %d out of range", device);
  HIP_OK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, device));
  auto* ix = new ngt_amd_index();
  ix->device = device;
  ix->metric = distance_type;
  ix->otype = object_type;
  ix->dim = dimension;
  // SparseJaccard keeps dimension+1 slots (Index.cpp:488-490 is the caller's job)
  ix->dp = ((dimension - 1) / 16 + 1) * 16;
  ix->esize = object_type == 2 ? 4 : 1;
  ix->row_bytes = (uint64_t)ix->dp * ix->esize;
  // test hook: a tiny unchecked-set spill makes the overflow flag reachable
  if (const char* v = ngt_amd::knob("NGT_AMD_SPILL_CAP")) ix->spill_cap = (uint32_t)std::max(1, atoi(v));
  ix->cu_count = prop.multiProcessorCount;
  ix->lds_per_cu = prop.maxSharedMemoryPerMultiProcessor ? prop.maxSharedMemoryPerMultiProcessor : 160 * 1024;
  ix->lds_per_block = prop.sharedMemPerBlock ? prop.sharedMemPerBlock : 64 * 1024;
  if (hipStreamCreateWithFlags(&ix->stream, hipStreamDefault) != hipSuccess) {
    delete ix;
    return fail("ngt_amd_index_create: stream/event creation failed");
  }
  if (ix->error.alloc(1) != hipSuccess) {
    delete ix;
    return fail("ngt_amd_index_create: allocation failed");
  }
  (void)hipMemset(ix->error.p, 0, sizeof(int));
  *out = ix;
  return 0;
}

extern "C" void ngt_amd_index_destroy(ngt_amd_index* ix) {
  if (!ix) return;
  (void)hipSetDevice(ix->device);
  serve_destroy(ix);  // the resident serving grid reads the index: stop it first
  if (ix->stream) (void)hipStreamSynchronize(ix->stream);
  if (ix->stream) (void)hipStreamDestroy(ix->stream);
  delete ix;
}

extern "C" uint32_t ngt_amd_index_padded_dimension(const ngt_amd_index* ix) {
  return ix ? ix->dp : 0;
}

extern "C" int ngt_amd_index_set_objects(ngt_amd_index* ix, const void* rows, uint64_t nrows,
                                         const uint8_t* valid) {
  if (!ix || !rows || nrows == 0) return fail("ngt_amd_index_set_objects: bad arguments");
  HIP_OK(hipSetDevice(ix->device));
  ServeHold serve_hold(ix);
  HIP_OK(ix->rows.upload(static_cast<const uint8_t*>(rows), nrows * ix->row_bytes));
  ix->nrows = nrows;
  ix->rows_version++;
  ix->h_valid.assign(nrows, 1);
  ix->h_valid[0] = 0;
  if (valid) ix->h_valid.assign(valid, valid + nrows);
  HIP_OK(ix->valid.upload(ix->h_valid.data(), nrows));
  return 0;
}

extern "C" int ngt_amd_index_set_objects_device(ngt_amd_index* ix, const void* d_rows, uint64_t nrows) {
  if (!ix || !d_rows || nrows == 0) return fail("ngt_amd_index_set_objects_device: bad arguments");
  HIP_OK(hipSetDevice(ix->device));
  ServeHold serve_hold(ix);
  ix->rows.release();
  ix->rows.p = (uint8_t*)d_rows;
  ix->rows.n = nrows * ix->row_bytes;
  ix->rows.owned = false;
  ix->nrows = nrows;
  ix->rows_version++;
  ix->h_valid.assign(nrows, 1);
  ix->h_valid[0] = 0;
  HIP_OK(ix->valid.upload(ix->h_valid.data(), nrows));
  return 0;
}

static void note_graph_empty(ngt_amd_index* ix, const uint64_t* offsets, uint64_t nrows) {
  ix->h_graph_empty.assign(nrows, 1);
  for (uint64_t i = 0; i < nrows; i++) ix->h_graph_empty[i] = offsets[i + 1] == offsets[i];
}

// Padded adjacency [nrows][W] built on the device from the CSR: the first W
// edges of every list (W a multiple of 16, at most 256), 0-terminated when
// shorter -- one load per expansion instead of an offset load followed by a
// dependent edge load.  A search reads min(degree, edgeSize) edges of a list
// (Graph.cpp:436-439, getEdgeSize Graph.h:675-692), so the copy serves every
// search with min(max degree, edgeSize) <= W: an NGT index's hubs (an ANNG's
// reverse edges give some nodes hundreds) do not matter at its
// EdgeSizeForSearch of 40.  W grows on demand; searches needing more than 256
// edges of a list take the CSR path.
int ngt_amd::build_padded_adjacency(ngt_amd_index* ix, uint64_t need) {
  if (need == 0 || need > 256) return 0;
  if (ix->adj.p && ix->adj_stride >= need) return 0;
  const uint64_t stride = (need + 15) & ~15ull;
  ServeHold serve_hold(ix);  // a running grid reads the copy being replaced
  ix->adj.release();
  ix->adj_stride = 0;
  HIP_OK(ix->adj.alloc(ix->nrows * stride));
  HIP_OK(launch_pad_adjacency(ix->edge_off.p, ix->edges.p, ix->nrows, stride, ix->adj.p, ix->stream));
  HIP_OK(hipStreamSynchronize(ix->stream));
  ix->adj_stride = stride;
  ix->adj_version++;
  return 0;
}

static uint64_t max_degree_of(const uint64_t* h_offsets, uint64_t nrows) {
  uint64_t maxdeg = 0;
  for (uint64_t i = 0; i < nrows; i++) maxdeg = std::max<uint64_t>(maxdeg, h_offsets[i + 1] - h_offsets[i]);
  return maxdeg;
}

// edges a search with resolved edge size `es` reads of the widest list
uint64_t ngt_amd::adjacency_need(const ngt_amd_index* ix, uint64_t es) {
  return std::min<uint64_t>(ix->max_degree, es);
}

static int reset_adjacency(ngt_amd_index* ix, const uint64_t* h_offsets) {
  ServeHold serve_hold(ix);
  ix->max_degree = max_degree_of(h_offsets, ix->nrows);
  ix->adj.release();
  ix->adj_stride = 0;
  ix->adj_version++;
  // sized for the index's own EdgeSizeForSearch now; grown if a search asks for more
  const int64_t es = ix->edge_size_for_search;
  const uint64_t want = es > 0 ? (uint64_t)es : (uint64_t)INT_MAX;
  return build_padded_adjacency(ix, adjacency_need(ix, want));
}

extern "C" int ngt_amd_index_set_graph(ngt_amd_index* ix, const uint64_t* offsets,
                                       const uint32_t* edges, uint64_t nedges) {
  if (!ix || !offsets || (!edges && nedges)) return fail("ngt_amd_index_set_graph: bad arguments");
  if (ix->nrows == 0) return fail("ngt_amd_index_set_graph: set the objects first");
  if (offsets[ix->nrows] != nedges) return fail("ngt_amd_index_set_graph: offsets[nrows] != nedges");
  for (uint64_t i = 0; i < nedges; i++)
    if (edges[i] == 0 || edges[i] >= ix->nrows)
      return fail("ngt_amd_index_set_graph: edge %llu -> %u out of range", (unsigned long long)i, edges[i]);
  HIP_OK(hipSetDevice(ix->device));
  ServeHold serve_hold(ix);
  HIP_OK(ix->edge_off.upload(offsets, ix->nrows + 1));
  HIP_OK(ix->edges.upload(edges, nedges));
  ix->nedges = nedges;
  ix->has_graph = true;
  note_graph_empty(ix, offsets, ix->nrows);
  return reset_adjacency(ix, offsets);
}

extern "C" int ngt_amd_index_set_graph_device(ngt_amd_index* ix, const uint64_t* d_offsets,
                                              const uint32_t* d_edges, uint64_t nedges) {
  if (!ix || !d_offsets) return fail("ngt_amd_index_set_graph_device: bad arguments");
  HIP_OK(hipSetDevice(ix->device));
  ServeHold serve_hold(ix);
  ix->edge_off.release();
  ix->edges.release();
  ix->edge_off.p = const_cast<uint64_t*>(d_offsets);
  ix->edge_off.owned = false;
  ix->edges.p = const_cast<uint32_t*>(d_edges);
  ix->edges.owned = false;
  ix->nedges = nedges;
  ix->has_graph = true;
  std::vector<uint64_t> h(ix->nrows + 1);
  HIP_OK(hipMemcpy(h.data(), d_offsets, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  note_graph_empty(ix, h.data(), ix->nrows);
  return reset_adjacency(ix, h.data());
}

extern "C" int ngt_amd_index_set_tree(ngt_amd_index* ix, const void* in_pivot, uint32_t n_internal,
                                      const uint32_t* in_child, const float* in_border,
                                      uint32_t children, uint32_t root, const uint64_t* leaf_off,
                                      uint32_t n_leaf, const uint32_t* leaf_ids, uint64_t n_leaf_ids) {
  if (!ix || children < 2 || !leaf_off) return fail("ngt_amd_index_set_tree: bad arguments");
  HIP_OK(hipSetDevice(ix->device));
  ServeHold serve_hold(ix);
  HIP_OK(ix->in_pivot.upload(static_cast<const uint8_t*>(in_pivot), (size_t)n_internal * ix->row_bytes));
  HIP_OK(ix->in_child.upload(in_child, (size_t)n_internal * children));
  HIP_OK(ix->in_border.upload(in_border, (size_t)n_internal * (children - 1)));
  HIP_OK(ix->leaf_off.upload(leaf_off, (size_t)n_leaf + 1));
  HIP_OK(ix->leaf_ids.upload(leaf_ids, n_leaf_ids));
  ix->children = children;
  ix->root = root;
  ix->has_tree = true;
  ix->tree_version++;
  return 0;
}

extern "C" int ngt_amd_index_set_search_property(ngt_amd_index* ix, int32_t edge_size_for_search,
                                                 int32_t dynamic_edge_size_base,
                                                 int32_t dynamic_edge_size_rate, int32_t seed_size,
                                                 int32_t seed_type) {
  if (!ix) return fail("ngt_amd_index_set_search_property: null index");
  ix->edge_size_for_search = edge_size_for_search;
  ix->dyn_base = dynamic_edge_size_base;
  ix->dyn_rate = dynamic_edge_size_rate;
  ix->seed_size = seed_size;
  ix->seed_type = seed_type;
  return 0;
}

float ngt_amd::coef_of(float epsilon) {
  // SearchContainer::setEpsilon (Common.h:2041); 0 => NGT_EXPLORATION_COEFFICIENT (Graph.cpp:403-405)
  float c = (float)((double)epsilon + 1.0);
  if (c == 0.0f) c = (float)1.1;
  return c;
}

extern "C" uint64_t ngt_amd_resolve_edge_size(const ngt_amd_index* ix, int64_t edge_size, float epsilon) {
  // NeighborhoodGraph::getEdgeSize (Graph.h:675-692)
  int64_t esize = edge_size == -1 ? ix->edge_size_for_search : edge_size;
  if (esize == 0) return INT_MAX;
  if (esize > 0) return (uint64_t)esize;
  if (esize == -2) {
    float coef = coef_of(epsilon);
    double add = pow(10, ((double)coef - 1.0) * (double)(float)ix->dyn_rate);
    return add >= (double)INT_MAX ? (uint64_t)INT_MAX : (uint64_t)(ix->dyn_base + add);
  }
  return 0;  // invalid -> caller reports
}

// Launch context of stream s: per-slot scratch of the persistent search
// kernels (slot = resident wave), seed lists, events, error flag.  Created on
// first use; the list is shared by every thread searching this index.
ngt_amd::SearchCtx* ngt_amd::ctx_for(ngt_amd_index* ix, hipStream_t s) {
  std::lock_guard<std::mutex> lk(ix->mu);
  for (auto* c : ix->ctxs)
    if (c->stream == s) {
      ix->last_ctx = c;
      return c;
    }
  auto* c = new SearchCtx();
  c->stream = s;
  // the error word is zeroed on s itself and waited for: a null-stream
  // hipMemset is not ordered with a non-blocking stream, and recycled device
  // memory may hold anything until it lands (GPUTEST_r03's flag 36: a fresh
  // call stream read a stale word while the null stream's fill sat behind the
  // resident serving grid)
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      c->work.alloc(4) != hipSuccess || c->err.alloc(1) != hipSuccess ||
      hipMemsetAsync(c->err.p, 0, sizeof(int), s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
    delete c;
    fail("search: cannot create the launch context of stream %p", (void*)s);
    return nullptr;
  }
  ix->ctxs.push_back(c);
  ix->last_ctx = c;
  return c;
}

int ngt_amd::clear_device_error(ngt_amd_index* ix, hipStream_t s) {
  SearchCtx* c = ctx_for(ix, s);
  if (!c) return -1;
  HIP_OK(hipMemsetAsync(c->err.p, 0, sizeof(int), s));
  return 0;
}

// The bits the device code sets in a launch context's error word.
std::string ngt_amd::device_error_text(int flag) {
  static const char* names[] = {
      "unchecked-set spill capacity exceeded (result list truncated)",        // 1: every search kernel
      "zero-norm query under a normalized metric",                            // 2: prep_kernels.hip
      "one-expansion kernel: stale chunk minimum (invariant)",                // 4: search_kernels.hip
      "lookahead kernel: selection target exceeded by equal keys (invariant)",  // 8: search_la.hip
      "latency kernel: a speculation slot never became ready (timeout)",      // 16: search_lat.hip
      "latency / NGTQG kernel: tail-to-spill threshold selection check",      // 32
      "latency / NGTQG kernel: spill refill selection check",                 // 64
      "latency / NGTQG kernel: head refill selection check",                  // 128
      "(unused since round 5)",                                               // 256
  };
  std::string out;
  for (int b = 0; b < 31; b++) {
    if (!(flag & (1 << b))) continue;
    if (!out.empty()) out += "; ";
    char num[16];
    snprintf(num, sizeof num, "%d: ", 1 << b);
    out += num;
    out += b < 9 ? names[b] : "unknown bit";
  }
  return out;
}

int ngt_amd::take_device_error(ngt_amd_index* ix, hipStream_t s, int* flag) {
  *flag = 0;
  SearchCtx* c = ctx_for(ix, s);
  if (!c) return -1;
  HIP_OK(hipMemcpyAsync(flag, c->err.p, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  if (*flag) HIP_OK(hipMemsetAsync(c->err.p, 0, sizeof(int), s));
  return 0;
}

ngt_amd::CallCtx* ngt_amd::acquire_call(ngt_amd_index* ix) {
  {
    std::lock_guard<std::mutex> lk(ix->mu);
    if (!ix->calls.empty()) {
      CallCtx* c = ix->calls.back();
      ix->calls.pop_back();
      return c;
    }
  }
  auto* c = new CallCtx();
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    fail("search: cannot create a call stream");
    return nullptr;
  }
  return c;
}

void ngt_amd::release_call(ngt_amd_index* ix, CallCtx* c) {
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->calls.push_back(c);
}

// Visited epochs take slots x nrows bytes.  Slots = resident waves of the
// launch (per_cu x CUs, fewer for small batches), bounded only by a share of
// the free HBM (NGT_AMD_VIS_MEM_FRAC, default 0.45 of what is free): a
// 12.5M-row shard keeps 16 waves per CU (51 GB of epochs on a 288 GB GPU).
int ngt_amd::ensure_vis_scratch(ngt_amd_index* ix, SearchCtx* c, size_t lds, uint32_t nq, hipStream_t s) {
  uint32_t per_cu = (uint32_t)(ix->lds_per_cu / lds);
  static const uint32_t max_per_cu = [] {
    const char* v = ngt_amd::knob("NGT_AMD_WAVES_PER_CU");
    return v ? (uint32_t)std::max(1, std::min(32, atoi(v))) : 16u;
  }();
  static const double mem_frac = [] {
    const char* v = ngt_amd::knob("NGT_AMD_VIS_MEM_FRAC");
    return v ? std::max(0.01, std::min(0.9, atof(v))) : 0.45;
  }();
  if (per_cu > max_per_cu) per_cu = max_per_cu;
  if (per_cu < 1) per_cu = 1;
  const uint64_t stride = (ix->nrows + 15) & ~15ull;
  const uint32_t full = per_cu * (uint32_t)ix->cu_count;
  // small launches (coalesced C-API calls) take slots in steps of 64
  uint32_t want = std::min<uint32_t>(full, (nq + 63) & ~63u);
  if (want < c->slots && stride == c->vis_stride && c->spill.p) return 0;  // never shrink
  if (want == c->slots && stride == c->vis_stride && c->spill.p) return 0;
  size_t freeb = 0, totalb = 0;
  HIP_OK(hipMemGetInfo(&freeb, &totalb));
  const double avail = (double)freeb + (double)c->vis.n + (double)c->spill.n * 8.0;
  const uint64_t per_slot = stride + (uint64_t)ix->spill_cap * 8 + 4;
  const uint64_t max_slots = (uint64_t)(avail * mem_frac) / per_slot;
  if (max_slots < 1) return fail("search: no HBM left for the visited scratch (%llu rows)", (unsigned long long)ix->nrows);
  // a context that already holds as many slots as the memory allows now keeps
  // them: reallocating to fewer (other contexts took memory meanwhile) would
  // only cost a synchronizing free + alloc per launch and fewer waves
  // (the 12.5M-row NGTQG line on three streams: 0.7-1.2 s gaps between
  // launches, grids of 1,000-3,300 slots; profiles/r6e)
  if (stride == c->vis_stride && c->spill.p && max_slots <= c->slots) return 0;
  const uint32_t slots = (uint32_t)std::min<uint64_t>(std::max(want, c->slots), max_slots);
  if (slots == c->slots && stride == c->vis_stride && c->spill.p) return 0;
  c->vis.release();
  c->spill.release();
  HIP_OK(c->vis.alloc((size_t)slots * stride));
  // zeroed on the launch stream so the first search is ordered after it
  HIP_OK(hipMemsetAsync(c->vis.p, 0, (size_t)slots * stride, s));
  HIP_OK(c->slot_epoch.alloc(slots));
  HIP_OK(hipMemsetAsync(c->slot_epoch.p, 0, (size_t)slots * sizeof(uint32_t), s));
  HIP_OK(c->spill.alloc((size_t)slots * ix->spill_cap));
  c->slots = slots;
  c->vis_stride = stride;
  return 0;
}

// GraphAndTreeIndex::getSeedsFromTree (Index.h:1524-1567) for a batch: seed
// lists land in c->seeds ([nq][kTreeSeedStride]) and c->seed_count.
int ngt_amd::run_tree_seeds(ngt_amd_index* ix, SearchCtx* c, const void* d_queries, uint64_t query_bytes,
                            uint32_t nq, uint32_t k, int all_leaf_nodes, hipStream_t s) {
  if (!ix->has_tree) return fail("search: tree seeds requested but the index has no tree");
  const uint32_t stride = kTreeSeedStride;
  HIP_OK(c->seeds.alloc((size_t)nq * stride));
  HIP_OK(c->seed_count.alloc(nq));
  TreeSeedArgs t{};
  t.queries = static_cast<const uint8_t*>(d_queries);
  t.query_bytes = query_bytes;
  t.nq = nq;
  t.dp = (int)ix->dp;
  t.row_bytes = ix->row_bytes;
  t.in_pivot = ix->in_pivot.p;
  t.in_child = ix->in_child.p;
  t.in_border = ix->in_border.p;
  t.children = ix->children;
  t.root = ix->root;
  t.leaf_off = ix->leaf_off.p;
  t.leaf_ids = ix->leaf_ids.p;
  t.seed_size = (uint32_t)std::max(ix->seed_size, 0);
  t.k = k;
  t.all_leaf_nodes = all_leaf_nodes || ix->seed_type == 4;
  t.seeds = c->seeds.p;
  t.seed_stride = stride;
  t.seed_count = c->seed_count.p;
  HIP_OK(launch_tree_seeds(t, ix->metric, ix->otype, s));
  return 0;
}

// The filter copy of the current rows, built once per version of the rows
// (synchronously: every stream's launches may read it afterwards).
static int ensure_filter(ngt_amd_index* ix) {
  std::lock_guard<std::mutex> lk(ix->mu);
  if (ix->filt.version == ix->rows_version) return 0;
  // L2 rows of 96/128 elements: dense rows (the search kernel's quads take dp
  // bytes per row); long rows: rows padded to whole 128-B lines
  ix->filt.stride = ix->dp <= 128 ? ix->dp : (ix->dp + 127) / 128 * 128;
  HIP_OK(ix->filt.codes.alloc((size_t)ix->nrows * ix->filt.stride));
  HIP_OK(ix->filt.st.alloc(8));
  HIP_OK(ix->filt.params.alloc(8));
  HIP_OK(launch_filter_build(ix->rows.p, ix->row_bytes, ix->nrows, ix->dp, ix->filt.stride, ix->filt.codes.p, ix->filt.st.p,
                             ix->filt.params.p, ix->stream));
  HIP_OK(hipStreamSynchronize(ix->stream));
  ix->filt.version = ix->rows_version;
  return 0;
}

// Which search kernel a launch takes: -1 the one-expansion-per-pop kernel
// (search_kernels.hip; every metric), 0 / 1 the lookahead kernel
// (search_la.hip; L2 over float rows of 96/128 elements with the padded
// adjacency) in its throughput (a wave per query) or latency (eight waves per
// query: launches of under two queries per CU -- single C-API calls,
// coalesced batches, construction batches) form.  NGT_AMD_LA=0 turns the
// lookahead kernel off, =1 keeps only the throughput form (for any list
// length), =2 only latency.
static int lookahead_mode(const ngt_amd_index* ix, const SearchArgs& a, const ngt_amd_search_params* prm,
                          uint32_t nq) {
  const char* ev = ngt_amd::knob("NGT_AMD_LA");
  const int env = ev ? atoi(ev) : 3;
  if (env == 0) return -1;
  if (ix->metric != NGT_AMD_DISTANCE_L2 || ix->otype != NGT_AMD_OBJECT_FLOAT || (ix->dp != 128 && ix->dp != 96))
    return -1;
  if (!a.adj || a.adj_stride > 256) return -1;
  if (prm->distance_filter < 0) return -1;  // the lookahead kernel always filters
  if (ngt_amd::knob("NGT_AMD_FILTER") && atoi(ngt_amd::knob("NGT_AMD_FILTER")) == 0) return -1;
  const int mode = nq < 2u * (uint32_t)ix->cu_count ? 1 : 0;
  // a wave per query pays off on short lists (an NGT index at its
  // EdgeSizeForSearch of 40: ~4 lists per step); long lists (the C2 kNN graph,
  // ~136 ids) fill a step with one list, and the one-expansion kernel's
  // chunk pipeline with 16 waves per CU is faster there
  const uint64_t deg = std::min<uint64_t>(a.adj_stride, a.edge_size);
  if (mode == 0 && deg > 64 && env != 1) return -1;
  if ((env & (1 << mode)) == 0) return -1;
  return mode;
}

// NGT_AMD_SCHED=0: every search one launch in query order
static int sched_mode() {
  const char* v = ngt_amd::knob("NGT_AMD_SCHED");
  return v ? atoi(v) : 1;
}

static uint32_t __float_as_uint_host(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

// the finished earlier launch's mean expansions per query, into the table
static void sched_collect(SearchCtx* c) {
  if (!c->stat_pending || hipEventQuery(c->ev_stat) != hipSuccess) return;
  c->stat_pending = false;
  if (c->h_stat[1] == 0) return;
  const double mean = (double)c->h_stat[0] / (double)c->h_stat[1];
  for (auto& m : c->sched_mean)
    if (m.first == c->stat_key) {
      m.second = mean;
      return;
    }
  if (c->sched_mean.size() >= 64) c->sched_mean.erase(c->sched_mean.begin());
  c->sched_mean.push_back({c->stat_key, mean});
}

static int run_search(ngt_amd_index* ix, SearchCtx* c, const ngt_amd_search_params* prm, const void* d_queries,
                      uint64_t query_bytes, uint32_t nq, const uint32_t* d_seeds,
                      const uint64_t* d_seed_off, uint32_t* d_ids, float* d_dists, uint32_t* d_n,
                      uint64_t* d_counters, hipStream_t s) {
  if (!ix->has_graph) return fail("search: the index has no graph");
  if (prm->k == 0) return fail("search: k must be > 0");
  uint64_t es = ngt_amd_resolve_edge_size(ix, prm->edge_size, prm->epsilon);
  if (es == 0) return fail("search: invalid edge size %lld", (long long)prm->edge_size);

  SearchArgs a{};
  a.rows = ix->rows.p;
  a.row_bytes = ix->row_bytes;
  a.nrows = (uint32_t)ix->nrows;
  a.dp = (int)ix->dp;
  a.edge_off = ix->edge_off.p;
  a.edges = ix->edges.p;
  {
    // the padded copy, when it holds every edge this search reads
    const uint64_t need = adjacency_need(ix, es);
    std::lock_guard<std::mutex> lk(ix->mu);
    if (build_padded_adjacency(ix, need)) return -1;
    const bool fits = ix->adj.p && need <= ix->adj_stride;
    a.adj = fits ? ix->adj.p : nullptr;
    a.adj_stride = fits ? ix->adj_stride : 0;
  }
  if (const char* v = ngt_amd::knob("NGT_AMD_ADJ"))
    if (atoi(v) == 0) a.adj = nullptr;
  int la_mode = -1;
  a.queries = static_cast<const uint8_t*>(d_queries);
  a.query_bytes = query_bytes;
  a.nq = nq;
  a.k = prm->k;
  a.coef = coef_of(prm->epsilon);
  a.radius = prm->radius < 0.0f ? FLT_MAX : prm->radius;
  a.edge_size = es;
  // LDS capacities of the visited hash and the unchecked array; overridable
  // (NGT_AMD_HT_LOG2 / NGT_AMD_CQ_CAP) so tests can force the exact HBM
  // overflow paths.
  a.ht_log2 = 12;
  a.cq_cap = 1024;
  a.vf_log2 = 0;
  // Small launches (construction batches) leave most of the chip idle and
  // their time is the slowest query's: give each query a larger LDS visited
  // hash and unchecked array (57 KB, two per CU) so long searches stay out
  // of the HBM epochs and the HBM spill.
  if (nq <= 2048 && prm->visited_hash_log2 == 0) {
    a.ht_log2 = 13;
    a.cq_cap = 3072;
    a.vf_log2 = 15;  // for the long ones that outgrow the hash (61.5 KB in all)
    a.k = prm->k;
    if (search_lds_bytes(a, ix->otype) > 64 * 1024) {  // large k: the default sizes
      a.ht_log2 = 12;
      a.cq_cap = 1024;
      a.vf_log2 = 0;
    }
    // up to one wave per CU (a construction batch of 200): each query may take
    // most of its CU's LDS, so the slowest searches -- which decide the batch
    // time -- keep their visited set and unchecked keys out of HBM (a pop
    // otherwise rescans the HBM spill: the tail of 1M ANNG construction)
    if (nq <= (uint32_t)ix->cu_count && ix->lds_per_block >= 128 * 1024) {
      SearchArgs b = a;
      b.ht_log2 = 14;
      b.cq_cap = 8192;
      b.vf_log2 = 15;
      if (search_lds_bytes(b, ix->otype) <= ix->lds_per_block) a = b;
    }
  }
  if (prm->visited_hash_log2 < 0) {
    // HBM-epoch visited set (searches visiting ~1e5 ids, the C2 bench): a
    // 32 Kbit LDS filter proves most fresh ids unvisited without their HBM
    // probe, paid for by a 512-key unchecked array (same 9 KB of LDS, 16
    // waves per CU); measured +8 % QPS on C2 at identical results.
    // Long rows (C3: 3,840 B) dwarf the 128-B probe and their searches
    // saturate any LDS-sized filter: epochs alone there.
    a.ht_log2 = 0;
    // 512 unchecked keys in LDS (exact HBM spill beyond): C3's long rows then
    // fit 16 waves per CU instead of 11 (+6 % QPS).  Long cosine/angle rows
    // run at 12 waves per CU (search_kernels.hip), whose LDS holds 768: 794
    // vs 808 ms per C3 launch (profiles/r5zk)
    a.cq_cap = 512;
    if (ix->row_bytes > 1024 && ix->otype == NGT_AMD_OBJECT_FLOAT &&
        (ix->metric == NGT_AMD_DISTANCE_COSINE || ix->metric == NGT_AMD_DISTANCE_ANGLE))
      a.cq_cap = 768;
    if (ix->row_bytes <= 1024) {
      a.vf_log2 = 15;
      // -2: the filter and epochs hold accepted ids only (a few thousand per
      // query instead of ~7e4), so the filter stays sparse and almost no
      // neighbour costs an HBM probe or a mark store; rejected neighbours met
      // again are re-evaluated (search_common.h: not_accepted).  C2: +33 % QPS
      // at identical results for +14 % distance evaluations.
      a.accepted_only = prm->visited_hash_log2 == -2;
    }
  }
  else if (prm->visited_hash_log2 > 0) a.ht_log2 = (uint32_t)std::max(8, std::min(15, prm->visited_hash_log2));
  if (const char* v = ngt_amd::knob("NGT_AMD_HT_LOG2")) a.ht_log2 = (uint32_t)std::max(8, std::min(15, atoi(v)));
  if (const char* v = ngt_amd::knob("NGT_AMD_CQ_CAP")) a.cq_cap = (uint32_t)std::max(64, std::min(8192, atoi(v)));
  if (const char* v = ngt_amd::knob("NGT_AMD_ACCEPTED_ONLY")) a.accepted_only = atoi(v) != 0;
  if (const char* v = ngt_amd::knob("NGT_AMD_VFILTER")) {
    const int f = atoi(v);
    a.vf_log2 = f <= 0 ? 0u : (uint32_t)std::max(11, std::min(18, f));
  }
  a.out_ids = d_ids;
  a.out_dists = d_dists;
  a.out_n = d_n;
  a.counters = d_counters;
  a.error = c->err.p;
  // 1-byte filter copy for throughput launches over L2 float rows of 96/128
  // elements: a neighbour the bound places outside the exploration radius
  // costs Dp bytes instead of 4 Dp (filter_kernels.hip); latency-bound small
  // launches (construction batches) skip it, since a surviving neighbour then
  // costs a second round trip.  NGT_AMD_FILTER=0/1 forces it off/on.
  {
    static const int force = [] {
      const char* v = ngt_amd::knob("NGT_AMD_FILTER");
      return v ? atoi(v) : -1;
    }();
    // L2 rows of 96/128 floats (integer bound, pipelined expansion) or
    // cosine/angle long rows (streamed comparator; search_common.h filter_cos_u8)
    const bool shape = ix->otype == NGT_AMD_OBJECT_FLOAT &&
                       ((ix->metric == NGT_AMD_DISTANCE_L2 && (ix->dp == 128 || ix->dp == 96)) ||
                        ((ix->metric == NGT_AMD_DISTANCE_COSINE || ix->metric == NGT_AMD_DISTANCE_ANGLE) &&
                         ix->dp > 128 && ix->dp % 64 == 0 && !ngt_amd::knob("NGT_AMD_NO_STREAM")));
    const bool want = force >= 0 ? force != 0
                                 : (prm->distance_filter != 0 ? prm->distance_filter > 0
                                                              : nq >= 2u * (uint32_t)ix->cu_count);
    // the lookahead kernel (search_la.hip) shares one filter round trip
    // among a step's expansions, so it takes the filter at every launch size
    la_mode = lookahead_mode(ix, a, prm, nq);
    if (shape && (want || la_mode >= 0)) {
      if (ensure_filter(ix)) return -1;
      a.fcodes = ix->filt.codes.p;
      a.fstride = ix->filt.stride;
      a.fparams = ix->filt.params.p;
    }
    c->launch_filtered = a.fcodes != nullptr;
    if (!a.fcodes) la_mode = -1;
  }
  if (la_mode >= 0) {
    // one step's target lists (<= 256 ids each) and the exact per-step id set
    static const uint32_t env_lmax = [] {
      const char* v = ngt_amd::knob("NGT_AMD_LA_LMAX");
      return v ? (uint32_t)std::max(256, std::min(8192, atoi(v))) : 0u;
    }();
    // list capacity: the targets' lists of the longest kind (t0's always fits)
    const uint32_t deg_cap = (uint32_t)std::min<uint64_t>(a.adj_stride, a.edge_size);
    const uint32_t P = la_targets(la_mode);
    a.la_lmax = env_lmax ? env_lmax
                         : (la_mode == 0 ? std::max<uint32_t>(deg_cap, std::min<uint32_t>(256u, (P * deg_cap + 15) & ~15u))
                                         : 2048u);
    a.la_lmax = std::max<uint32_t>(a.la_lmax, deg_cap);
    // per-step id set: twice the ids a step can insert -- every list entry
    // with the full visited set; the accepted-only set inserts only accepted
    // ids, and the commit loop stops before a target could overfill it, so
    // there 4 x the longest list is plenty (and keeps 12 waves per CU)
    const uint32_t sh_want = (la_mode == 0 && a.accepted_only) ? std::min<uint32_t>(2u * a.la_lmax, 4u * deg_cap)
                                                               : 2u * a.la_lmax;
    a.la_sh_log2 = 1;
    while ((1u << a.la_sh_log2) < sh_want) a.la_sh_log2++;
    if (a.vf_log2 == 0) a.vf_log2 = 15;
    a.cq_cap = la_mode == 0 ? 512u : 2048u;
    if (la_mode == 0 && la_wpe() == 4) {
      a.vf_log2 = 14;
      a.cq_cap = 256u;
    }
    if (const char* v = ngt_amd::knob("NGT_AMD_CQ_CAP")) a.cq_cap = (uint32_t)std::max(64, std::min(8192, atoi(v)));
    if (const char* v = ngt_amd::knob("NGT_AMD_VFILTER"))
      if (atoi(v) > 0) a.vf_log2 = (uint32_t)std::max(11, std::min(18, atoi(v)));
  }

  if (prm->seed_mode == NGT_AMD_SEED_TREE) {
    if (run_tree_seeds(ix, c, d_queries, query_bytes, nq, prm->k, prm->all_leaf_nodes, s)) return -1;
    a.seeds = c->seeds.p;
    a.seed_stride = kTreeSeedStride;
    a.seed_count = c->seed_count.p;
  } else {
    if (!d_seeds || !d_seed_off) return fail("search: seed lists required for this seed mode");
    a.seeds = d_seeds;
    a.seed_off = d_seed_off;
  }
  const size_t lds_max = std::max<size_t>(64 * 1024, std::min<size_t>(ix->lds_per_block, ix->lds_per_cu));
  // latency launches: the speculating kernel (search_lat.hip) when the exact
  // LDS visited bitmap of every object fits one CU's LDS with its slots
  bool lat = false;
  if (la_mode == 1) {
    static const bool lat_on = [] {
      const char* v = ngt_amd::knob("NGT_AMD_LAT");
      return !v || atoi(v) != 0;
    }();
    const uint32_t cap = (uint32_t)std::min<uint64_t>(a.adj_stride, a.edge_size);
    if (lat_on && a.adj && cap <= 256u && a.k <= 64u) {  // lists of <= 256 ids, results in one wave's registers
      SearchArgs b = a;
      b.lat_slots = cap <= 64 ? 32u : 16u;
      b.lat_tail = 4096u;
      b.lat_hop = lat_hop_default();
      b.lat_feed = lat_feed_default();
      while (search_lat_lds_bytes(b) > lds_max && b.lat_tail > 512u) b.lat_tail -= 256u;
      while (search_lat_lds_bytes(b) > lds_max && b.lat_slots > 8u) b.lat_slots -= 2u;
      // test knobs: a small tail forces the HBM spill, few slots the orphan path
      if (const char* v = ngt_amd::knob("NGT_AMD_LAT_TAIL")) b.lat_tail = (uint32_t)std::max(128, std::min(4096, atoi(v)));
      if (const char* v = ngt_amd::knob("NGT_AMD_LAT_SLOTS")) b.lat_slots = (uint32_t)std::max(2, std::min(64, atoi(v)));
      if (search_lat_lds_bytes(b) <= lds_max) {
        a = b;
        lat = true;
      }
    }
  }
  if (!lat && la_mode >= 0 && search_la_lds_bytes(a, (int)la_targets(la_mode)) > lds_max) la_mode = -1;  // large k
  const size_t lds = lat ? search_lat_lds_bytes(a)
                         : la_mode >= 0 ? search_la_lds_bytes(a, (int)la_targets(la_mode)) : search_lds_bytes(a, ix->otype);
  if (lds > lds_max) return fail("search: k=%u needs %zu bytes of LDS per query (max %zu)", a.k, lds, lds_max);
  if (ensure_vis_scratch(ix, c, lds, nq, s)) return -1;
  a.vis = c->vis.p;
  a.vis_stride = c->vis_stride;
  a.slot_epoch = c->slot_epoch.p;
  a.spill = c->spill.p;
  a.spill_cap = ix->spill_cap;
  a.work = c->work.p;
  HIP_OK(hipMemsetAsync(c->work.p, 0, 3 * sizeof(uint32_t), s));
  uint32_t slots = std::min<uint32_t>(c->slots, nq);
  c->launch_slots = slots;
  c->launch_la = la_mode;
  // ---- launch schedule: "probe and resume" ------------------------------
  // A launch's time is its slowest slot's: with ~2.4 queries per slot, a long
  // search that happens to start last decides it (C2: 22.1 ms in query order,
  // 16.6 ms longest-first with the true costs, profiles/r4d).  Cheap query
  // features do not predict the cost (centroid distance, sampled distance
  // contrast: rank correlation < 0.1); the search's own state does: the
  // unchecked keys within the exploration radius after part of the search.
  // So a probe launch runs every query for B expansions (B = 0.25 x the mean
  // expansions per query of earlier launches of this configuration) and
  // pauses the unfinished ones with their state saved; a one-workgroup
  // counting sort orders them by that count; a resume launch continues them
  // in that order.  Accepted-only visited sets only (the resume rebuilds the
  // set from the popped ids and the unchecked keys; search_kernels.hip), so
  // the results, distance bits and expansion counts are the single
  // launch's.  Measured (profiles/r4e, r4f): C2 22.2 -> 18.6 ms per 10k-query
  // search at 0.12 (19.4 at 0.25, 20.2 at 0.4) on the kNN128 graph; on the
  // denser kNN256 graph (327 expansions per query, profiles/r5o, r5p) 16.3 /
  // 16.2 / 15.4 / 15.4 / 15.1 / 15.3 ms at 0.06 / 0.12 / 0.2 / 0.25 / 0.3 /
  // 0.4.  The lookahead kernel (the ANNG's short lists) took the same scheme
  // and ran slower at every fraction (0.08-0.5: 164-174 ms against 156), so
  // it is not scheduled.
  const bool sched_shape = !lat && la_mode < 0 && a.accepted_only && a.ht_log2 == 0 && a.vf_log2 != 0 && a.adj &&
                           a.fcodes && a.k <= 64;
  uint32_t budget = 0;
  uint64_t skey = 0;
  if (sched_shape && sched_mode() != 0) {
    skey = (uint64_t)a.edge_size * 0x9E3779B97F4A7C15ull ^ ((uint64_t)__float_as_uint_host(a.coef) << 17) ^
           ((uint64_t)a.k << 49) ^ (ix->rows_version * 0xC2B2AE3D27D4EB4Full) ^ (ix->adj_version << 7) ^
           ((uint64_t)a.cq_cap << 33);
    sched_collect(c);
    double mean = 0.0;
    for (auto& m : c->sched_mean)
      if (m.first == skey) mean = m.second;
    static const double frac = [] {
      const char* v = ngt_amd::knob("NGT_AMD_SCHED_FRAC");
      return v ? std::max(0.01, std::min(0.9, atof(v))) : 0.25;
    }();
    // test knob: a fixed budget for every eligible launch
    const int forced = ngt_amd::knob("NGT_AMD_SCHED_B") ? std::max(0, atoi(ngt_amd::knob("NGT_AMD_SCHED_B"))) : 0;
    if (forced) budget = (uint32_t)forced;
    else if (mean > 0.0) budget = (uint32_t)std::max(8.0, mean * frac);
    // a tail needs more queries than slots (forced: any launch, for tests)
    if (!forced && (uint64_t)nq * 4 < (uint64_t)slots * 5) budget = 0;
  }
  if (budget) {
    // the paused queries' records (~17 KB per query at cq_cap 1024) must fit
    // beside everything else: at most a quarter of the free HBM, else (or if
    // the allocation fails) the search is one dispatch -- same results
    const PauseLayout lay(a.k, a.cq_cap, budget);
    const size_t need = (size_t)nq * lay.total;
    if (!(c->qstate.p && c->qstate.owned && c->qstate.n >= need)) {
      size_t fr = 0, tot = 0;
      HIP_OK(hipMemGetInfo(&fr, &tot));
      const size_t bytes = need * sizeof(*c->qstate.p) + (size_t)nq * 16;
      if (bytes > fr / 4 || c->qstate.alloc(need) != hipSuccess) {
        (void)hipGetLastError();
        c->qstate.release();
        budget = 0;
      }
    }
  }
  c->launch_budget = budget;
  if (sched_shape) {
    HIP_OK(c->stat.alloc(2));
    HIP_OK(hipMemsetAsync(c->stat.p, 0, 2 * sizeof(unsigned long long), s));
    a.stat = c->stat.p;
  }
  HIP_OK(hipEventRecord(c->ev0, s));
  if (lat) {
    HIP_OK(launch_graph_search_lat(a, slots, s));
  } else if (la_mode >= 0) {
    // full visited set unless the caller asked for the accepted-only one
    HIP_OK(launch_graph_search_la(a, la_mode, !a.accepted_only, slots, s));
  } else if (budget) {
    const PauseLayout lay(a.k, a.cq_cap, budget);
    HIP_OK(c->qstate.alloc((size_t)nq * lay.total));
    HIP_OK(c->qflag.alloc(nq));
    HIP_OK(c->prio.alloc(nq));
    HIP_OK(c->order.alloc(nq));
    HIP_OK(hipMemsetAsync(c->qflag.p, 0, (size_t)nq * sizeof(uint32_t), s));
    SearchArgs p = a;
    p.pause_after = budget;
    p.qstate = c->qstate.p;
    p.qstate_stride = lay.total;
    p.qflag = c->qflag.p;
    p.prio = c->prio.p;
    auto go = [&](const SearchArgs& x) -> hipError_t { return launch_graph_search(x, ix->metric, ix->otype, slots, s); };
    HIP_OK(go(p));
    HIP_OK(launch_schedule(c->qflag.p, c->prio.p, nq, c->order.p, c->work.p + 2, s));
    SearchArgs r = p;
    r.pause_after = 0;
    r.order = c->order.p;
    r.nwork_dev = c->work.p + 2;
    r.work = c->work.p + 1;
    HIP_OK(go(r));
  } else {
    HIP_OK(launch_graph_search(a, ix->metric, ix->otype, slots, s));
  }
  HIP_OK(hipEventRecord(c->ev1, s));
  if (sched_shape) {
    // this launch's mean expansions per query, for the next launch's budget
    if (!c->h_stat) HIP_OK(hipHostMalloc((void**)&c->h_stat, 2 * sizeof(unsigned long long), hipHostMallocDefault));
    if (!c->ev_stat) HIP_OK(hipEventCreateWithFlags(&c->ev_stat, hipEventDisableTiming));
    HIP_OK(hipMemcpyAsync(c->h_stat, c->stat.p, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIP_OK(hipEventRecord(c->ev_stat, s));
    c->stat_pending = true;
    c->stat_key = skey;
  }
  return 0;
}

// The rand() stream getRandomSeeds draws from.  The reference calls the
// process-wide glibc rand(), so a fresh `ngt search -i g` process draws from
// seed 1.  The GPU runtime in this process may call rand() itself, which
// would shift that stream between searches; the library therefore keeps its
// own glibc TYPE_3 generator (random_r restated, index_internal.h), seeded 1
// like a fresh process and reseeded only by ngt_amd_srand -- the reference's
// sequence, independent of anything else in the process.
static std::mutex g_rand_mu;
static GlibcRandHost& seed_rand() {
  static GlibcRandHost r = [] {
    GlibcRandHost g;
    g.seed(1);
    return g;
  }();
  return r;
}

extern "C" void ngt_amd_srand(unsigned int seed) {
  std::lock_guard<std::mutex> lk(g_rand_mu);
  seed_rand().seed(seed);
}

std::vector<uint32_t> ngt_amd::random_seed_lists(ngt_amd_index* ix, uint32_t nq, std::vector<uint64_t>& off) {
  // GraphIndex::getRandomSeeds (Index.h:775-801) over the rand() stream, one
  // query after another as the reference's callers do.
  std::lock_guard<std::mutex> lk(g_rand_mu);
  GlibcRandHost& rnd = seed_rand();
  std::vector<uint32_t> seeds;
  off.assign(nq + 1, 0);
  size_t repo = ix->nrows == 0 ? 0 : ix->nrows - 1;
  size_t ss = std::min<size_t>(repo, (size_t)std::max(ix->seed_size, 0));
  for (uint32_t q = 0; q < nq; q++) {
    size_t start = seeds.size();
    size_t empty = 0;
    while (seeds.size() - start < ss) {
      double random = ((double)rnd.next() + 1.0) / ((double)RAND_MAX + 2.0);
      size_t idx = (size_t)floor((double)repo * random) + 1;
      if (ix->h_graph_empty[idx]) {
        if (++empty > repo) break;
        continue;
      }
      if (std::find(seeds.begin() + start, seeds.end(), (uint32_t)idx) != seeds.end()) continue;
      seeds.push_back((uint32_t)idx);
    }
    off[q + 1] = seeds.size();
  }
  return seeds;
}

extern "C" int ngt_amd_search_device(ngt_amd_index* ix, const ngt_amd_search_params* prm,
                                     const void* d_queries, uint64_t query_bytes, uint32_t nq,
                                     const uint32_t* d_seeds, const uint64_t* d_seed_off,
                                     uint32_t* d_ids, float* d_dists, uint32_t* d_n,
                                     uint64_t* d_counters, void* stream) {
  if (!ix || !prm || (!d_queries && nq)) return fail("ngt_amd_search_device: bad arguments");
  if (nq && query_bytes < ix->row_bytes)
    return fail("ngt_amd_search_device: query stride %llu < %llu bytes (queries are prepared rows of the padded dimension)",
                (unsigned long long)query_bytes, (unsigned long long)ix->row_bytes);
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(ix->device));
  hipStream_t s = (hipStream_t)stream;  // null = the default stream
  SearchCtx* c = ctx_for(ix, s);
  if (!c) return -1;
  if (prm->seed_mode == NGT_AMD_SEED_RANDOM) {
    std::vector<uint64_t> off;
    std::vector<uint32_t> seeds = random_seed_lists(ix, nq, off);
    HIP_OK(c->seed_off.upload(off.data(), off.size()));
    HIP_OK(c->seeds.upload(seeds.data(), std::max<size_t>(seeds.size(), 1)));
    return run_search(ix, c, prm, d_queries, query_bytes, nq, c->seeds.p, c->seed_off.p, d_ids,
                      d_dists, d_n, d_counters, s);
  }
  return run_search(ix, c, prm, d_queries, query_bytes, nq, d_seeds, d_seed_off, d_ids, d_dists,
                    d_n, d_counters, s);
}

extern "C" int ngt_amd_tree_seeds_device(ngt_amd_index* ix, const void* d_queries, uint64_t query_bytes, uint32_t nq,
                                         uint32_t k, uint32_t* d_seeds, uint32_t seed_stride, uint32_t* d_count,
                                         void* stream) {
  if (!ix || (!d_queries && nq) || !d_seeds || !d_count || k == 0 || seed_stride < kTreeSeedStride)
    return fail("ngt_amd_tree_seeds_device: bad arguments (seed_stride must be >= %u)", kTreeSeedStride);
  if (nq && query_bytes < ix->row_bytes) return fail("ngt_amd_tree_seeds_device: query stride too small");
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(ix->device));
  hipStream_t s = (hipStream_t)stream;
  SearchCtx* c = ctx_for(ix, s);
  if (!c) return -1;
  if (run_tree_seeds(ix, c, d_queries, query_bytes, nq, k, 0, s)) return -1;
  HIP_OK(hipMemcpy2DAsync(d_seeds, (size_t)seed_stride * sizeof(uint32_t), c->seeds.p,
                          (size_t)kTreeSeedStride * sizeof(uint32_t), (size_t)kTreeSeedStride * sizeof(uint32_t), nq,
                          hipMemcpyDeviceToDevice, s));
  HIP_OK(hipMemcpyAsync(d_count, c->seed_count.p, (size_t)nq * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  return 0;
}

extern "C" int ngt_amd_last_search_filtered(const ngt_amd_index* ix) {
  if (!ix) return 0;
  SearchCtx* c = ix->last_ctx.load();
  return c && c->launch_filtered ? 1 : 0;
}

extern "C" int ngt_amd_last_search_lookahead(const ngt_amd_index* ix) {
  if (!ix) return -1;
  SearchCtx* c = ix->last_ctx.load();
  return c ? c->launch_la : -1;
}

extern "C" uint32_t ngt_amd_last_search_budget(const ngt_amd_index* ix) {
  if (!ix) return 0;
  SearchCtx* c = ix->last_ctx.load();
  return c ? c->launch_budget : 0;
}

extern "C" int ngt_amd_stream_error_word(ngt_amd_index* ix, void* stream, int* word) {
  if (!ix || !word) return fail("ngt_amd_stream_error_word: bad arguments");
  HIP_OK(hipSetDevice(ix->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  SearchCtx* c = ctx_for(ix, s);
  if (!c) return -1;
  HIP_OK(hipMemcpyAsync(word, c->err.p, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

extern "C" uint32_t ngt_amd_last_search_slots(const ngt_amd_index* ix) {
  if (!ix) return 0;
  SearchCtx* c = ix->last_ctx.load();
  return c ? c->launch_slots : 0;
}

extern "C" float ngt_amd_last_search_kernel_ms(const ngt_amd_index* ix) {
  if (!ix) return 0.f;
  SearchCtx* c = ix->last_ctx.load();
  if (!c) return -1.f;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.f;
  return ms;
}

// Upload host float queries and prepare them on the device.
int ngt_amd::upload_queries(ngt_amd_index* ix, const void* queries, uint32_t nq, DevBuf<float>& raw,
                          DevBuf<uint8_t>& prep, hipStream_t s) {
  // host queries are float [nq][dim] for every object type (Index::allocateObject
  // converts them to the object type, ObjectRepository.h:222-253)
  HIP_OK(raw.upload_async(static_cast<const float*>(queries), (size_t)nq * ix->dim, s));
  HIP_OK(prep.alloc((size_t)nq * ix->row_bytes));
  if (ngt_amd_prepare_queries_device(ix, raw.p, nq, prep.p, s)) return -1;
  return 0;
}

extern "C" int ngt_amd_prepare_queries_device(ngt_amd_index* ix, const float* d_in, uint32_t nq,
                                              void* d_out, void* stream) {
  if (!ix || (!d_in && nq) || (!d_out && nq)) return fail("ngt_amd_prepare_queries_device: bad arguments");
  if (nq == 0) return 0;
  hipStream_t s = (hipStream_t)stream;  // null = the default stream
  SearchCtx* c = ctx_for(ix, s);
  if (!c) return -1;
  bool normalize = ix->metric == 5 || ix->metric == 6 || ix->metric == 9;
  HIP_OK(launch_prepare_queries(d_in, ix->dim, nq, ix->dp, ix->otype, normalize, d_out, c->err.p, s));
  return 0;
}

extern "C" int ngt_amd_search(ngt_amd_index* ix, const ngt_amd_search_params* prm, const void* queries,
                              uint32_t nq, const uint32_t* seeds, const uint64_t* seed_off,
                              uint32_t* ids, float* dists, uint32_t* n, uint64_t* counters) {
  if (!ix || !prm || (!queries && nq) || !ids || !dists || !n) return fail("ngt_amd_search: bad arguments");
  if (nq == 0) return 0;
  if (prm->seed_mode == NGT_AMD_SEED_GIVEN) {
    if (!seeds || !seed_off) return fail("ngt_amd_search: NGT_AMD_SEED_GIVEN needs seeds and seed_off");
    for (uint64_t i = 0; i < seed_off[nq]; i++)
      if (seeds[i] == 0 || seeds[i] >= ix->nrows) return fail("ngt_amd_search: seed id %u out of range", seeds[i]);
  }
  HIP_OK(hipSetDevice(ix->device));
  CallGuard g(ix);
  CallCtx* cc = g.c;
  if (!cc) return -1;
  hipStream_t s = cc->stream;
  // this call's error word starts clear on its own stream: a flag names the
  // launches of this call and nothing earlier
  if (clear_device_error(ix, s)) return -1;
  if (upload_queries(ix, queries, nq, cc->raw, cc->prep, s)) return -1;
  HIP_OK(cc->ids.alloc((size_t)nq * prm->k));
  HIP_OK(cc->dists.alloc((size_t)nq * prm->k));
  HIP_OK(cc->n.alloc(nq));
  if (counters) HIP_OK(cc->cnt.alloc((size_t)nq * NGT_AMD_COUNTERS_PER_QUERY));
  const uint32_t* sp = nullptr;
  const uint64_t* so = nullptr;
  if (prm->seed_mode == NGT_AMD_SEED_GIVEN) {
    HIP_OK(cc->seeds.alloc(std::max<uint64_t>(seed_off[nq], 1)));
    HIP_OK(cc->seed_off.alloc((size_t)nq + 1));
    HIP_OK(hipMemcpyAsync(cc->seeds.p, seeds, seed_off[nq] * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(cc->seed_off.p, seed_off, ((size_t)nq + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    sp = cc->seeds.p;
    so = cc->seed_off.p;
  }
  if (ngt_amd_search_device(ix, prm, cc->prep.p, ix->row_bytes, nq, sp, so, cc->ids.p, cc->dists.p, cc->n.p,
                            counters ? cc->cnt.p : nullptr, s))
    return -1;
  HIP_OK(hipMemcpyAsync(ids, cc->ids.p, (size_t)nq * prm->k * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(dists, cc->dists.p, (size_t)nq * prm->k * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(n, cc->n.p, (size_t)nq * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (counters)
    HIP_OK(hipMemcpyAsync(counters, cc->cnt.p, (size_t)nq * NGT_AMD_COUNTERS_PER_QUERY * sizeof(uint64_t),
                          hipMemcpyDeviceToHost, s));
  int herr = 0;
  if (take_device_error(ix, s, &herr)) return -1;
  if (herr) return fail("ngt_amd_search: device error flag %d (%s)", herr, device_error_text(herr).c_str());
  return 0;
}

// Error-bound constants of the matrix-core filter (scan_mfma.hip, DESIGN.md
// 4d): the bf16 hi+lo split (3 passes) leaves < 3.1 * 2^-16 |q||x| of the
// dot product, bf16 alone (1 pass) < (2^-7 + 2^-16) |q||x|; the fp32
// accumulation of P dp + 16 terms < (P dp + 16) 2^-24 of the sum of
// magnitudes; both doubled (Cosine: quadrupled, it also absorbs the
// normalization), plus the comparator's own rounding (rho) where used.
static int scan_passes() {
  static const int p = [] {
    const char* v = ngt_amd::knob("NGT_AMD_SCAN_PASSES");
    return v && atoi(v) == 1 ? 1 : 3;
  }();
  return p;
}
static double scan_kappa(const ngt_amd_index* ix, int passes) {
  const double dp = (double)ix->dp;
  const double split = passes == 3 ? 3.2 * std::ldexp(1.0, -16) : 1.02 * std::ldexp(1.0, -7);
  const double base = split + (passes * dp + 64.0) * std::ldexp(1.0, -23);
  return ix->metric == NGT_AMD_DISTANCE_COSINE ? 4.0 * base : 2.0 * base;
}

// The rows' bf16 hi/lo image in fragment order plus the norm column, built
// once per version of the rows (first batch scan after set_objects).
static int ensure_scan_rows(ngt_amd_index* ix, int passes, hipStream_t s) {
  std::lock_guard<std::mutex> lk(ix->mu);
  if (ix->scan.version == ix->rows_version && ix->scan.passes == passes) return 0;
  const uint32_t ks = ix->dp / 16 + 1;
  const uint64_t ntiles = (ix->nrows + 255) / 256;  // 256-row scan tiles
  const size_t elems = (size_t)ntiles * 8 * ks * 512;
  HIP_OK(ix->scan.rh.alloc(elems));
  HIP_OK(ix->scan.rl.alloc(elems));
  HIP_OK(ix->scan.xmax.alloc(1));
  HIP_OK(hipMemsetAsync(ix->scan.xmax.p, 0, sizeof(uint32_t), s));
  const double kappa = scan_kappa(ix, passes);
  ScanPrepArgs p{};
  p.src = ix->rows.p;
  p.stride = ix->row_bytes;
  p.n = ix->nrows;
  p.valid = ix->valid.p;
  p.dp = (int)ix->dp;
  p.ks = ks;
  p.ntiles32 = ntiles * 8;
  p.out_h = ix->scan.rh.p;
  p.out_l = ix->scan.rl.p;
  p.one_minus_kappa = (float)(1.0 - kappa);
  p.kappa = (float)kappa;
  p.xmax_bits = ix->scan.xmax.p;
  HIP_OK(launch_scan_prep(p, ix->metric == NGT_AMD_DISTANCE_COSINE, false, s));
  // other streams may scan as soon as the version is published
  HIP_OK(hipStreamSynchronize(s));
  ix->scan.version = ix->rows_version;
  ix->scan.passes = passes;
  return 0;
}

static int linear_search_mfma(ngt_amd_index* ix, SearchCtx* c, LinearArgs& a, hipStream_t s) {
  const int passes = scan_passes();
  if (ensure_scan_rows(ix, passes, s)) return -1;
  const bool cosine = ix->metric == NGT_AMD_DISTANCE_COSINE;
  const uint32_t ks = ix->dp / 16 + 1;
  const uint32_t mblocks = (a.nq + 127) / 128;  // 128 queries per workgroup
  const uint64_t nqpad = (uint64_t)mblocks * 128;
  HIP_OK(c->sqh.alloc((size_t)nqpad * ks * 16));
  HIP_OK(c->sql.alloc((size_t)nqpad * ks * 16));
  HIP_OK(c->shb.alloc(nqpad * 2));
  const double kappa = scan_kappa(ix, passes);
  ScanPrepArgs p{};
  p.src = a.queries;
  p.stride = a.query_bytes;
  p.n = a.nq;
  p.n_pad = nqpad;
  p.dp = (int)ix->dp;
  p.ks = ks;
  p.ntiles32 = nqpad / 32;
  p.out_h = c->sqh.p;
  p.out_l = c->sql.p;
  p.one_minus_kappa = (float)(1.0 - kappa);
  p.kappa = (float)kappa;
  p.slack = std::ldexp(1.0f, -100);
  p.xmax_bits = ix->scan.xmax.p;
  p.hb = c->shb.p;
  p.hm = c->shb.p + nqpad;
  // bootstrap margin: two filter errors plus the comparator's rounding
  const double rho = ((double)ix->dp + 64.0) * std::ldexp(1.0, -22);
  p.kappa_boot = (float)(cosine ? 2.0 * kappa : kappa + rho);
  HIP_OK(launch_scan_prep(p, cosine, true, s));

  // Launches of at most one workgroup per CU.  Default: one launch, every
  // query block x floor(CUs / blocks) parts (a workgroup keeps its queries'
  // k-lists for its whole part; each part costs ~k ln(rows / k) candidates per
  // query, so few long parts).
  const uint32_t ntiles = (uint32_t)((ix->nrows + 255) / 256);
  const uint32_t per_launch = mblocks;
  auto parts_of = [&](uint32_t mbc) -> uint32_t {
    uint32_t np = std::max<uint32_t>(1, (uint32_t)ix->cu_count / mbc);
    np = std::min(np, ntiles);
    const uint32_t per = (ntiles + np - 1) / np;
    return (ntiles + per - 1) / per;
  };
  MfmaScanArgs m{};
  m.rh = ix->scan.rh.p;
  m.rl = ix->scan.rl.p;
  m.qh = c->sqh.p;
  m.ql = c->sql.p;
  m.hb = c->shb.p;
  m.hm = c->shb.p + nqpad;
  m.rows = ix->rows.p;
  m.row_bytes = ix->row_bytes;
  m.queries = a.queries;
  m.query_bytes = a.query_bytes;
  m.nq = a.nq;
  m.k = a.k;
  m.ks = ks;
  m.dp = (int)ix->dp;
  m.ntiles = ntiles;
  m.radius = a.radius;
  if (cosine) {
    m.scale = 1.0f;
    m.t_init = a.radius < 0.0 || a.radius >= 3.0e38 ? INFINITY : (float)a.radius;
  } else {
    m.scale = (float)((1.0 + rho) * 0.5);
    m.t_init = INFINITY;
    if (a.radius >= 0.0 && a.radius < 3.0e38) {
      // squared-sum bound of the radius (scan_sq_bound on the host)
      float d = (float)a.radius;
      uint32_t u;
      memcpy(&u, &d, 4);
      u++;
      float dn;
      memcpy(&dn, &u, 4);
      float s2 = (float)((double)dn * (double)dn);
      memcpy(&u, &s2, 4);
      u++;
      memcpy(&m.t_init, &u, 4);
    }
  }
  if (const char* v = ngt_amd::knob("NGT_AMD_SCAN_DBG")) m.dbg = (uint32_t)atoi(v);
  static const bool stats = ngt_amd::knob("NGT_AMD_SCAN_STATS") != nullptr;
  static DevBuf<unsigned long long> d_stats;
  if (stats) {
    HIP_OK(d_stats.alloc(4));
    HIP_OK(hipMemsetAsync(d_stats.p, 0, 4 * sizeof(unsigned long long), s));
    m.stats = d_stats.p;
  }
  HIP_OK(c->gthr.alloc(a.nq));
  HIP_OK(hipMemsetAsync(c->gthr.p, 0xff, (size_t)a.nq * sizeof(uint64_t), s));
  m.gthr = reinterpret_cast<unsigned long long*>(c->gthr.p);
  // partial lists of every launch, back to back
  size_t partial_total = 0;
  for (uint32_t mb0 = 0; mb0 < mblocks; mb0 += per_launch) {
    const uint32_t mbc = std::min(per_launch, mblocks - mb0);
    const uint32_t nqc = std::min<uint32_t>(a.nq - mb0 * 128, mbc * 128);
    partial_total += (size_t)nqc * parts_of(mbc) * a.k;
  }
  HIP_OK(c->partial.alloc(partial_total));
  size_t poff = 0;
  m.xcd = 0;
  for (uint32_t mb0 = 0; mb0 < mblocks; mb0 += per_launch) {
    const uint32_t mbc = std::min(per_launch, mblocks - mb0);
    const uint32_t nqc = std::min<uint32_t>(a.nq - mb0 * 128, mbc * 128);
    const uint32_t nparts = parts_of(mbc);
    m.mb0 = mb0;
    m.mblocks = mbc;
    m.nparts = nparts;
    m.tiles_per_part = (ntiles + nparts - 1) / nparts;
    m.partial = c->partial.p + poff;
    HIP_OK(launch_scan_mfma(m, ix->metric, passes, s));
    LinearArgs ac = a;
    ac.nq = nqc;
    ac.partial = m.partial;
    ac.out_ids = a.out_ids + (size_t)mb0 * 128 * a.k;
    ac.out_dists = a.out_dists + (size_t)mb0 * 128 * a.k;
    ac.out_n = a.out_n + (size_t)mb0 * 128;
    HIP_OK(launch_linear_merge(ac, nparts, s));
    poff += (size_t)nqc * nparts * a.k;
  }
  if (stats) {
    unsigned long long h[4];
    HIP_OK(hipMemcpyAsync(h, d_stats.p, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    fprintf(stderr, "scan_mfma: nq %u launches %u candidates %llu rounds %llu process_requests %llu\n", a.nq,
            (mblocks + per_launch - 1) / per_launch, h[0], h[1], h[2]);
  }
  return 0;
}

extern "C" int ngt_amd_linear_search_device(ngt_amd_index* ix, const void* d_queries, uint64_t query_bytes,
                                            uint32_t nq, uint32_t k, double radius, uint32_t* d_ids,
                                            float* d_dists, uint32_t* d_n, void* stream) {
  if (!ix || (!d_queries && nq) || k == 0) return fail("ngt_amd_linear_search_device: bad arguments");
  if (nq && query_bytes < ix->row_bytes)
    return fail("ngt_amd_linear_search_device: query stride %llu < %llu bytes (queries are prepared rows of the padded dimension)",
                (unsigned long long)query_bytes, (unsigned long long)ix->row_bytes);
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(ix->device));
  hipStream_t s = (hipStream_t)stream;  // null = the default stream
  SearchCtx* c = ctx_for(ix, s);  // the slice buffer belongs to this index and stream
  if (!c) return -1;
  LinearArgs a{};
  a.rows = ix->rows.p;
  a.row_bytes = ix->row_bytes;
  a.nrows = ix->nrows;
  a.dp = (int)ix->dp;
  a.valid = ix->valid.p;
  a.queries = static_cast<const uint8_t*>(d_queries);
  a.query_bytes = query_bytes;
  a.nq = nq;
  a.k = k;
  a.radius = radius;
  a.out_ids = d_ids;
  a.out_dists = d_dists;
  a.out_n = d_n;
  // Batches of queries, L2 / Cosine: the matrix-core filtered scan
  // (scan_mfma.hip) -- bf16 MFMA dot products with a proven error bound pick
  // the candidates, the comparator recomputes them bit for bit.
  static const bool use_mfma = [] {
    const char* v = ngt_amd::knob("NGT_AMD_LINEAR_MFMA");
    return !(v && atoi(v) == 0);
  }();
  if (use_mfma && nq >= 32 && ix->otype == NGT_AMD_OBJECT_FLOAT && k <= 16 &&
      (ix->metric == NGT_AMD_DISTANCE_L2 || ix->metric == NGT_AMD_DISTANCE_COSINE))
    return linear_search_mfma(ix, c, a, s);
  // Batches of queries: the query-tiled scan (128 queries per workgroup,
  // packed FMA, scan_kernels.hip) over enough row parts for ~3 workgroups
  // per CU slot; small batches keep the quad-per-row kernel below.
  static const bool tiled = [] {
    const char* v = ngt_amd::knob("NGT_AMD_LINEAR_TILED");
    return !(v && atoi(v) == 0);
  }();
  if (tiled && nq >= 32 && ix->metric == NGT_AMD_DISTANCE_L2 && ix->otype == NGT_AMD_OBJECT_FLOAT && k <= 32 &&
      ix->dp <= 256) {
    const uint64_t qblocks = (nq + 127) / 128;
    uint64_t nparts = ((uint64_t)ix->cu_count * 12 + qblocks - 1) / qblocks;
    nparts = std::max<uint64_t>(1, std::min<uint64_t>(nparts, (ix->nrows + 1023) / 1024));
    const uint64_t per = ((ix->nrows + nparts - 1) / nparts + 7) & ~7ull;
    nparts = (ix->nrows + per - 1) / per;
    HIP_OK(c->partial.alloc((size_t)nq * nparts * k));
    a.partial = c->partial.p;
    hipError_t e = launch_linear_scan(a, ix->metric, ix->otype, (uint32_t)nparts, (uint32_t)per, s);
    if (e == hipSuccess) {
      HIP_OK(launch_linear_merge(a, (uint32_t)nparts, s));
      return 0;
    }
    if (e != hipErrorNotSupported) return fail("ngt_amd_linear_search_device: scan launch failed: %s",
                                               hipGetErrorString(e));
  }
  // enough slices to fill the chip: ~4 waves per CU over all queries
  uint64_t want = ((uint64_t)ix->cu_count * 16 + nq - 1) / nq;
  uint64_t maxs = (ix->nrows + 255) / 256;
  uint32_t nslices = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, std::max<uint64_t>(maxs, 1)));
  HIP_OK(c->partial.alloc((size_t)nq * nslices * k));
  a.partial = c->partial.p;
  HIP_OK(launch_linear_search(a, ix->metric, ix->otype, nslices, s));
  return 0;
}

extern "C" int ngt_amd_linear_search(ngt_amd_index* ix, const void* queries, uint32_t nq, uint32_t k,
                                     double radius, uint32_t* ids, float* dists, uint32_t* n) {
  if (!ix || (!queries && nq) || !ids || !dists || !n || k == 0) return fail("ngt_amd_linear_search: bad arguments");
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(ix->device));
  CallGuard g(ix);
  CallCtx* cc = g.c;
  if (!cc) return -1;
  hipStream_t s = cc->stream;
  if (upload_queries(ix, queries, nq, cc->raw, cc->prep, s)) return -1;
  HIP_OK(cc->ids.alloc((size_t)nq * k));
  HIP_OK(cc->dists.alloc((size_t)nq * k));
  HIP_OK(cc->n.alloc(nq));
  if (ngt_amd_linear_search_device(ix, cc->prep.p, ix->row_bytes, nq, k, radius, cc->ids.p, cc->dists.p, cc->n.p, s))
    return -1;
  HIP_OK(hipMemcpyAsync(ids, cc->ids.p, (size_t)nq * k * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(dists, cc->dists.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(n, cc->n.p, (size_t)nq * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int ngt_amd_distances(ngt_amd_index* ix, const void* queries, uint32_t nq, const uint32_t* qidx,
                                 const uint32_t* oid, uint64_t npairs, float* out) {
  // queries are taken as prepared objects: [nq][padded dim] of the object type
  // (the comparator compares two allocated objects, PrimitiveComparator.h:650-752).
  if (!ix || !queries || !qidx || !oid || !out) return fail("ngt_amd_distances: bad arguments");
  if (npairs == 0) return 0;
  HIP_OK(hipSetDevice(ix->device));
  for (uint64_t i = 0; i < npairs; i++) {
    if (qidx[i] >= nq) return fail("ngt_amd_distances: query index %u out of range", qidx[i]);
    if (oid[i] >= ix->nrows) return fail("ngt_amd_distances: object id %u out of range", oid[i]);
  }
  CallGuard g(ix);
  if (!g.c) return -1;
  hipStream_t s = g.c->stream;
  DevBuf<uint8_t> q;
  HIP_OK(q.upload(static_cast<const uint8_t*>(queries), (size_t)nq * ix->row_bytes));
  DevBuf<uint32_t> dq, dobj;
  DevBuf<float> dout;
  HIP_OK(dq.upload(qidx, npairs));
  HIP_OK(dobj.upload(oid, npairs));
  HIP_OK(dout.alloc(npairs));
  DistanceArgs a{};
  a.rows = ix->rows.p;
  a.row_bytes = ix->row_bytes;
  a.queries = q.p;
  a.query_bytes = ix->row_bytes;
  a.qidx = dq.p;
  a.oid = dobj.p;
  a.out = dout.p;
  a.npairs = npairs;
  a.dp = (int)ix->dp;
  HIP_OK(launch_distances(a, ix->metric, ix->otype, s));
  HIP_OK(hipMemcpyAsync(out, dout.p, npairs * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int ngt_amd_merge_results_device(int device, const uint32_t* d_ids, const float* d_dists,
                                            const uint32_t* d_n, uint32_t nparts, uint32_t nq, uint32_t k,
                                            const uint32_t* id_offsets, uint32_t* d_out_ids, float* d_out_dists,
                                            uint32_t* d_out_n, void* stream) {
  if (!d_ids || !d_dists || !d_n || !id_offsets || !d_out_ids || !d_out_dists || !d_out_n || nparts == 0 || k == 0)
    return fail("ngt_amd_merge_results_device: bad arguments");
  if ((uint64_t)nparts * k * sizeof(uint64_t) > 64 * 1024)
    return fail("ngt_amd_merge_results_device: %u parts x k=%u exceed one workgroup's LDS", nparts, k);
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(device));
  hipStream_t s = (hipStream_t)stream;
  DevBuf<uint32_t> off;
  HIP_OK(off.alloc(nparts));
  HIP_OK(hipMemcpyAsync(off.p, id_offsets, nparts * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  MergeArgs a{};
  a.in_ids = d_ids;
  a.in_dists = d_dists;
  a.in_n = d_n;
  a.id_offsets = off.p;
  a.nparts = nparts;
  a.nq = nq;
  a.k = k;
  a.out_ids = d_out_ids;
  a.out_dists = d_out_dists;
  a.out_n = d_out_n;
  HIP_OK(launch_merge_results(a, s));
  // `off` is freed on return: order the free after the kernel
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int ngt_amd_pack_results_device(int device, const uint32_t* d_ids, const float* d_dists,
                                           const uint32_t* d_n, uint32_t nq, uint32_t k, uint64_t* d_packed,
                                           void* stream) {
  if ((!d_ids || !d_dists || !d_n || !d_packed) && nq) return fail("ngt_amd_pack_results_device: bad arguments");
  if (nq == 0 || k == 0) return 0;
  HIP_OK(hipSetDevice(device));
  HIP_OK(launch_pack_results(d_ids, d_dists, d_n, nq, k, d_packed, (hipStream_t)stream));
  return 0;
}

extern "C" int ngt_amd_merge_packed_device(int device, const uint64_t* d_packed, uint32_t nparts, uint32_t nq,
                                           uint32_t k, const uint32_t* id_offsets, uint32_t* d_out_ids,
                                           float* d_out_dists, uint32_t* d_out_n, void* stream) {
  if (!d_packed || !id_offsets || !d_out_ids || !d_out_dists || !d_out_n || nparts == 0 || k == 0)
    return fail("ngt_amd_merge_packed_device: bad arguments");
  if ((uint64_t)nparts * k * sizeof(uint64_t) > 64 * 1024)
    return fail("ngt_amd_merge_packed_device: %u parts x k=%u exceed one workgroup's LDS", nparts, k);
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(device));
  hipStream_t s = (hipStream_t)stream;
  DevBuf<uint32_t> off;
  HIP_OK(off.alloc(nparts));
  HIP_OK(hipMemcpyAsync(off.p, id_offsets, nparts * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  MergeArgs a{};
  a.id_offsets = off.p;
  a.nparts = nparts;
  a.nq = nq;
  a.k = k;
  a.out_ids = d_out_ids;
  a.out_dists = d_out_dists;
  a.out_n = d_out_n;
  HIP_OK(launch_merge_packed(a, d_packed, s));
  HIP_OK(hipStreamSynchronize(s));  // `off` is freed on return
  return 0;
}
