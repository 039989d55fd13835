// serve.cpp -- the resident serving grid behind single-query searches
// (ngt_amd_search_served, include/ngt_amd.h): the reference's concurrent
// single-query callers (Capi.cpp:377-406 ngt_search_index, one
// NeighborhoodGraph::search per call) answered by one long-lived launch of
// the latency kernel's serving form (search_lat.hip, SERVE = true) instead of
// a launch per call or per group of calls.
//
//   caller                       pinned host memory            device
//   ------                       ------------------            ------
//   ticket t, fill slot t % R -> ring[t % R] (query, seeds,  <- dispatcher lane
//   release seq = t + 1           k, coefficient, radius)       publishes t
//                                                             <- a worker (one
//   spin on resp[t % R].seq   <- resp[t % R] (ids, dists,       query per CU)
//                                 counters, error bits)         claims, answers
//
// Each caller polls its own response slot in host memory, so a query costs its
// own search and nothing of anyone else's: no batch waits for its slowest
// member.  The grid leaves when nothing was posted or in flight for idle_ms
// (a search longer than idle_ms keeps it: a sequential caller's next query
// finds it running), after life_s,
// or when asked (a configuration change, destroy); a caller that finds its
// ticket unanswered with the grid gone launches the next grid, which starts at
// the first unclaimed ticket.  The search is the batch kernel's (the same
// commit wave), so results equal the reference's.
//
//   NGT_AMD_SERVE=0             never serve (callers take the launch path)
//   NGT_AMD_SERVE_WORKERS=n     worker workgroups, one query each (default: CUs - 1)
//   NGT_AMD_SERVE_IDLE_MS=n     idle time (nothing posted or in flight) before the grid leaves (default 20)
//   NGT_AMD_SERVE_LOG=1         a stderr line per grid: lifetime, why it left
#include <float.h>
#include <stdio.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "index_internal.h"

namespace ngt_amd {

namespace {

bool serve_enabled() {
  static const bool on = [] {
    const char* v = ngt_amd::knob("NGT_AMD_SERVE");
    const char* l = ngt_amd::knob("NGT_AMD_LAT");
    return !(v && atoi(v) == 0) && !(l && atoi(l) == 0);
  }();
  return on;
}

// what a grid is launched with: a request of another configuration waits for
// a moment with nothing in flight to relaunch, or takes the launch path
struct ServeConfig {
  const void* rows;
  const void* adj;
  const void* pivot;
  const void* leaf_ids;
  uint64_t nrows, adj_stride, es, rows_version, adj_version, tree_version;
  int32_t use_tree, all_leaf, seed_size, lat_slots, lat_tail;
  bool operator==(const ServeConfig& o) const { return memcmp(this, &o, sizeof o) == 0; }
};

}  // namespace

struct Server {
  std::mutex mu;  // the launch state below
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  bool launched = false;
  ServeConfig cfg{};
  SearchArgs a{};
  uint32_t start = 0;  // first ticket of the next launch
  // the ring (pinned host memory; d* the device's view of it)
  uint32_t nring = 1024;
  uint64_t req_bytes = 0;
  uint8_t* ring = nullptr;
  ServeResp* resp = nullptr;
  uint32_t* stop = nullptr;
  uint8_t* dring = nullptr;
  ServeResp* dresp = nullptr;
  uint32_t* dstop = nullptr;
  DevBuf<ServeDevCtl> dctl;
  DevBuf<uint64_t> spill;
  DevBuf<int> err;
  uint32_t workers = 0;  // server_init: CUs - 1
  uint64_t clock_khz = 100000;
  double idle_ms = 20.0, life_s = 10.0;
  // tickets
  std::mutex tk_mu;
  std::condition_variable tk_cv;
  uint32_t next = 0;
  std::vector<uint8_t> busy;
  int inflight = 0;  // under mu: calls on the grid's configuration (a switch waits for none)
  std::atomic<uint64_t> served{0}, launches{0};
  bool log = false;  // NGT_AMD_SERVE_LOG=1: a stderr line per grid
  std::chrono::steady_clock::time_point t_launch;

  ~Server() {
    if (s) {
      if (stop) __atomic_store_n(stop, 1u, __ATOMIC_RELEASE);
      (void)hipStreamSynchronize(s);
    }
    if (ev) (void)hipEventDestroy(ev);
    if (s) (void)hipStreamDestroy(s);
    if (ring) (void)hipHostFree(ring);
    if (resp) (void)hipHostFree(resp);
    if (stop) (void)hipHostFree(stop);
  }
};

namespace {

int server_init(ngt_amd_index* ix, Server* sv) {
  HIP_OK(hipStreamCreateWithFlags(&sv->s, hipStreamNonBlocking));
  HIP_OK(hipEventCreateWithFlags(&sv->ev, hipEventDisableTiming));
  sv->req_bytes = ((uint64_t)kServeQueryOff + 4ull * ix->dp + 63) & ~63ull;
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
  HIP_OK(hipHostMalloc((void**)&sv->ring, sv->req_bytes * sv->nring, fl));
  HIP_OK(hipHostMalloc((void**)&sv->resp, sizeof(ServeResp) * sv->nring, fl));
  HIP_OK(hipHostMalloc((void**)&sv->stop, 64, fl));
  memset(sv->ring, 0, sv->req_bytes * sv->nring);
  memset(sv->resp, 0, sizeof(ServeResp) * sv->nring);
  sv->stop[0] = sv->stop[1] = 0;
  HIP_OK(hipHostGetDevicePointer((void**)&sv->dring, sv->ring, 0));
  HIP_OK(hipHostGetDevicePointer((void**)&sv->dresp, sv->resp, 0));
  HIP_OK(hipHostGetDevicePointer((void**)&sv->dstop, sv->stop, 0));
  sv->busy.assign(sv->nring, 0);
  HIP_OK(sv->dctl.alloc(1));
  HIP_OK(sv->err.alloc(1));
  HIP_OK(hipMemsetAsync(sv->err.p, 0, sizeof(int), sv->s));
  HIP_OK(hipStreamSynchronize(sv->s));
  // one worker per CU but the dispatcher's (each workgroup owns its CU's LDS)
  const char* v = ngt_amd::knob("NGT_AMD_SERVE_WORKERS");
  const int w = v ? atoi(v) : ix->cu_count - 1;
  sv->workers = (uint32_t)std::max(1, std::min(w, ix->cu_count - 1));
  if (const char* t = ngt_amd::knob("NGT_AMD_SERVE_IDLE_MS")) sv->idle_ms = std::max(1.0, atof(t));
  if (const char* t = ngt_amd::knob("NGT_AMD_SERVE_LOG")) sv->log = atoi(t) != 0;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ix->device) == hipSuccess && khz > 0)
    sv->clock_khz = (uint64_t)khz;
  HIP_OK(sv->spill.alloc((size_t)sv->workers * ix->spill_cap));
  return 0;
}

bool server_running(Server* sv) { return sv->launched && hipEventQuery(sv->ev) == hipErrorNotReady; }

// the grid has left or is asked to: wait for it, and start the next one at
// the first ticket no worker claimed (caller holds sv->mu)
int server_reap(Server* sv, bool ask) {
  if (!sv->launched) return 0;
  if (ask) __atomic_store_n(sv->stop, 1u, __ATOMIC_RELEASE);
  HIP_OK(hipEventSynchronize(sv->ev));
  ServeDevCtl c{};
  HIP_OK(hipMemcpyAsync(&c, sv->dctl.p, sizeof c, hipMemcpyDeviceToHost, sv->s));
  HIP_OK(hipStreamSynchronize(sv->s));
  __atomic_store_n(sv->stop, 0u, __ATOMIC_RELEASE);
  sv->start = c.claimed;
  sv->launched = false;
  if (sv->log) {
    const double alive = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - sv->t_launch).count();
    fprintf(stderr, "[serve] grid %llu left after %.1f ms (%s), tickets up to %u\n",
            (unsigned long long)sv->launches.load(), alive,
            c.pad == 1 ? "asked" : c.pad == 2 ? "idle" : c.pad == 3 ? "lifetime" : "workers' own bound", c.claimed);
  }
  return 0;
}

// a grid for sv->cfg / sv->a (caller holds sv->mu; none running)
int server_launch(ngt_amd_index* ix, Server* sv) {
  ServeDevCtl c{sv->start, sv->start, 0u, 0u, sv->start};
  HIP_OK(hipMemcpyAsync(sv->dctl.p, &c, sizeof c, hipMemcpyHostToDevice, sv->s));
  HIP_OK(hipStreamSynchronize(sv->s));
  __atomic_store_n(sv->stop, 0u, __ATOMIC_RELEASE);
  ServeArgs g{};
  g.ring = sv->dring;
  g.req_bytes = sv->req_bytes;
  g.resp = sv->dresp;
  g.nring = sv->nring;
  g.workers = sv->workers;
  g.dctl = sv->dctl.p;
  g.stop = sv->dstop;
  g.start = sv->start;
  g.use_tree = (uint32_t)sv->cfg.use_tree;
  g.idle_ticks = (uint64_t)(sv->idle_ms * (double)sv->clock_khz);
  g.life_ticks = (uint64_t)(sv->life_s * 1e3 * (double)sv->clock_khz);
  if (sv->cfg.use_tree) {
    TreeSeedArgs& t = g.tree;
    t.dp = (int)ix->dp;
    t.row_bytes = ix->row_bytes;
    t.in_pivot = ix->in_pivot.p;
    t.in_child = ix->in_child.p;
    t.in_border = ix->in_border.p;
    t.children = ix->children;
    t.root = ix->root;
    t.leaf_off = ix->leaf_off.p;
    t.leaf_ids = ix->leaf_ids.p;
    t.seed_size = (uint32_t)sv->cfg.seed_size;
    t.all_leaf_nodes = sv->cfg.all_leaf;
  }
  SearchArgs a = sv->a;
  a.spill = sv->spill.p;
  a.spill_cap = ix->spill_cap;
  a.error = sv->err.p;
  HIP_OK(launch_graph_serve_lat(a, g, sv->s));
  HIP_OK(hipEventRecord(sv->ev, sv->s));
  sv->t_launch = std::chrono::steady_clock::now();
  sv->launched = true;
  sv->launches++;
  return 0;
}

// the latency kernel's arguments for this index and request shape; 1 when the
// serving form does not take it (the caller launches instead)
int serve_args(ngt_amd_index* ix, const ngt_amd_search_params* prm, SearchArgs& a, ServeConfig& cfg) {
  if (!ix->has_graph || ix->metric != NGT_AMD_DISTANCE_L2 || ix->otype != NGT_AMD_OBJECT_FLOAT) return 1;
  if (ix->dp != 128 && ix->dp != 96) return 1;
  if (prm->k == 0 || prm->k > 64) return 1;
  const bool tree = prm->seed_mode == NGT_AMD_SEED_TREE;
  if (!tree && prm->seed_mode != NGT_AMD_SEED_RANDOM) return 1;
  if (tree && !ix->has_tree) return 1;
  if (!tree && ix->seed_size > (int32_t)kServeMaxSeeds) return 1;
  const uint64_t es = ngt_amd_resolve_edge_size(ix, prm->edge_size, prm->epsilon);
  if (es == 0) return 1;
  a = SearchArgs{};
  {
    std::lock_guard<std::mutex> lk(ix->mu);
    const uint64_t need = adjacency_need(ix, es);
    if (build_padded_adjacency(ix, need)) return -1;
    if (!ix->adj.p || need > ix->adj_stride) return 1;
    a.adj = ix->adj.p;
    a.adj_stride = ix->adj_stride;
  }
  const uint32_t cap = (uint32_t)std::min<uint64_t>(a.adj_stride, es);
  if (cap > 256u) return 1;
  a.rows = ix->rows.p;
  a.row_bytes = ix->row_bytes;
  a.nrows = (uint32_t)ix->nrows;
  a.dp = (int)ix->dp;
  a.edge_off = ix->edge_off.p;
  a.edges = ix->edges.p;
  a.edge_size = es;
  a.k = prm->k;
  // the batch latency launch's LDS sizing (ngt_amd_api.cpp run_search)
  const size_t lds_max = std::max<size_t>(64 * 1024, std::min<size_t>(ix->lds_per_block, ix->lds_per_cu));
  a.lat_slots = cap <= 64 ? 32u : 16u;
  a.lat_tail = 4096u;
  a.lat_hop = lat_hop_default();
  a.lat_feed = lat_feed_default();
  while (search_lat_lds_bytes(a) > lds_max && a.lat_tail > 512u) a.lat_tail -= 256u;
  while (search_lat_lds_bytes(a) > lds_max && a.lat_slots > 8u) a.lat_slots -= 2u;
  if (const char* v = ngt_amd::knob("NGT_AMD_LAT_TAIL")) a.lat_tail = (uint32_t)std::max(128, std::min(4096, atoi(v)));
  if (const char* v = ngt_amd::knob("NGT_AMD_LAT_SLOTS")) a.lat_slots = (uint32_t)std::max(2, std::min(64, atoi(v)));
  if (search_lat_lds_bytes(a) > lds_max) return 1;
  cfg = ServeConfig{};
  cfg.rows = ix->rows.p;
  cfg.adj = a.adj;
  cfg.pivot = tree ? (const void*)ix->in_pivot.p : nullptr;
  cfg.leaf_ids = tree ? (const void*)ix->leaf_ids.p : nullptr;
  cfg.nrows = ix->nrows;
  cfg.adj_stride = a.adj_stride;
  cfg.es = es;
  cfg.rows_version = ix->rows_version;
  cfg.adj_version = ix->adj_version;
  cfg.tree_version = tree ? ix->tree_version : 0;
  cfg.use_tree = tree ? 1 : 0;
  cfg.all_leaf = tree ? ((prm->all_leaf_nodes || ix->seed_type == 4) ? 1 : 0) : 0;
  cfg.seed_size = tree ? std::max(ix->seed_size, 0) : 0;
  cfg.lat_slots = (int32_t)a.lat_slots;
  cfg.lat_tail = (int32_t)a.lat_tail;
  return 0;
}

}  // namespace

// The index is about to change (rows, graph, padded adjacency, tree): new
// served calls take the launch path, the calls in flight finish, and the grid
// leaves -- it holds the old buffers' pointers, and so does the relaunch
// state sv->a.  The hold lasts until serve_resume, i.e. until the mutator has
// swapped its buffers: a served call that read the index before the hold
// began sees serve_gen changed when it tries to register and takes the launch
// path, so no grid or relaunch is ever configured with a freed pointer.
// The callers in flight never take ix->mu, so a caller holding it may wait here.
void serve_quiesce(ngt_amd_index* ix) {
  {
    std::lock_guard<std::mutex> lk(ix->serve_mu);
    ix->serve_hold++;
    ix->serve_gen++;
  }
  for (;;) {
    {
      std::lock_guard<std::mutex> lk(ix->serve_mu);
      if (ix->serve_inflight == 0) break;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  Server* sv = ix->serve.load();
  if (!sv) return;
  std::lock_guard<std::mutex> lk(sv->mu);
  (void)server_reap(sv, true);
  sv->cfg = ServeConfig{};
}

void serve_resume(ngt_amd_index* ix) {
  std::lock_guard<std::mutex> lk(ix->serve_mu);
  ix->serve_hold--;
}

void serve_destroy(ngt_amd_index* ix) {
  Server* sv = ix->serve.load();
  if (!sv) return;
  {
    std::lock_guard<std::mutex> lk(sv->mu);
    (void)server_reap(sv, true);
  }
  delete sv;
  ix->serve.store(nullptr);
}

}  // namespace ngt_amd

using namespace ngt_amd;

extern "C" int ngt_amd_search_served(ngt_amd_index* ix, const ngt_amd_search_params* prm, const float* query,
                                     uint32_t* ids, float* dists, uint32_t* n, uint64_t* counters) {
  if (!ix || !prm || !query || !ids || !dists || !n) return fail("ngt_amd_search_served: bad arguments");
  if (!serve_enabled()) return 1;
  // the index's buffers are read below without a lock: valid only if no
  // mutation (serve_quiesce .. serve_resume) began meanwhile
  uint64_t gen0;
  {
    std::lock_guard<std::mutex> lk(ix->serve_mu);
    if (ix->serve_hold) return 1;
    gen0 = ix->serve_gen;
  }
  SearchArgs a{};
  ServeConfig cfg{};
  {
    const int r = serve_args(ix, prm, a, cfg);
    if (r) return r;
  }
  HIP_OK(hipSetDevice(ix->device));
  Server* sv;
  {
    std::lock_guard<std::mutex> lk(ix->mu);
    if (!ix->serve.load()) {
      Server* fresh = new Server();
      if (server_init(ix, fresh)) {
        delete fresh;
        return -1;
      }
      ix->serve.store(fresh);
    }
    sv = ix->serve.load();
  }
  // register: from here a mutator's quiesce waits for this call
  {
    std::lock_guard<std::mutex> lk(ix->serve_mu);
    if (ix->serve_hold || ix->serve_gen != gen0) return 1;
    ix->serve_inflight++;
  }
  struct Unregister {
    ngt_amd_index* ix;
    ~Unregister() {
      std::lock_guard<std::mutex> lk(ix->serve_mu);
      ix->serve_inflight--;
    }
  } unregister{ix};
  // join the grid's configuration, or switch it when nothing is in flight
  {
    std::lock_guard<std::mutex> lk(sv->mu);
    if (!(sv->cfg == cfg)) {
      if (sv->inflight > 0) return 1;
      if (server_reap(sv, true)) return -1;
      sv->cfg = cfg;
      sv->a = a;
    }
    sv->inflight++;
  }
  struct Leave {
    Server* sv;
    ~Leave() {
      std::lock_guard<std::mutex> lk(sv->mu);
      sv->inflight--;
    }
  } leave{sv};
  // a ticket and its slot
  uint32_t t;
  {
    std::unique_lock<std::mutex> lk(sv->tk_mu);
    t = sv->next++;
    __atomic_store_n(sv->stop + 1, sv->next, __ATOMIC_RELEASE);  // the grid stays while tickets are out
    sv->tk_cv.wait(lk, [&] { return sv->busy[t % sv->nring] == 0; });
    sv->busy[t % sv->nring] = 1;
  }
  struct Release {
    Server* sv;
    uint32_t slot;
    ~Release() {
      std::lock_guard<std::mutex> lk(sv->tk_mu);
      sv->busy[slot] = 0;
      sv->tk_cv.notify_all();
    }
  } rel{sv, t % sv->nring};
  uint8_t* req = sv->ring + (uint64_t)(t % sv->nring) * sv->req_bytes;
  ServeReqHdr* h = reinterpret_cast<ServeReqHdr*>(req);
  h->k = prm->k;
  h->coef = coef_of(prm->epsilon);
  h->radius = prm->radius < 0.0f ? FLT_MAX : prm->radius;
  h->ns = 0;
  if (!cfg.use_tree) {
    std::vector<uint64_t> off;
    std::vector<uint32_t> seeds = random_seed_lists(ix, 1, off);
    const uint32_t ns = (uint32_t)std::min<size_t>(seeds.size(), kServeMaxSeeds);
    memcpy(req + 32, seeds.data(), 4ull * ns);
    h->ns = ns;
  }
  float* q = reinterpret_cast<float*>(req + kServeQueryOff);
  memcpy(q, query, 4ull * ix->dim);
  for (uint32_t i = ix->dim; i < ix->dp; i++) q[i] = 0.f;
  ServeResp* r = sv->resp + (t % sv->nring);
  __atomic_store_n(&h->seq, t + 1u, __ATOMIC_RELEASE);
  // a grid to take it
  {
    std::lock_guard<std::mutex> lk(sv->mu);
    if (!server_running(sv)) {
      if (server_reap(sv, false) || server_launch(ix, sv)) return -1;
    }
  }
  // wait for the answer: spin briefly, then sleep between looks -- callers
  // may outnumber the cores, and a spinning waiter must not keep a caller
  // that holds an unposted ticket (and every ticket behind it) off its core
  const auto t0 = std::chrono::steady_clock::now();
  auto checked = t0;
  for (uint64_t spin = 1;; spin++) {
    if (__atomic_load_n(&r->seq, __ATOMIC_ACQUIRE) == t + 1u) break;
    if (spin < 2048) {
      _mm_pause();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (spin >= 2048 || (spin & 255) == 0) {
      const auto now = std::chrono::steady_clock::now();
      if (now - checked > std::chrono::microseconds(500)) {
        checked = now;
        // the grid left before this ticket was published: the next one
        std::lock_guard<std::mutex> lk(sv->mu);
        if (__atomic_load_n(&r->seq, __ATOMIC_ACQUIRE) != t + 1u && !server_running(sv)) {
          if (server_reap(sv, false) || server_launch(ix, sv)) return -1;
        }
      }
      if (now - t0 > std::chrono::seconds(60)) return fail("ngt_amd_search_served: no answer from the serving grid");
    }
  }
  if (r->err)
    return fail("ngt_amd_search_served: device error flag %u (%s)", r->err, device_error_text((int)r->err).c_str());
  const uint32_t nr = std::min(r->n, prm->k);
  memcpy(ids, r->ids, 4ull * nr);
  memcpy(dists, r->dists, 4ull * nr);
  *n = nr;
  if (counters) memcpy(counters, r->counters, sizeof r->counters);
  sv->served++;
  return 0;
}

extern "C" int ngt_amd_serve_stop(ngt_amd_index* ix) {
  if (!ix) return fail("ngt_amd_serve_stop: null index");
  Server* sv;
  {
    std::lock_guard<std::mutex> lk(ix->mu);
    sv = ix->serve;
  }
  if (!sv) return 0;
  HIP_OK(hipSetDevice(ix->device));
  std::lock_guard<std::mutex> lk(sv->mu);
  return server_reap(sv, true);
}

extern "C" int ngt_amd_serve_stats(ngt_amd_index* ix, uint64_t* served, uint64_t* launches) {
  if (!ix || !served || !launches) return fail("ngt_amd_serve_stats: bad arguments");
  std::lock_guard<std::mutex> lk(ix->mu);
  Server* sv = ix->serve.load();
  *served = sv ? sv->served.load() : 0;
  *launches = sv ? sv->launches.load() : 0;
  return 0;
}
