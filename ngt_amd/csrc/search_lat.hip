// search_lat.hip -- the latency form of NeighborhoodGraph::searchReadOnlyGraph
// (lib/NGT/Graph.cpp:398-495) for launches of a few queries per CU: single
// ngt_search_index calls (Capi.cpp:377-406), coalesced C-API batches and
// construction batches.  One workgroup serves one query and owns its CU:
//
//  * wave 0 COMMITS: it pops the unchecked set in the reference's order,
//    marks visited ids, accepts neighbours (Graph.cpp:462-483) and keeps the
//    results -- the sequential part, all in registers and LDS;
//  * waves 1..W-1 SPECULATE: the commit wave hands them the nodes at the
//    front of the unchecked set, and they evaluate each node's neighbour list
//    ahead of its pop (adjacency row, 1-byte filter codes, exact f32 rows of
//    the neighbours the bound cannot reject) into an LDS slot.
//
// The commit wave therefore waits on memory only when it pops a node nobody
// has evaluated yet (typically one just accepted).  Why the result is the
// reference's:
//  * a neighbour's distance does not depend on the search state: the slot
//    holds the comparator's exact value (eval as PrimitiveComparator::compareL2
//    through l2_fold_rows) or +inf when the filter bound proves it larger than
//    the exploration radius at speculation time -- which only shrinks, so the
//    reference rejects it at commit time too;
//  * the visited set is an exact bitmap of every evaluated id in LDS (one bit
//    per object), tested and marked only by the commit wave in pop order;
//    the speculation waves drop neighbours already visited when they read the
//    list (visited bits are never cleared during a query), every other
//    neighbour is re-tested at commit;
//  * the unchecked set is exact: a sorted head of the 64 smallest keys in the
//    commit wave's registers (lane i = i-th smallest), an unsorted LDS tail of
//    larger keys and an HBM spill of larger ones still (threshold T).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ngt_device.h"
#include "ngt_kernels.h"
#include "search_common.h"

namespace ngt_amd {

namespace {

constexpr uint32_t kNoTag = 0xffu;  // head entry without a slot
constexpr uint32_t kFree = 0u, kIssued = 1u;

struct LatCtl {
  uint32_t done;  // the commit wave has finished the query
  uint32_t qi;
  uint32_t quit;  // serving form: no more work for this workgroup
  uint32_t k;     // this query's SearchContainer::size, coefficient, radius
  float coef;
  float radius;
  float expr;     // the commit wave's exploration radius (read by the hop prefetch)
  uint32_t ns;    // serving form: seeds staged in the tail
  uint64_t sp[4]; // diagnostic build: speculation-wave cycles ([0] adjacency, [2] exact rows)
};

// one node's speculation: key (its unchecked-set key, the priority), state,
// the claim word of its list parts (generation << 8 | parts taken), parts
// finished, list length, fresh entries per part
struct LatSlot {
  uint64_t key;
  uint32_t state;
  uint32_t claim;
  uint32_t pready; // parts finished (bit p: part p's entries and count are final)
  uint32_t deg;    // list length read (getEdgeSize cap), summed over the parts
  uint32_t pn[8];  // neighbours not yet visited when the part was read
};

struct LatLayout {
  uint32_t off_slot, off_eid, off_ed, off_tail, off_q, off_nid, off_nd, off_hist, off_bm,
      total;
  __host__ __device__ static uint32_t up16(uint32_t v) { return (v + 15u) & ~15u; }
  __host__ __device__ LatLayout(const SearchArgs& a, uint32_t cap, uint32_t waves) {
    uint32_t o = up16(sizeof(LatCtl));
    const uint32_t ns = a.lat_slots;
    off_slot = o; o = up16(o + sizeof(LatSlot) * ns);
    off_eid = o; o = up16(o + 4u * ns * cap);
    off_ed = o; o = up16(o + 4u * ns * cap);
    off_tail = o; o = up16(o + 8u * a.lat_tail);
    off_q = o; o = up16(o + 4u * (uint32_t)a.dp);
    off_nid = o; o = up16(o + 256u);
    off_nd = o; o = up16(o + 256u);
    off_hist = o; o = up16(o + 256u);
    off_bm = o; o = up16(o + 4u * ((a.nrows + 31u) / 32u));
    total = o;
  }
};

__device__ __forceinline__ bool bm_test(const uint32_t* bm, uint32_t id) { return (bm[id >> 5] >> (id & 31)) & 1u; }

__device__ __forceinline__ float wave_min_f32(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float lds_load_f32(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP));
}

__device__ __forceinline__ uint32_t lds_load_acq(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---- serving form (ngt_kernels.h ServeArgs) ---------------------------------
// The dispatcher (one lane of block 0): publishes each ticket whose
// request slot the host has posted, in ticket order, until the host asks it
// to stop, nothing was posted or in flight for idle_ticks, or life_ticks have
// passed; then tells the workers to drain.  The idle time counts from the
// last answer, not the last post: a lone caller's search that outlasts
// idle_ticks would otherwise close the grid under it, and its next call
// would pay a relaunch.
__device__ void serve_dispatch(const ServeArgs& sv) {
  if (lane_id() != 0) return;
  uint32_t avail = sv.start;
  const uint64_t t0 = wall_clock64();
  uint64_t last = t0;
  uint32_t why = 0;  // 1 asked to stop, 2 idle, 3 lifetime
  for (;;) {
    const uint64_t now = wall_clock64();
    // a posted ticket not answered yet: not idle
    if (__hip_atomic_load(&sv.dctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != avail) last = now;
    if (__hip_atomic_load(sv.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) why = 1;
    // idle: nothing posted for idle_ticks and no ticket handed out unposted
    // (a caller between taking its ticket and posting it)
    else if (now - last > sv.idle_ticks &&
             __hip_atomic_load(sv.stop + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == avail)
      why = 2;
    else if (now - t0 > sv.life_ticks) why = 3;
    if (why) break;
    const ServeReqHdr* h = reinterpret_cast<const ServeReqHdr*>(sv.ring + (uint64_t)(avail % sv.nring) * sv.req_bytes);
    // polled relaxed, acquired once per ticket: an acquire at agent or
    // system scope invalidates caches, and a poll loop issuing one every few
    // hundred cycles would keep flushing the lines the searching workers of
    // this XCD are warming
    if (__hip_atomic_load(&h->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == avail + 1u) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      avail++;
      __hip_atomic_store(&sv.dctl->avail, avail, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      last = now;
      continue;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  __hip_atomic_store(&sv.dctl->pad, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&sv.dctl->closing, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// A worker's next ticket (returns false when it should leave): tickets
// below `avail` are claimed in order; once the dispatcher closes, `avail` is
// final.  Workers also leave on their own after life + idle + 1 s, so a grid
// whose dispatcher block never got a CU still drains.
__device__ bool serve_claim(const ServeArgs& sv, uint64_t t0, uint32_t& ticket) {
  // idle workers back off (all of them poll the same control line); the polls
  // are relaxed, as in serve_dispatch: the successful claim's CAS is the
  // acquire, and it reads `avail`'s release by the dispatcher
  for (uint32_t idle = 0;; idle++) {
    uint32_t c = __hip_atomic_load(&sv.dctl->claimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t av = __hip_atomic_load(&sv.dctl->avail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int32_t)(av - c) > 0) {
      if (__hip_atomic_compare_exchange_strong(&sv.dctl->claimed, &c, c + 1u, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        ticket = c;
        return true;
      }
      continue;
    }
    if (__hip_atomic_load(&sv.dctl->closing, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const uint32_t av2 = __hip_atomic_load(&sv.dctl->avail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t c2 = __hip_atomic_load(&sv.dctl->claimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int32_t)(av2 - c2) > 0) continue;
      return false;
    }
    if (wall_clock64() - t0 > sv.life_ticks + sv.idle_ticks + 100000000ull) return false;
    if (idle < 16) __builtin_amdgcn_s_sleep(2);
    else if (idle < 256) __builtin_amdgcn_s_sleep(8);
    else __builtin_amdgcn_s_sleep(32);
  }
}

// GraphAndTreeIndex::getSeedsFromTree for the serving form, on one wave: the
// DVPTree leaf-mode descent (Tree.cpp:400-480, 531-563) and the leaf's
// thinning (Index.h:1555-1562), as ngt_tree_seed_kernel does for a batch.
// Leaf ids land in out[0, n) (LDS); returns n.
__device__ uint32_t serve_tree_seeds(const TreeSeedArgs& t, const float* qlds, int dp, uint32_t k, uint32_t* out) {
  const int lane = lane_id();
  uint32_t node = t.root;
  while (!(node & 0x80000000u)) {
    const uint32_t iid = node & 0x7fffffffu;
    float d = 0.f;
    if (lane < 4) d = quad_distance<kL2, float>(qlds, row_ptr<float>(t.in_pivot, t.row_bytes, iid), dp, lane);
    d = __shfl(d, 0, 64);
    const float* borders = t.in_border + (uint64_t)iid * (t.children - 1);
    uint32_t mid = 0;
    for (; mid < t.children - 1; mid++)
      if (d < borders[mid]) break;
    node = t.in_child[(uint64_t)iid * t.children + mid];
  }
  const uint32_t lid = node & 0x7fffffffu;
  const uint64_t b = t.leaf_off[lid];
  uint32_t n = (uint32_t)(t.leaf_off[lid + 1] - b);
  if (n > kServeMaxSeeds) n = kServeMaxSeeds;
  for (uint32_t i = lane; i < n; i += 64) out[i] = t.leaf_ids[b + i];
  __threadfence_block();
  uint32_t ss = t.seed_size == 0 ? k : t.seed_size;
  if (ss > k) ss = k;
  if (t.all_leaf_nodes) ss = n;
  if (n > ss) {
    if (lane == 0) {
      GlibcRand rnd;
      rnd.seed(lid);
      for (uint32_t i = n; i > ss; i--) {
        const double random = ((double)rnd.next() + 1.0) / ((double)2147483647 + 2.0);
        const uint32_t idx = (uint32_t)floor((double)i * random);
        out[idx] = out[i - 1];
      }
    }
    __threadfence_block();
    n = ss;
  }
  return n;
}

}  // namespace

// NCH = dp / 16; W waves (1 commit + W-1 speculation).  A list of up to
// `cap` ids is speculated as `parts` parts of 32 entries, each taken by one
// speculation wave: its adjacency ids, then the exact rows of its fresh
// neighbours (EG groups of 16 rows in flight) -- two dependent round trips.
// SERVE: the resident serving form (queries from sv's ring, answers to its
// response slots); otherwise one launch over a.nq prepared queries.
template <int NCH, int W, bool SERVE>
__global__ void __launch_bounds__(64 * W) ngt_graph_search_lat_kernel(SearchArgs a, ServeArgs sv) {
  constexpr int EG = 2;
  if constexpr (SERVE) {
    // the dispatcher is block 0, so it is placed first even when the grid
    // (one workgroup per CU) has more blocks than free CUs
    if (blockIdx.x == 0) {
      if (threadIdx.x < 64) serve_dispatch(sv);
      return;
    }
  }
  const uint64_t t_start = SERVE ? wall_clock64() : 0ull;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t cap = (uint32_t)(a.adj_stride < a.edge_size ? a.adj_stride : a.edge_size);
  constexpr uint32_t span = 32u;  // ids per part: one group of EG x 16 rows
  const uint32_t parts = (cap + span - 1u) / span;  // <= 8
  const uint32_t pfull = (1u << parts) - 1u;        // every part finished
  // the parts a commit pass reads: p and p + 1 (when there is one)
  auto pmask = [&](uint32_t p) -> uint32_t { return pfull & (3u << p); };
  const LatLayout lay(a, cap, W);
  LatCtl* ctl = reinterpret_cast<LatCtl*>(smem);
  LatSlot* slots = reinterpret_cast<LatSlot*>(smem + lay.off_slot);
  uint32_t* eid = reinterpret_cast<uint32_t*>(smem + lay.off_eid);
  float* ed = reinterpret_cast<float*>(smem + lay.off_ed);
  uint64_t* tail = reinterpret_cast<uint64_t*>(smem + lay.off_tail);
  float* qlds = reinterpret_cast<float*>(smem + lay.off_q);
  uint32_t* nid = reinterpret_cast<uint32_t*>(smem + lay.off_nid);
  float* nd = reinterpret_cast<float*>(smem + lay.off_nd);
  uint32_t* bm = reinterpret_cast<uint32_t*>(smem + lay.off_bm);
  // threshold-selection counters: not nid/nd, which hold the accept step's
  // staged candidates when a full tail makes room in the middle of it
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + lay.off_hist);

  const int lane = lane_id();
  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t NT = 64u * W;
  const uint32_t bm_words = (a.nrows + 31u) / 32u;
  const uint32_t nslots = a.lat_slots;  // speculation slots, issued by the commit wave
  const uint32_t wg = SERVE ? blockIdx.x - 1u : blockIdx.x;  // serving: workers are blocks 1..workers
  uint64_t* spill = a.spill + (uint64_t)wg * a.spill_cap;
  const int g = lane & 3, rs = lane >> 2;

  for (;;) {
    if (tid == 0) {
      if constexpr (SERVE) {
        uint32_t t = 0;
        ctl->quit = serve_claim(sv, t_start, t) ? 0u : 1u;
        ctl->qi = t;
      } else {
        ctl->qi = atomicAdd(a.work, 1u);
        ctl->quit = 0u;
      }
    }
    __syncthreads();
    const uint32_t qi = ctl->qi;
    if (SERVE ? ctl->quit != 0u : qi >= a.nq) break;
    // the serving form's request slot (pinned host memory, posted before its
    // ticket was published: acquire at system scope before reading it)
    const uint8_t* req = SERVE ? sv.ring + (uint64_t)(qi % sv.nring) * sv.req_bytes : nullptr;
    if constexpr (SERVE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

    // ---- per-query init (every wave) -------------------------------------
    {
      uint4* b4 = reinterpret_cast<uint4*>(bm);
      for (uint32_t i = tid; i < (bm_words + 3) / 4; i += NT) b4[i] = make_uint4(0, 0, 0, 0);
      const uint4* s = reinterpret_cast<const uint4*>(SERVE ? req + kServeQueryOff
                                                            : a.queries + (uint64_t)qi * a.query_bytes);
      uint4* d = reinterpret_cast<uint4*>(qlds);
      for (uint32_t i = tid; i < (uint32_t)a.dp / 4; i += NT) d[i] = s[i];
      for (uint32_t i = tid; i < nslots; i += NT) {
        slots[i].state = kFree;
        slots[i].claim = 0u;
        slots[i].pready = 0u;
      }
      if (tid == 0) {
        ctl->done = 0u;
        // no hop prefetch before this query's first set_expr (the speculation
        // waves read it atomically; +inf would let a stale query's radius in)
        __hip_atomic_store(&ctl->expr, -1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ctl->sp[0] = ctl->sp[1] = ctl->sp[2] = ctl->sp[3] = 0ull;
        if constexpr (SERVE) {
          const ServeReqHdr* h = reinterpret_cast<const ServeReqHdr*>(req);
          ctl->k = h->k;
          ctl->coef = h->coef;
          ctl->radius = h->radius;
          ctl->ns = h->ns;
        } else {
          ctl->k = a.k;
          ctl->coef = a.coef;
          ctl->radius = a.radius;
        }
      }
      // the request's random seeds, staged in the (still empty) tail
      if constexpr (SERVE) {
        if (!sv.use_tree)
          for (uint32_t i = tid; i < kServeMaxSeeds; i += NT)
            reinterpret_cast<uint32_t*>(tail)[i] = reinterpret_cast<const uint32_t*>(req + 32)[i];
      }
    }
    __syncthreads();
    const uint32_t k = ctl->k;
    const float coefq = ctl->coef, radq = ctl->radius;

    if (wave == 0) {
      // =================== the commit wave ===================================
      uint32_t nres = 0, maxq = 0;
      // the result set (Graph.cpp:471-483's ResultSet, k <= 64) in registers:
      // lane i holds the i-th smallest (distance, id) key
      uint64_t rk = ~0ull;
      auto res_push = [&](uint64_t key) {
        const uint32_t pos = (uint32_t)__popcll(ballot64((uint32_t)lane < nres && rk < key));
        if (pos >= k) return;
        const uint64_t up = wave_up1_u64(rk);
        if ((uint32_t)lane > pos) rk = up;
        if ((uint32_t)lane == pos) rk = key;
        nres = nres + 1 < k ? nres + 1 : k;
      };
      uint32_t ndist = 0, nexp = 0, nedge = 0, nexact = 0, nwait = 0, ns = 0, nstall = 0;
      (void)nwait;
      // diagnostic build only: shader-clock totals per phase
      uint64_t t_pop = 0, t_wait = 0, t_list = 0, t_acc = 0, t_feed = 0, t_last = 0;
      (void)t_pop; (void)t_wait; (void)t_list; (void)t_acc; (void)t_feed; (void)t_last;
      float radius = radq;
      uint32_t qerr = 0;  // the batch kernel's error bits, this query's
      float expr = 0.f;
      auto set_expr = [&]() {
        expr = __fmul_rn(coefq, radius);
        if (lane == 0) __hip_atomic_store(&ctl->expr, expr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      };
      // unchecked set: head (registers, sorted, hn keys) < B <= tail (LDS,
      // ntail keys) < T <= spill (HBM, nspill keys)
      uint64_t hk = ~0ull;
      uint32_t ht = kNoTag;
      uint32_t hn = 0, ntail = 0, nspill = 0;
      uint64_t B = ~0ull, T = ~0ull;
      uint64_t freem = nslots >= 64 ? ~0ull : ((1ull << nslots) - 1ull);  // free slots
      uint32_t sgen = 0u;  // lane s: slot s's issue generation (only this wave issues)
      uint64_t orphan = 0ull;                                             // issued, no longer in the head
      const uint32_t Fd = a.lat_feed ? a.lat_feed : 16u;
      const uint32_t F = nslots < Fd ? nslots : Fd;                       // head entries kept speculated

      auto spill_push = [&](uint64_t key) {
        if (nspill >= a.spill_cap) {
          qerr |= 1u;
        } else {
          if (lane == 0) spill[nspill] = key;
          nspill++;
        }
      };
      auto select_t = [&](const uint64_t* arr, uint32_t n, uint32_t M, uint64_t lim) -> uint64_t {
        return lat_select(arr, n, M, lim, hist);
      };
      // the tail is full: drop keys beyond the exploration radius (never
      // popped, Graph.cpp:433-435); if still over half full, move the keys
      // from a threshold up to the spill (T drops)
      auto tail_room = [&]() {
        uint32_t out = 0;
        for (uint32_t b0 = 0; b0 < ntail; b0 += 64) {
          const uint32_t i = b0 + (uint32_t)lane;
          const uint64_t key = i < ntail ? tail[i] : ~0ull;
          const bool keep = i < ntail && key_dist(key) <= expr;
          const uint64_t km = ballot64(keep);
          __builtin_amdgcn_wave_barrier();
          if (keep) tail[out + mbcnt(km)] = key;
          __builtin_amdgcn_wave_barrier();
          out += (uint32_t)__popcll(km);
        }
        ntail = out;
        const uint32_t keep = a.lat_tail / 2;
        if (ntail <= keep) return;
        const uint64_t l = select_t(tail, ntail, keep, ~0ull);
        out = 0;
        for (uint32_t b0 = 0; b0 < ntail; b0 += 64) {
          const uint32_t i = b0 + (uint32_t)lane;
          const uint64_t key = i < ntail ? tail[i] : ~0ull;
          const bool mv = i < ntail && key >= l;
          const bool kp = i < ntail && key < l;
          const uint64_t mm = ballot64(mv), km = ballot64(kp);
          const uint32_t nm = (uint32_t)__popcll(mm);
          if (nspill + nm > a.spill_cap) {
            qerr |= 1u;
          } else if (mv) {
            spill[nspill + mbcnt(mm)] = key;
          }
          if (nspill + nm <= a.spill_cap) nspill += nm;
          __builtin_amdgcn_wave_barrier();
          if (kp) tail[out + mbcnt(km)] = key;
          __builtin_amdgcn_wave_barrier();
          out += (uint32_t)__popcll(km);
        }
        if (out == 0u || out > keep) qerr |= 32u;  // selection check
        ntail = out;
        T = l;
      };
      auto tail_push = [&](uint64_t key) {
        if (key >= T) {
          spill_push(key);
        } else {
          if (ntail >= a.lat_tail) tail_room();
          if (key >= T) {
            spill_push(key);
          } else {
            if (lane == 0) tail[ntail] = key;
            ntail++;
          }
        }
        __builtin_amdgcn_wave_barrier();
      };
      // an issued head entry leaving the head: its slot is freed once ready
      auto orphan_tag = [&](uint32_t tag) {
        if (tag != kNoTag) orphan |= 1ull << tag;
      };
      auto insert_key = [&](uint64_t key) {
        if (key < B) {
          const uint32_t pos = (uint32_t)__popcll(ballot64((uint32_t)lane < hn && hk < key));
          if (hn == 64u) {
            // the head is full: its largest key (or this one) moves to the tail
            if (pos == 64u) {
              B = key;
              tail_push(key);
              return;
            }
            const uint64_t e = readlane_u64(hk, 63);
            orphan_tag((uint32_t)__builtin_amdgcn_readlane((int)ht, 63));
            const uint64_t uk = wave_up1_u64(hk);
            const uint32_t ut = wave_up1(ht);
            if ((uint32_t)lane > pos) { hk = uk; ht = ut; }
            if ((uint32_t)lane == pos) { hk = key; ht = kNoTag; }
            B = e;
            tail_push(e);
          } else {
            const uint64_t uk = wave_up1_u64(hk);
            const uint32_t ut = wave_up1(ht);
            if ((uint32_t)lane > pos && (uint32_t)lane <= hn) { hk = uk; ht = ut; }
            if ((uint32_t)lane == pos) { hk = key; ht = kNoTag; }
            hn++;
          }
        } else {
          tail_push(key);
        }
        const uint32_t q = hn + ntail + nspill;
        if (q > maxq) maxq = q;
      };
      // an empty head takes the smallest keys of the tail (the tail the
      // smallest of the spill first): a histogram threshold that moves 32..64
      // keys, then a bitonic sort across the lanes
      auto refill_tail = [&]() {
        // nothing in LDS: the smallest spill keys within the radius move in,
        // the ones beyond it are dropped
        const uint32_t want = a.lat_tail / 2;
        const uint64_t lim = ((uint64_t)ord_of(expr) << 32) | 0xffffffffull;
        const uint64_t l = select_t(spill, nspill, want, lim);
        if (l == 0ull) {  // nothing within the radius: the search ends
          nspill = 0;
          T = ~0ull;
          return;
        }
        uint32_t out = 0;
        for (uint32_t b0 = 0; b0 < nspill; b0 += 64) {
          const uint32_t i = b0 + (uint32_t)lane;
          const uint64_t key = i < nspill ? spill[i] : ~0ull;
          const bool in = i < nspill && key <= lim;
          const bool mv = in && key < l;
          const bool st = in && !mv;
          const uint64_t mm = ballot64(mv), sm = ballot64(st);
          __builtin_amdgcn_wave_barrier();
          if (mv) tail[ntail + mbcnt(mm)] = key;
          if (st) spill[out + mbcnt(sm)] = key;
          __builtin_amdgcn_wave_barrier();
          ntail += (uint32_t)__popcll(mm);
          out += (uint32_t)__popcll(sm);
        }
        nspill = out;
        T = nspill ? l : ~0ull;
        if (ntail == 0u || ntail > want) qerr |= 64u;  // selection check
      };
      auto refill_head = [&]() {
        if (ntail == 0 && nspill != 0) refill_tail();
        if (ntail == 0) return;
        // the (at most 64, at least 32 when there are) smallest tail keys
        const uint64_t t = select_t(tail, ntail, 64u, ~0ull);
        // move tail keys < t into the head lanes (unsorted), compact the tail
        uint64_t v = ~0ull;
        uint32_t got = 0, out = 0;
        for (uint32_t b0 = 0; b0 < ntail; b0 += 64) {
          const uint32_t i = b0 + (uint32_t)lane;
          const uint64_t key = i < ntail ? tail[i] : ~0ull;
          const bool mv = i < ntail && key < t;
          const bool kp = i < ntail && !mv;
          const uint64_t mm = ballot64(mv), km = ballot64(kp);
          // lane (got + rank) of the head receives the key
          const uint32_t dst = got + mbcnt(mm);
          uint32_t* stage = nid;  // 64 x u64 staged through nid/nd (adjacent 256 B each)
          uint64_t* st64 = reinterpret_cast<uint64_t*>(stage);
          __builtin_amdgcn_wave_barrier();
          if (mv) st64[dst] = key;
          if (kp) tail[out + mbcnt(km)] = key;
          __builtin_amdgcn_wave_barrier();
          got += (uint32_t)__popcll(mm);
          out += (uint32_t)__popcll(km);
        }
        {
          const uint64_t* st64 = reinterpret_cast<const uint64_t*>(nid);
          v = (uint32_t)lane < got ? st64[lane] : ~0ull;
        }
        ntail = out;
        if (got == 0u || got > 64u) qerr |= 128u;  // selection check
        // bitonic sort of the 64 lanes (ascending; empty lanes hold ~0)
#pragma unroll
        for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
          for (int j = kk >> 1; j > 0; j >>= 1) {
            const uint64_t o = shfl_xor_u64(v, j);
            const bool up = ((lane & kk) == 0);
            const bool lower = (lane & j) == 0;
            const uint64_t mn = o < v ? o : v, mx = o < v ? v : o;
            v = (lower == up) ? mn : mx;
          }
        }
        hk = v;
        ht = kNoTag;
        hn = got;
        B = (ntail + nspill) ? readlane_u64(hk, (int)got - 1) + 1 : ~0ull;
      };
      auto pop = [&](uint64_t& key, uint32_t& tag) -> bool {
        if (hn == 0) refill_head();
        if (hn == 0) return false;
        key = readlane_u64(hk, 0);
        tag = (uint32_t)__builtin_amdgcn_readlane((int)ht, 0);
        const uint64_t dk = wave_down1_u64(hk);
        const uint32_t dt = wave_down1(ht);
        hk = (uint32_t)lane < hn - 1 ? dk : ~0ull;
        ht = (uint32_t)lane < hn - 1 ? dt : kNoTag;
        hn--;
        return true;
      };
      // a slot the commit wave is done with goes back to freem
      auto release_slot = [&](uint32_t t) {
        if (lane == 0) slots[t].state = kFree;
        freem |= 1ull << t;
      };
      // free the orphaned slots whose speculation has finished
      auto reap = [&]() {
        uint64_t o = orphan;
        while (o) {
          const int s = __ffsll((long long)o) - 1;
          o &= o - 1;
          if (lds_load_acq(&slots[s].pready) == pfull) {
            release_slot((uint32_t)s);
            orphan &= ~(1ull << s);
          }
        }
      };
      // hand a node to the speculation waves (they take the issued slot of
      // the smallest key first: the commit wave's next pops)
      // every wait below is bounded: a slot that never becomes ready (never
      // expected) flags error 16 and ends the query instead of hanging the CU
      bool stuck = false;
      auto issue = [&](uint64_t key) -> uint32_t {
        if (freem == 0ull && orphan == 0ull) {
          // every slot is held by a head entry (tagged entries pushed past the
          // first F lanes by smaller accepted keys, then F more tagged), and
          // the node to expand has none: nothing comes back to freem by
          // itself, so the deepest tagged head entry gives its slot up
          // (orphaned, freed once its speculation is done; the entry is
          // issued again when it nears the front)
          const uint64_t om = ballot64(ht < nslots);
          if (om != 0ull) {
            const int l = 63 - __builtin_clzll(om);
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)ht, l);
            if (lane == l) ht = kNoTag;
            orphan |= 1ull << t;
          }
        }
        for (uint32_t spin = 0; freem == 0ull; spin++) {
          reap();
          if (freem != 0ull) break;
          if (spin > (1u << 24)) {
            qerr |= 16u;
            stuck = true;
            return 0u;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t s = (uint32_t)(__ffsll((long long)freem) - 1);
        freem &= ~(1ull << s);
        const uint32_t gen = ((uint32_t)__builtin_amdgcn_readlane((int)sgen, (int)s) + 1u) & 0xffffffu;
        if ((uint32_t)lane == s) sgen = gen;
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
          slots[s].key = key;
          slots[s].pready = 0u;
          slots[s].deg = 0u;
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
          // released on its own as well: a speculation wave that CASes this
          // word (having read the slot's previous kIssued state) acquires
          // the key written above through it
          __hip_atomic_store(&slots[s].claim, gen << 8, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          lds_store_rel(&slots[s].state, kIssued);
        }
        return s;
      };
      // speculation for the first F head entries that have none
      auto feed = [&]() {
        if (orphan) reap();
        uint64_t need = ballot64((uint32_t)lane < (hn < F ? hn : F) && ht == kNoTag);
        while (need) {
          const int l = __ffsll((long long)need) - 1;
          need &= need - 1;
          const uint64_t key = readlane_u64(hk, l);
          if (freem == 0ull) break;
          const uint32_t s = issue(key);
          if (stuck) break;
          if (lane == l) ht = s;
        }
      };
      // accept the candidates held in registers in neighbour order
      // (Graph.cpp:471-483), the sequential outcome exactly: lanes of `cmask`
      // (neighbour order = lane order), ids in idv, distances in dv -- no LDS
      // staging on the commit path
      auto accept_reg = [&](uint64_t cmask, uint32_t idv, float dv) {
        auto push = [&](uint64_t m) {
          while (m) {
            const int j = __ffsll((long long)m) - 1;
            m &= m - 1;
            insert_key(make_key(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(dv), j)),
                                (uint32_t)__builtin_amdgcn_readlane((int)idv, j)));
          }
        };
        uint64_t okmask = cmask & ballot64(dv <= expr);
        while (okmask) {
          const uint64_t rmask = okmask & ballot64(dv <= radius);
          if (rmask == 0ull) {
            push(okmask);
            break;
          }
          const int j = __ffsll((long long)rmask) - 1;
          push(okmask & ((1ull << j) - 1ull));
          const uint64_t key = make_key(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(dv), j)),
                                        (uint32_t)__builtin_amdgcn_readlane((int)idv, j));
          insert_key(key);
          res_push(key);
          if (nres >= k) {
            radius = key_dist(readlane_u64(rk, (int)k - 1));
            set_expr();
          }
          __builtin_amdgcn_wave_barrier();
          okmask &= ~((2ull << j) - 1ull);
          okmask &= ballot64(dv <= expr);
        }
      };

      // ---- setupDistances + setupSeeds (Graph.cpp:293-367) ----------------
      // (the serving form's seeds sit in the tail: the head takes the first 64
      // keys, so no key reaches the tail before the last chunk is read)
      uint64_t sb = 0;
      const uint32_t* sp;
      if constexpr (SERVE) {
        sp = reinterpret_cast<const uint32_t*>(tail);
        ns = sv.use_tree ? serve_tree_seeds(sv.tree, qlds, a.dp, k, reinterpret_cast<uint32_t*>(tail)) : ctl->ns;
      } else {
        sb = a.seed_off ? a.seed_off[qi] : (uint64_t)qi * a.seed_stride;
        ns = a.seed_off ? (uint32_t)(a.seed_off[qi + 1] - sb) : a.seed_count[qi];
        sp = a.seeds;
      }
      set_expr();
      for (uint32_t base = 0; base < ns; base += 64) {
        const uint32_t m = ns - base < 64 ? (uint32_t)(ns - base) : 64u;
        if ((uint32_t)lane < m) nid[lane] = sp[sb + base + lane];
        __builtin_amdgcn_wave_barrier();
        eval_l2f_fast<NCH, 1>(qlds, a.rows, a.row_bytes, nid, nd, (int)m);
        __builtin_amdgcn_wave_barrier();
        if ((uint32_t)lane < m) {
          const uint32_t id = nid[lane];
          atomicOr(bm + (id >> 5), 1u << (id & 31));
        }
        __builtin_amdgcn_wave_barrier();
        for (uint32_t j = 0; j < m; j++) {
          const float d = nd[j];
          const uint64_t key = make_key(d, nid[j]);
          insert_key(key);
          if (d <= radq) res_push(key);
        }
        __builtin_amdgcn_wave_barrier();
      }
      ndist = ns;
      if (nres >= k) radius = key_dist(readlane_u64(rk, (int)k - 1));
      set_expr();
      feed();

      // ---- best-first loop (Graph.cpp:430-486) ------------------------------
#ifdef NGT_AMD_STAMPS
      t_last = stamp();
#endif
      for (;;) {
        uint64_t key;
        uint32_t tag;
        if (!pop(key, tag)) break;
        if (key_dist(key) > expr) break;  // Graph.cpp:433-435
        if (tag == kNoTag) {
          tag = issue(key);
          nwait++;
        }
        if (stuck) break;
        NGT_MARK(t_pop);
        feed();  // keep the speculation ahead while this node's list lands
        NGT_MARK(t_feed);
        // each pass waits only for its own two parts: the first parts of a
        // list are applied (and their accepts handed out) while the later
        // ones are still in flight
        uint32_t pr = lds_load_acq(&slots[tag].pready);  // reused by the first pass
        if ((pr & pmask(0u)) != pmask(0u)) nstall++;
        NGT_MARK(t_wait);
        uint32_t dg = 0u;  // the list length read, final once every part is
        nexp++;
        // the parts of the list in order, two per pass (lanes 0-31 part p,
        // 32-63 part p+1; each part compacted in list order, so lane order
        // is neighbour order): visited test, mark, then the accepts in
        // neighbour order.  Ids of one list are distinct, so testing and
        // marking them in parallel is the sequential outcome.  Speculation
        // for the accepted keys that reach the head's front is handed out
        // after every pass, not only after the list.
        {
          const uint32_t* sid = eid + tag * cap;
          const float* sd = ed + tag * cap;
          const uint32_t half = (uint32_t)lane >> 5, sub = (uint32_t)lane & 31u;
#pragma unroll 1
          for (uint32_t p = 0; p < parts; p += 2) {
            NGT_MARK(t_list);
            for (uint32_t spin = 0; (pr & pmask(p)) != pmask(p); spin++) {
              pr = lds_load_acq(&slots[tag].pready);
              if ((pr & pmask(p)) == pmask(p)) break;
              if (spin > (1u << 24)) {
                qerr |= 16u;
                stuck = true;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
            }
            if (stuck) break;
            NGT_MARK(t_wait);
            const uint32_t pp = p + half;
            // the entries are read with the count, not after it (one LDS
            // round trip; lanes past the count discard theirs)
            const uint32_t rid = pp < parts ? sid[pp * span + sub] : 0u;
            const float rdv = pp < parts ? sd[pp * span + sub] : 0.f;
            const uint32_t np = pp < parts ? slots[tag].pn[pp] : 0u;
            if (p + 2u >= parts) dg = slots[tag].deg;  // the last pass: every part is final
            const bool in = sub < np;
            const uint32_t idv = in ? rid : 0u;
            const float dv = in ? rdv : 0.f;
            const bool f = idv != 0u && !bm_test(bm, idv);
            if (f) atomicOr(bm + (idv >> 5), 1u << (idv & 31));
            const uint32_t nf = (uint32_t)__popcll(ballot64(f));
            ndist += nf;
            nexact += nf;
            const uint64_t km = ballot64(f && dv <= expr);
            if (km) {
              NGT_MARK(t_list);
              accept_reg(km, idv, dv);
              NGT_MARK(t_acc);
              if (p + 2u < parts) feed();
              NGT_MARK(t_feed);
            }
          }
        }
        if (stuck) break;
        nedge += dg;
        release_slot(tag);
        NGT_MARK(t_list);
        feed();
        NGT_MARK(t_feed);
      }
      // the speculation waves leave once every issued slot is done
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) lds_store_rel(&ctl->done, 1u);

      // ---- results (moveFrom: ascending (distance, id), ObjectSpace.h:49-57)
      uint64_t cv[8] = {ndist, ndist - ns, nexp, nstall, nedge, maxq, nexact, ns};
#ifdef NGT_AMD_STAMPS
      // phase cycles: [5] pop (+ refills, issue), [6] waits for list parts,
      // [1] list reads + visited test and mark, [3] accepts, [7] feeding the
      // speculation; the speculation waves' sums: [0] adjacency + visited
      // pre-test, [2] exact rows
      __builtin_amdgcn_s_waitcnt(0);
      cv[5] = t_pop;
      cv[6] = t_wait;
      cv[1] = t_list;
      cv[7] = t_feed;
      cv[3] = t_acc;
      cv[0] = ctl->sp[0];
      cv[4] = ctl->sp[1];
      cv[2] = ctl->sp[2];
#endif
      if constexpr (SERVE) {
        // the answer, then its ticket (system-scope release: the caller polls
        // the slot in host memory)
        ServeResp* r = sv.resp + (qi % sv.nring);
        if ((uint32_t)lane < nres) {
          r->ids[lane] = key_id(rk);
          r->dists[lane] = key_dist(rk);
        }
        if (lane == 0) {
          r->n = nres;
          r->err = qerr;
#pragma unroll
          for (int i = 0; i < 8; i++) r->counters[i] = cv[i];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (lane == 0) {
          __hip_atomic_store(&r->seq, qi + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_fetch_add(&sv.dctl->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        if ((uint32_t)lane < nres) {
          a.out_ids[(uint64_t)qi * k + lane] = key_id(rk);
          a.out_dists[(uint64_t)qi * k + lane] = key_dist(rk);
        }
        if (lane == 0) {
          a.out_n[qi] = nres;
          if (qerr) atomicOr(a.error, (int)qerr);
          if (a.counters) {
            uint64_t* c = a.counters + (uint64_t)qi * 8;
#pragma unroll
            for (int i = 0; i < 8; i++) c[i] = cv[i];
          }
        }
      }
    } else {
      // =================== speculation waves =================================
      for (;;) {
        if (lds_load_acq(&ctl->done)) break;
        // the issued slot with the smallest key
        const uint32_t st = (uint32_t)lane < nslots ? lds_load_acq(&slots[lane].state) : kFree;
        const uint32_t cw = (uint32_t)lane < nslots ? lds_load_acq(&slots[lane].claim) : 0u;
        const uint64_t cand = st == kIssued && (cw & 0xffu) < parts ? slots[lane].key : ~0ull;
        const uint64_t m = uniform_u64_lat(wave_min_u64(cand));
        if (m == ~0ull) {
          if (lds_load_acq(&ctl->done)) break;
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const int sl = __ffsll((long long)ballot64(cand == m)) - 1;
        // claim the next part of that list: CAS on (generation, parts taken),
        // so a claim from before the slot's reissue cannot succeed
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)cw, sl);
        uint32_t got = 0;
        if (lane == 0) {
          uint32_t expect = w;
          got = __hip_atomic_compare_exchange_strong(&slots[sl].claim, &expect, w + 1u, __ATOMIC_ACQUIRE,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ? 1u : 0u;
        }
        if (!__builtin_amdgcn_readfirstlane((int)got)) continue;  // another wave took it
        const uint32_t part = w & 0xffu;
        const uint32_t node = key_id(slots[sl].key);
#ifdef NGT_AMD_STAMPS
        uint64_t st0 = stamp();
#endif
        // this part's adjacency ids (the first min(degree, edgeSize) of the
        // list, Graph.cpp:436-439) and the ones not visited yet, in order
        const uint32_t p0 = part * span;
        const uint32_t len = cap - p0 < span ? cap - p0 : span;
        const uint32_t id = (uint32_t)lane < len ? a.adj[(uint64_t)node * a.adj_stride + p0 + lane] : 0u;
        const uint32_t live = (uint32_t)__popcll(ballot64(id != 0u));
        const bool fresh = id != 0u && !bm_test(bm, id);
        const uint64_t fm = ballot64(fresh);
        const uint32_t np = (uint32_t)__popcll(fm);
        uint32_t* sid = eid + sl * cap + p0;
        float* sd = ed + sl * cap + p0;
        if (fresh) sid[mbcnt(fm)] = id;
        __builtin_amdgcn_wave_barrier();
#ifdef NGT_AMD_STAMPS
        {
          const uint64_t t1 = stamp();
          if (lane == 0) atomicAdd((unsigned long long*)&ctl->sp[0], (unsigned long long)(t1 - st0));
          st0 = t1;
        }
#endif
        // the comparator's exact distances of those neighbours
        // (PrimitiveComparator::compareL2 through l2_fold_rows): a quad per
        // row, EG groups of 16 rows in flight
        float hop_d = __int_as_float(0x7f800000);  // this lane's nearest fresh neighbour
        uint32_t hop_id = 0u;
        {
          const float4* qq = reinterpret_cast<const float4*>(qlds) + g;
          for (uint32_t r0 = 0; r0 < np; r0 += 16u * EG) {
            float4 v[EG][NCH];
            uint32_t rid[EG];
#pragma unroll
            for (int j = 0; j < EG; j++) {
              rid[j] = 0u;
              if (r0 + 16u * j >= np) continue;
              const uint32_t rr = r0 + 16u * j + (uint32_t)rs;
              rid[j] = rr < np ? sid[rr] : 0u;
              const float4* x = reinterpret_cast<const float4*>(a.rows + (uint64_t)rid[j] * a.row_bytes) + g;
#pragma unroll
              for (int i = 0; i < NCH; i++) v[j][i] = x[4 * i];
            }
#pragma unroll
            for (int j = 0; j < EG; j++) {
              if (r0 + 16u * j >= np) continue;
              const uint32_t rr = r0 + 16u * j + (uint32_t)rs;
              const float d = l2_fold_rows<NCH>(qq, v[j]);
              if (g == 0 && rr < np) {
                sd[rr] = d;
                if (d < hop_d) {
                  hop_d = d;
                  hop_id = rid[j];
                }
              }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
#ifdef NGT_AMD_STAMPS
        if (lane == 0) atomicAdd((unsigned long long*)&ctl->sp[2], (unsigned long long)(stamp() - st0));
#endif
        if (lane == 0) {
          slots[sl].pn[part] = np;
          atomicAdd(&slots[sl].deg, live);
        }
        __builtin_amdgcn_wave_barrier();
        // the part's bit is this wave's last touch of the slot: once every
        // bit is set, the commit wave may free and reissue it
        if (lane == 0)
          __hip_atomic_fetch_or(&slots[sl].pready, 1u << part, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        // hop prefetch.  The commit wave waits on memory when it pops a node
        // nobody has speculated -- typically one its previous expansion just
        // accepted, i.e. the nearest neighbour of a list like this one.  The
        // part's nearest fresh neighbour within the exploration radius is
        // therefore read ahead: its adjacency row, then one word of every
        // 128-byte line of its fresh neighbours' rows, so that when it is
        // issued its own speculation's two round trips hit L2.  Nothing is
        // stored: results cannot change, only where the later loads hit.
        if (a.lat_hop) {
          const float hd = wave_min_f32(g == 0 ? hop_d : __int_as_float(0x7f800000));
          const uint64_t hm = ballot64(g == 0 && hop_d == hd && hop_id != 0u);
          if (hm != 0ull && hd <= lds_load_f32(&ctl->expr)) {
            const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)hop_id, __ffsll((long long)hm) - 1);
            const uint32_t wl = cap < 64u ? cap : 64u;
            const uint32_t nb = (uint32_t)lane < wl ? a.adj[(uint64_t)w * a.adj_stride + lane] : 0u;
            uint32_t acc = 0u;
            if (nb != 0u && !bm_test(bm, nb)) {
              const uint32_t* x = reinterpret_cast<const uint32_t*>(a.rows + (uint64_t)nb * a.row_bytes);
              for (uint32_t l = 0; l < (uint32_t)a.row_bytes / 128u; l++) acc += x[32u * l];
            }
            asm volatile("" ::"v"(acc));
          }
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace ngt_amd

namespace ngt_amd {

uint32_t search_lat_lds_bytes(const SearchArgs& a) {
  const uint32_t cap = (uint32_t)(a.adj_stride < a.edge_size ? a.adj_stride : a.edge_size);
  return LatLayout(a, cap, 8).total;
}

hipError_t launch_graph_search_lat(const SearchArgs& a, uint32_t slots, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const uint32_t cap = (uint32_t)(a.adj_stride < a.edge_size ? a.adj_stride : a.edge_size);
  // parts of 32 entries, at most 8 per list; results in one wave's registers
  if ((a.dp != 128 && a.dp != 96) || !a.adj || cap > 256u || a.k > 64u) return hipErrorNotSupported;
  const size_t lds = search_lat_lds_bytes(a);
  const ServeArgs none{};
#define LAT(NCH)                                                                                                \
  do {                                                                                                          \
    auto kern = ngt_graph_search_lat_kernel<NCH, 8, false>;                                                     \
    hipError_t e_ = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    if (e_ != hipSuccess) return e_;                                                                            \
    hipLaunchKernelGGL(kern, dim3(slots), dim3(512), lds, s, a, none);                                          \
  } while (0)
  if (a.dp == 128) LAT(8); else LAT(6);
#undef LAT
  return hipGetLastError();
}

hipError_t launch_graph_serve_lat(const SearchArgs& a, const ServeArgs& sv, hipStream_t s) {
  const uint32_t cap = (uint32_t)(a.adj_stride < a.edge_size ? a.adj_stride : a.edge_size);
  if ((a.dp != 128 && a.dp != 96) || !a.adj || cap > 256u || sv.workers == 0 || sv.nring == 0)
    return hipErrorNotSupported;
  const size_t lds = search_lat_lds_bytes(a);
#define SRV(NCH)                                                                                                \
  do {                                                                                                          \
    auto kern = ngt_graph_search_lat_kernel<NCH, 8, true>;                                                      \
    hipError_t e_ = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    if (e_ != hipSuccess) return e_;                                                                            \
    hipLaunchKernelGGL(kern, dim3(sv.workers + 1), dim3(512), lds, s, a, sv);                                   \
  } while (0)
  if (a.dp == 128) SRV(8); else SRV(6);
#undef SRV
  return hipGetLastError();
}

}  // namespace ngt_amd
