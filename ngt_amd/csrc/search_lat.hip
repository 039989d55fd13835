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
constexpr uint32_t kFree = 0u, kIssued = 1u, kTaken = 2u, kReady = 3u;

struct LatCtl {
  uint32_t done;  // the commit wave has finished the query
  uint32_t qi;
  uint32_t fthr;  // filter threshold of the current exploration radius
  uint32_t fsq;   // sum q''^2
  uint64_t sp[4]; // diagnostic build: speculation-wave cycles (adjacency, filter, exact, idle)
};

// one node's speculation: key (its unchecked-set key, the priority), state,
// entries, list length
struct LatSlot {
  uint64_t key;
  uint32_t state;
  uint32_t n;    // neighbours not yet visited when the list was read
  uint32_t deg;  // list length read (getEdgeSize cap)
  uint32_t pad[3];
};

struct LatLayout {
  uint32_t off_slot, off_eid, off_ed, off_tail, off_res, off_q, off_qb, off_nid, off_nd, off_hist, off_stg, off_bm,
      total;
  __host__ __device__ static uint32_t up16(uint32_t v) { return (v + 15u) & ~15u; }
  __host__ __device__ LatLayout(const SearchArgs& a, uint32_t cap, uint32_t waves) {
    uint32_t o = up16(sizeof(LatCtl));
    off_slot = o; o = up16(o + sizeof(LatSlot) * a.lat_slots);
    off_eid = o; o = up16(o + 4u * a.lat_slots * cap);
    off_ed = o; o = up16(o + 4u * a.lat_slots * cap);
    off_tail = o; o = up16(o + 8u * a.lat_tail);
    off_res = o; o = up16(o + 8u * (a.k + 1));
    off_q = o; o = up16(o + 4u * (uint32_t)a.dp);
    off_qb = o; o = up16(o + (uint32_t)a.dp);
    off_nid = o; o = up16(o + 256u);
    off_nd = o; o = up16(o + 256u);
    off_hist = o; o = up16(o + 256u);
    off_stg = o; o = up16(o + 256u * waves);
    off_bm = o; o = up16(o + 4u * ((a.nrows + 31u) / 32u));
    total = o;
  }
};

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}
// whole-wave lane shifts by one on the DPP path (gfx9 wave_shr:1 /
// wave_shl:1: one VALU op instead of an LDS-crossbar ds_bpermute): up1 gives
// lane i the value of lane i-1, down1 the value of lane i+1; the lane with
// no source keeps its own value (the callers overwrite or mask it)
__device__ __forceinline__ uint32_t wave_up1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_down1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint64_t wave_up1_u64(uint64_t v) {
  return ((uint64_t)wave_up1((uint32_t)(v >> 32)) << 32) | wave_up1((uint32_t)v);
}
__device__ __forceinline__ uint64_t wave_down1_u64(uint64_t v) {
  return ((uint64_t)wave_down1((uint32_t)(v >> 32)) << 32) | wave_down1((uint32_t)v);
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t uniform_u64_lat(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ bool bm_test(const uint32_t* bm, uint32_t id) { return (bm[id >> 5] >> (id & 31)) & 1u; }

__device__ __forceinline__ uint32_t lds_load_acq(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A threshold t over the keys of arr[0..n) that are <= lim (wave-uniform
// arguments): at most M keys lie below t, at least one does, and M/2 or more
// when the keys allow.  Histogram passes over 64 power-of-two bins of the key
// range (64 LDS counters in hist), refining the first bin that overflows.
// Returns 0 when no key is <= lim.  Not inlined: it runs a few times per
// query and would otherwise share the commit loop's registers.
__device__ __noinline__ uint64_t lat_select(const uint64_t* arr, uint32_t n, uint32_t M, uint64_t lim, uint32_t* hist) {
  const int lane = lane_id();
  uint64_t lo = ~0ull, hi = 0;
  for (uint32_t i = lane; i < n; i += 64) {
    const uint64_t v = arr[i];
    if (v <= lim) {
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
  }
  lo = uniform_u64_lat(wave_min_u64(lo));
  hi = uniform_u64_lat(~wave_min_u64(~hi));
  if (lo > hi) return 0ull;
  uint32_t base = 0;
  for (int it = 0; it < 16; it++) {
    const uint64_t span = hi - lo;
    const int bits = span ? 64 - __clzll((long long)span) : 0;
    const int shift = bits > 6 ? bits - 6 : 0;
    // hist is LDS reached through a generic pointer: flat accesses may
    // complete out of order, so each phase drains before the next
    hist[lane] = 0u;
    __threadfence_block();
    for (uint32_t i = lane; i < n; i += 64) {
      const uint64_t v = arr[i];
      if (v >= lo && v <= hi && v <= lim) atomicAdd(hist + (uint32_t)((v - lo) >> shift), 1u);
    }
    __threadfence_block();
    uint32_t incl = hist[lane];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = (uint32_t)__shfl_up((int)incl, o, 64);
      if (lane >= o) incl += u;
    }
    const uint32_t b = (uint32_t)__popcll(ballot64(base + incl <= M));  // bins [0, b) fit
    if (b == 64u) return hi + 1;
    const uint32_t below = base + (b ? (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)b - 1) : 0u);
    if ((below >= M / 2 && below > 0) || shift == 0) return lo + ((uint64_t)b << shift);
    base = below;
    lo = lo + ((uint64_t)b << shift);
    const uint64_t top = lo + ((1ull << shift) - 1ull);
    hi = top < hi ? top : hi;
  }
  return lo + 1;  // never expected: the minimum alone
}

}  // namespace

// NCH = dp / 16; W waves (1 commit + W-1 speculation); RG = 16-entry filter
// groups in flight per speculation wave (RG * 16 >= the list capacity)
template <int NCH, int W, int RG>
__global__ void __launch_bounds__(64 * W) ngt_graph_search_lat_kernel(SearchArgs a) {
  constexpr int E = 4 * NCH;  // filter-code bytes per lane of a quad
  constexpr int NW = E / 8;   // 8-byte code words per lane
  static_assert((NCH & 1) == 0, "whole 8-byte code words per lane");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t cap = (uint32_t)(a.adj_stride < a.edge_size ? a.adj_stride : a.edge_size);
  const LatLayout lay(a, cap, W);
  LatCtl* ctl = reinterpret_cast<LatCtl*>(smem);
  LatSlot* slots = reinterpret_cast<LatSlot*>(smem + lay.off_slot);
  uint32_t* eid = reinterpret_cast<uint32_t*>(smem + lay.off_eid);
  float* ed = reinterpret_cast<float*>(smem + lay.off_ed);
  uint64_t* tail = reinterpret_cast<uint64_t*>(smem + lay.off_tail);
  uint64_t* res = reinterpret_cast<uint64_t*>(smem + lay.off_res);
  float* qlds = reinterpret_cast<float*>(smem + lay.off_q);
  uint8_t* qb = smem + lay.off_qb;
  uint32_t* nid = reinterpret_cast<uint32_t*>(smem + lay.off_nid);
  float* nd = reinterpret_cast<float*>(smem + lay.off_nd);
  uint32_t* bm = reinterpret_cast<uint32_t*>(smem + lay.off_bm);
  // threshold-selection counters: not nid/nd, which hold the accept step's
  // staged candidates when a full tail makes room in the middle of it
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + lay.off_hist);
  uint32_t* stg = reinterpret_cast<uint32_t*>(smem + lay.off_stg) + 64 * (threadIdx.x >> 6);  // per wave

  const int lane = lane_id();
  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t NT = 64u * W;
  const uint32_t bm_words = (a.nrows + 31u) / 32u;
  const uint32_t nslots = a.lat_slots;
  const float fa = a.fparams[0], fb = a.fparams[1], fe = a.fparams[2];
  const double finv_b = 1.0 / (double)fb;
  const uint32_t wg = blockIdx.x;
  uint64_t* spill = a.spill + (uint64_t)wg * a.spill_cap;
  const uint32_t k = a.k;
  const int g = lane & 3, rs = lane >> 2;

  for (;;) {
    if (tid == 0) ctl->qi = atomicAdd(a.work, 1u);
    __syncthreads();
    const uint32_t qi = ctl->qi;
    if (qi >= a.nq) break;

    // ---- per-query init (every wave) -------------------------------------
    {
      uint4* b4 = reinterpret_cast<uint4*>(bm);
      for (uint32_t i = tid; i < (bm_words + 3) / 4; i += NT) b4[i] = make_uint4(0, 0, 0, 0);
      const uint4* s = reinterpret_cast<const uint4*>(a.queries + (uint64_t)qi * a.query_bytes);
      uint4* d = reinterpret_cast<uint4*>(qlds);
      for (uint32_t i = tid; i < (uint32_t)a.dp / 4; i += NT) d[i] = s[i];
      for (uint32_t i = tid; i < nslots; i += NT) slots[i].state = kFree;
      if (tid == 0) {
        ctl->done = 0u;
        ctl->sp[0] = ctl->sp[1] = ctl->sp[2] = ctl->sp[3] = 0ull;
      }
    }
    __syncthreads();

    if (wave == 0) {
      // =================== the commit wave ===================================
      uint32_t fsq = 0;
      double frq = 0.0;
      filter_query(qlds, a.dp, fa, fb, qb, fsq, frq);
      uint32_t nres = 0, maxq = 0;
      uint32_t ndist = 0, nexp = 0, nedge = 0, nexact = 0, nwait = 0, ns = 0, nstall = 0;
      // diagnostic build only: shader-clock totals per phase
      uint64_t t_pop = 0, t_wait = 0, t_list = 0, t_feed = 0, t_last = 0;
      (void)t_pop; (void)t_wait; (void)t_list; (void)t_feed; (void)t_last;
      float radius = a.radius;
      float expr = 0.f;
      // unchecked set: head (registers, sorted, hn keys) < B <= tail (LDS,
      // ntail keys) < T <= spill (HBM, nspill keys)
      uint64_t hk = ~0ull;
      uint32_t ht = kNoTag;
      uint32_t hn = 0, ntail = 0, nspill = 0;
      uint64_t B = ~0ull, T = ~0ull;
      uint64_t freem = nslots >= 64 ? ~0ull : ((1ull << nslots) - 1ull);  // free slots
      uint64_t orphan = 0ull;                                             // issued, no longer in the head
      const uint32_t F = nslots < 16u ? nslots : 16u;                     // head entries kept speculated

      auto set_fthr = [&]() {
        if (lane == 0) ctl->fthr = filter_threshold(expr, (double)fe, finv_b, frq);
      };
      auto spill_push = [&](uint64_t key) {
        if (nspill >= a.spill_cap) {
          if (lane == 0) atomicOr(a.error, 1);
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
            if (lane == 0) atomicOr(a.error, 1);
          } else if (mv) {
            spill[nspill + mbcnt(mm)] = key;
          }
          if (nspill + nm <= a.spill_cap) nspill += nm;
          __builtin_amdgcn_wave_barrier();
          if (kp) tail[out + mbcnt(km)] = key;
          __builtin_amdgcn_wave_barrier();
          out += (uint32_t)__popcll(km);
        }
        if ((out == 0u || out > keep) && lane == 0) atomicOr(a.error, 32);  // selection check
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
        if ((ntail == 0u || ntail > want) && lane == 0) atomicOr(a.error, 64);  // selection check
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
        if ((got == 0u || got > 64u) && lane == 0) atomicOr(a.error, 128);  // selection check
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
      // free the orphaned slots whose speculation has finished
      auto reap = [&]() {
        uint64_t o = orphan;
        while (o) {
          const int s = __ffsll((long long)o) - 1;
          o &= o - 1;
          if (lds_load_acq(&slots[s].state) == kReady) {
            if (lane == 0) slots[s].state = kFree;
            orphan &= ~(1ull << s);
            freem |= 1ull << s;
          }
        }
      };
      // hand a node to the speculation waves (they take the issued slot of
      // the smallest key first: the commit wave's next pops)
      // every wait below is bounded: a slot that never becomes ready (never
      // expected) flags error 16 and ends the query instead of hanging the CU
      bool stuck = false;
      auto issue = [&](uint64_t key) -> uint32_t {
        for (uint32_t spin = 0; freem == 0ull; spin++) {
          reap();
          if (freem != 0ull) break;
          if (spin > (1u << 24)) {
            if (lane == 0) atomicOr(a.error, 16);
            stuck = true;
            return 0u;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t s = (uint32_t)(__ffsll((long long)freem) - 1);
        freem &= ~(1ull << s);
        if (lane == 0) slots[s].key = key;
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) lds_store_rel(&slots[s].state, kIssued);
        return s;
      };
      // speculation for the first F head entries that have none
      auto feed = [&]() {
        if (orphan) reap();
        uint64_t need = ballot64((uint32_t)lane < (hn < F ? hn : F) && ht == kNoTag);
        while (need) {
          const int l = __ffsll((long long)need) - 1;
          need &= need - 1;
          if (freem == 0ull) break;
          const uint32_t s = issue(readlane_u64(hk, l));
          if (stuck) break;
          if (lane == l) ht = s;
        }
      };
      auto push_batch = [&](uint64_t bm_) {
        uint64_t r = bm_;
        while (r) {
          const int j = __ffsll((long long)r) - 1;
          r &= r - 1;
          insert_key(make_key(nd[j], nid[j]));
        }
      };
      // accept `me` staged candidates (nid/nd, all fresh) in neighbour order
      // (Graph.cpp:471-483), the sequential outcome exactly
      auto accept = [&](uint32_t me) {
        const float dl = (uint32_t)lane < me ? nd[lane] : 0.f;
        const bool inl = (uint32_t)lane < me;
        uint64_t okmask = ballot64(inl && dl <= expr);
        while (okmask) {
          const uint64_t rmask = okmask & ballot64(inl && dl <= radius);
          if (rmask == 0ull) {
            push_batch(okmask);
            break;
          }
          const int j = __ffsll((long long)rmask) - 1;
          push_batch(okmask & ((1ull << j) - 1ull));
          const uint64_t key = make_key(nd[j], nid[j]);
          insert_key(key);
          res_insert(res, nres, k, key);
          if (nres >= k) {
            radius = key_dist(res[k - 1]);
            expr = __fmul_rn(a.coef, radius);
            set_fthr();
          }
          __builtin_amdgcn_wave_barrier();
          okmask &= ~((2ull << j) - 1ull);
          okmask &= ballot64(inl && dl <= expr);
        }
      };

      // the same accept on candidates held in registers: lanes of `cmask`
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
          res_insert(res, nres, k, key);
          if (nres >= k) {
            radius = key_dist(res[k - 1]);
            expr = __fmul_rn(a.coef, radius);
            set_fthr();
          }
          __builtin_amdgcn_wave_barrier();
          okmask &= ~((2ull << j) - 1ull);
          okmask &= ballot64(dv <= expr);
        }
      };

      // ---- setupDistances + setupSeeds (Graph.cpp:293-367) ----------------
      const uint64_t sb = a.seed_off ? a.seed_off[qi] : (uint64_t)qi * a.seed_stride;
      ns = a.seed_off ? (uint32_t)(a.seed_off[qi + 1] - sb) : a.seed_count[qi];
      expr = __fmul_rn(a.coef, radius);
      for (uint32_t base = 0; base < ns; base += 64) {
        const uint32_t m = ns - base < 64 ? (uint32_t)(ns - base) : 64u;
        if ((uint32_t)lane < m) nid[lane] = a.seeds[sb + base + lane];
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
          if (d <= a.radius) res_insert(res, nres, k, key);
        }
        __builtin_amdgcn_wave_barrier();
      }
      ndist = ns;
      if (nres >= k) radius = key_dist(res[k - 1]);
      expr = __fmul_rn(a.coef, radius);
      if (lane == 0) ctl->fsq = fsq;
      set_fthr();
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
        if (lds_load_acq(&slots[tag].state) != kReady) nstall++;
        for (uint32_t spin = 0; lds_load_acq(&slots[tag].state) != kReady; spin++) {
          if (spin > (1u << 24)) {
            if (lane == 0) atomicOr(a.error, 16);
            stuck = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (stuck) break;
        NGT_MARK(t_wait);
        const uint32_t n = slots[tag].n;
        nexp++;
        nedge += slots[tag].deg;
        const uint32_t* sid = eid + tag * cap;
        const float* sd = ed + tag * cap;
        // the whole list (<= 256 entries: 4 per lane) in one pass -- every
        // load issued before the first visited test, every test before the
        // marks -- then the accepts in neighbour order.  Ids of one list are
        // distinct, so testing and marking them in parallel is the sequential
        // outcome.
        {
          uint32_t id4[4];
          float d4[4];
          bool f4[4];
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const uint32_t e = 64u * c + (uint32_t)lane;
            id4[c] = e < n ? sid[e] : 0u;
            d4[c] = e < n ? sd[e] : 0.f;
          }
#pragma unroll
          for (int c = 0; c < 4; c++) f4[c] = id4[c] != 0u && !bm_test(bm, id4[c]);
#pragma unroll
          for (int c = 0; c < 4; c++) {
            if (64u * c >= n) break;
            if (f4[c]) atomicOr(bm + (id4[c] >> 5), 1u << (id4[c] & 31));
            ndist += (uint32_t)__popcll(ballot64(f4[c]));
            nexact += (uint32_t)__popcll(ballot64(f4[c] && d4[c] != __builtin_huge_valf()));
            // candidates within the radius (d = +inf: rejected by the bound),
            // accepted in neighbour order against the shrinking radius
            const uint64_t km = ballot64(f4[c] && d4[c] <= expr);
            if (km) accept_reg(km, id4[c], d4[c]);
          }
        }
        if (lane == 0) slots[tag].state = kFree;
        freem |= 1ull << tag;
        NGT_MARK(t_list);
        feed();
        NGT_MARK(t_feed);
      }
      // the speculation waves leave once every issued slot is done
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) lds_store_rel(&ctl->done, 1u);

      // ---- results (moveFrom: ascending (distance, id), ObjectSpace.h:49-57)
      for (uint32_t i = lane; i < nres; i += 64) {
        a.out_ids[(uint64_t)qi * k + i] = key_id(res[i]);
        a.out_dists[(uint64_t)qi * k + i] = key_dist(res[i]);
      }
      if (lane == 0) {
        a.out_n[qi] = nres;
        if (a.counters) {
          uint64_t* c = a.counters + (uint64_t)qi * 8;
          c[0] = ndist;
          c[1] = ndist - ns;
          c[2] = nexp;
          c[3] = nstall;  // pops that waited for their list (nwait of them: not yet handed out)
          c[4] = nedge;
          c[5] = maxq;
          c[6] = nexact;
          c[7] = ns;
#ifdef NGT_AMD_STAMPS
          // phase cycles: [5] pop (+ refills, issue), [6] wait for the list,
          // [1] list + accept, [7] feeding the speculation; [3] nwait
          c[5] = t_pop;
          c[6] = t_wait;
          c[1] = t_list;
          c[7] = t_feed;
          c[3] = nwait;
          // speculation waves, summed over the waves: [0] adjacency + visited
          // pre-test, [4] filter codes, [2] exact rows (expansions: nexp)
          __builtin_amdgcn_s_waitcnt(0);
          c[0] = ctl->sp[0];
          c[4] = ctl->sp[1];
          c[2] = ctl->sp[2];
#endif
        }
      }
    } else {
      // =================== speculation waves =================================
      for (;;) {
        if (lds_load_acq(&ctl->done)) break;
        // the issued slot with the smallest key
        const uint32_t st = (uint32_t)lane < nslots ? lds_load_acq(&slots[lane].state) : kFree;
        const uint64_t cand = st == kIssued ? slots[lane].key : ~0ull;
        const uint64_t m = uniform_u64_lat(wave_min_u64(cand));
        if (m == ~0ull) {
          if (lds_load_acq(&ctl->done)) break;
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const uint32_t s = (uint32_t)(__ffsll((long long)ballot64(cand == m)) - 1);
        uint32_t old = 0;
        if (lane == 0) old = atomicCAS(&slots[s].state, kIssued, kTaken);
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int)old) != kIssued) continue;  // another wave took it
        const uint32_t node = key_id(m);
#ifdef NGT_AMD_STAMPS
        uint64_t st0 = stamp();
#endif
        uint32_t* sid = eid + s * cap;
        float* sd = ed + s * cap;
        uint32_t n = 0, deg = 0;
        // the filter threshold of the current exploration radius (it only
        // shrinks: a neighbour the bound rejects is outside the radius at
        // commit time too)
        const uint32_t fthr = lds_load_acq(&ctl->fthr), fsq = ctl->fsq;
        uint2 q[NW];
        {
          const uint2* qp = reinterpret_cast<const uint2*>(qb + g * E);
#pragma unroll
          for (int w = 0; w < NW; w++) q[w] = qp[w];
        }
        {
        // adjacency row: the first min(degree, edgeSize) ids (Graph.cpp:436-439)
        uint32_t r0, r1, r2, r3;
        load_adj_row(a.adj + (uint64_t)node * a.adj_stride, cap, r0, r1, r2, r3);        deg = (uint32_t)(__popcll(ballot64(r0 != 0u)) + __popcll(ballot64(r1 != 0u)) +
                                        __popcll(ballot64(r2 != 0u)) + __popcll(ballot64(r3 != 0u)));
        // neighbours not visited yet, compacted in list order
        {
          const uint32_t rr[4] = {r0, r1, r2, r3};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            if ((uint32_t)(64 * c) >= deg) break;
            const bool f = rr[c] != 0u && !bm_test(bm, rr[c]);
            const uint64_t fm = ballot64(f);
            if (f) sid[n + mbcnt(fm)] = rr[c];
            n += (uint32_t)__popcll(fm);
          }
        }
        __builtin_amdgcn_wave_barrier();
#ifdef NGT_AMD_STAMPS
        {
          const uint64_t t1 = stamp();
          if (lane == 0) atomicAdd((unsigned long long*)&ctl->sp[0], (unsigned long long)(t1 - st0));
          st0 = t1;
        }
#endif
        // filter codes of every entry (quad per entry), RG groups of 16 in
        // flight; the threshold of the current exploration radius (it only
        // shrinks: a rejected neighbour is outside the radius at commit too)
        for (uint32_t base = 0; base < n; base += 16u * RG) {
          uint2 c[RG][NW];
#pragma unroll
          for (int j = 0; j < RG; j++) {
            const uint32_t e = base + 16u * j + (uint32_t)rs;
            const uint32_t id = e < n ? sid[e] : 0u;
            const uint2* cp = reinterpret_cast<const uint2*>(a.fcodes + (uint64_t)id * (4 * E)) + g * NW;
            if (base + 16u * j < n) {
#pragma unroll
              for (int w = 0; w < NW; w++) c[j][w] = cp[w];
            }
          }
#pragma unroll
          for (int j = 0; j < RG; j++) {
            if (base + 16u * j >= n) continue;
            uint32_t qc = 0u, cc = 0u;
#pragma unroll
            for (int w = 0; w < NW; w++) {
              qc = __builtin_amdgcn_udot4(q[w].x, c[j][w].x, qc, false);
              qc = __builtin_amdgcn_udot4(q[w].y, c[j][w].y, qc, false);
              cc = __builtin_amdgcn_udot4(c[j][w].x, c[j][w].x, cc, false);
              cc = __builtin_amdgcn_udot4(c[j][w].y, c[j][w].y, cc, false);
            }
            const uint32_t S = fsq + quad_sum_u32(cc - 2u * qc);
            const uint32_t e = base + 16u * j + (uint32_t)rs;
            // survivors: -1 until their exact distance lands; the rest +inf
            if (g == 0 && e < n) sd[e] = S <= fthr ? -1.f : __builtin_huge_valf();
          }
        }
        }
        __builtin_amdgcn_wave_barrier();
#ifdef NGT_AMD_STAMPS
        {
          const uint64_t t1 = stamp();
          if (lane == 0) atomicAdd((unsigned long long*)&ctl->sp[1], (unsigned long long)(t1 - st0));
          st0 = t1;
        }
#endif
        // exact comparator distances of the survivors (PrimitiveComparator::
        // compareL2 through l2_fold_rows), 16 rows per wave step
        {
          const float4* qq = reinterpret_cast<const float4*>(qlds) + g;
          uint32_t nsv = 0;
          for (uint32_t e0 = 0; e0 < n; e0 += 64) {
            const uint32_t e = e0 + (uint32_t)lane;
            const bool sv = e < n && sd[e] < 0.f;
            const uint64_t sm = ballot64(sv);
            __builtin_amdgcn_wave_barrier();
            if (sv && nsv + mbcnt(sm) < 64u) stg[nsv + mbcnt(sm)] = e;
            __builtin_amdgcn_wave_barrier();
            nsv += (uint32_t)__popcll(sm);
            if (nsv >= 48u || e0 + 64 >= n) {
              const uint32_t m_ = nsv < 64u ? nsv : 64u;
              for (uint32_t r0 = 0; r0 < m_; r0 += 16) {
                const uint32_t rr = r0 + (uint32_t)rs;
                const uint32_t pos = rr < m_ ? stg[rr] : 0u;
                const uint32_t id = rr < m_ ? sid[pos] : 0u;
                const float4* x = reinterpret_cast<const float4*>(a.rows + (uint64_t)id * a.row_bytes) + g;
                float4 v[NCH];
#pragma unroll
                for (int i = 0; i < NCH; i++) v[i] = x[4 * i];
                const float d = l2_fold_rows<NCH>(qq, v);
                if (g == 0 && rr < m_) sd[pos] = d;
              }
              __builtin_amdgcn_wave_barrier();
              // survivors past the 64 staged ones: a later pass of this loop
              // sees them still at -1
              if (nsv > 64u) {
                e0 -= 64;  // re-scan this chunk for the rest
              }
              nsv = 0;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
#ifdef NGT_AMD_STAMPS
        if (lane == 0) atomicAdd((unsigned long long*)&ctl->sp[2], (unsigned long long)(stamp() - st0));
#endif
        if (lane == 0) {
          slots[s].n = n;
          slots[s].deg = deg;
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) lds_store_rel(&slots[s].state, kReady);
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
  if ((a.dp != 128 && a.dp != 96) || !a.adj || !a.fcodes) return hipErrorNotSupported;
  const uint32_t cap = (uint32_t)(a.adj_stride < a.edge_size ? a.adj_stride : a.edge_size);
  const size_t lds = search_lat_lds_bytes(a);
#define LAT(NCH, RG)                                                                                            \
  do {                                                                                                          \
    auto kern = ngt_graph_search_lat_kernel<NCH, 8, RG>;                                                        \
    hipError_t e_ = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    if (e_ != hipSuccess) return e_;                                                                            \
    hipLaunchKernelGGL(kern, dim3(slots), dim3(512), lds, s, a);                                                \
  } while (0)
  if (a.dp == 128) {
    if (cap <= 64) LAT(8, 4); else LAT(8, 9);
  } else {
    if (cap <= 64) LAT(6, 4); else LAT(6, 10);
  }
#undef LAT
  return hipGetLastError();
}

}  // namespace ngt_amd
