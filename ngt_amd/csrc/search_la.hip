// search_la.hip -- the best-first search of NeighborhoodGraph::searchReadOnlyGraph
// (lib/NGT/Graph.cpp:398-495) with LOOKAHEAD: one step expands the node the
// reference pops next together with the next P-1 keys of the unchecked set, so
// a step's memory round trips (adjacency rows, filter codes + visited probes,
// exact rows) serve up to P expansions instead of one.
//
// Shape: L2 over float rows of dp = 16 * NCH (96 / 128 elements) with the
// 1-byte filter copy (filter_kernels.hip, bound in search_common.h) and the
// padded adjacency (each list's first min(degree, edgeSize) ids, <= 256).
//
// Why the traversal is the reference's:
//  * the distances of a node's neighbours do not depend on the search state,
//    so computing them before the node is popped changes nothing; only the
//    ACCEPT step (Graph.cpp:462-483) is order-dependent, and it runs strictly in
//    the reference's pop order ("commit"): target j > 0 is committed only if
//    it is exactly the key the reference pops next (minimum of the unchecked
//    set, LDS + spill, within the exploration radius); otherwise the rest of
//    the step's speculation is discarded and the next step pops normally;
//  * the filter threshold of a step comes from the exploration radius at the
//    step's start; the radius only shrinks, so a neighbour the bound rejects
//    is also outside the radius when it is committed;
//  * "fresh" (not visited) is decided at the step's start from the visited set
//    (LDS filter bits + HBM epoch bytes); ids marked by this step's earlier
//    commits are caught at commit time by an exact per-step LDS hash.
//  FULL = every evaluated id is marked (the reference's visited set and its
//  distance-computation count); !FULL = the accepted-only set of
//  search_common.h (not_accepted): identical results, re-evaluations counted.
//
// Workgroup = W waves serve one query (W = 1: throughput launches, a wave per
// query per SIMD slot; W = 8: latency launches -- single C-API queries, small
// batches -- where a lone query gets a CU's worth of loads in flight).  Wave 0
// owns the sequential state (unchecked keys, results, radius); every wave
// shares the gathers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ngt_device.h"
#include "ngt_kernels.h"
#include "search_common.h"

namespace ngt_amd {

struct LaCtl {
  uint32_t qi, done, nt, ntl, nl, nx, fthr, fsq;
  uint32_t epoch, pad[7];
  // the filter threshold's double-precision terms, kept in LDS: in registers
  // they spill, and a scratch reload waits for every store still in flight
  double fe, finv_b, frq;
};

// 16-byte aligned LDS carve-out; the host's search_la_lds_bytes mirrors it.
struct LaLayout {
  uint32_t off_tkey, off_tcnt, off_loff, off_xoff, off_vf, off_cq, off_res, off_q, off_qb, off_l,
      off_lfl, off_x, off_xe, off_xd, off_sh, off_nid, off_nd, total;
  __host__ __device__ static uint32_t up16(uint32_t v) { return (v + 15u) & ~15u; }
  __host__ __device__ LaLayout(const SearchArgs& a, int P) {
    uint32_t o = up16(sizeof(LaCtl));
    off_tkey = o; o = up16(o + 8u * P);
    off_tcnt = o; o = up16(o + 4u * P);
    off_loff = o; o = up16(o + 4u * (P + 1));
    off_xoff = o; o = up16(o + 4u * (P + 1));
    off_vf = o; o = up16(o + ((1u << a.vf_log2) >> 3));
    off_cq = o; o = up16(o + 8u * a.cq_cap);
    off_res = o; o = up16(o + 8u * (a.k + 1));
    off_q = o; o = up16(o + 4u * (uint32_t)a.dp);
    off_qb = o; o = up16(o + (uint32_t)a.dp);
    off_l = o; o = up16(o + 4u * a.la_lmax);
    off_lfl = o; o = up16(o + a.la_lmax);
    off_x = o; o = up16(o + 4u * a.la_lmax);
    off_xe = o; o = up16(o + 4u * a.la_lmax);
    off_xd = o; o = up16(o + 4u * a.la_lmax);
    off_sh = o; o = up16(o + (4u << a.la_sh_log2));
    off_nid = o; o = up16(o + 256u);
    off_nd = o; o = up16(o + 256u);
    total = o;
  }
};

// exact per-step set of ids (open addressing, 0 = empty)
__device__ __forceinline__ uint32_t sh_slot(uint32_t id, uint32_t log2) { return (id * 0x9E3779B1u) >> (32 - log2); }
__device__ __forceinline__ bool sh_contains(const uint32_t* sh, uint32_t log2, uint32_t id) {
  const uint32_t mask = (1u << log2) - 1u;
  for (uint32_t h = sh_slot(id, log2);; h = (h + 1) & mask) {
    const uint32_t v = sh[h];
    if (v == id) return true;
    if (v == 0u) return false;
  }
}
__device__ __forceinline__ void sh_insert(uint32_t* sh, uint32_t log2, uint32_t id) {
  const uint32_t mask = (1u << log2) - 1u;
  for (uint32_t h = sh_slot(id, log2);; h = (h + 1) & mask) {
    const uint32_t old = atomicCAS(sh + h, 0u, id);
    if (old == 0u || old == id) return;
  }
}

__device__ __forceinline__ void vf_set(uint32_t* vf, uint32_t shift, uint32_t id) {
  const uint32_t b = (id * 0x85EBCA77u) >> shift;
  atomicOr(vf + (b >> 5), 1u << (b & 31));
}
__device__ __forceinline__ bool vf_test(const uint32_t* vf, uint32_t shift, uint32_t id) {
  const uint32_t b = (id * 0x85EBCA77u) >> shift;
  return (vf[b >> 5] >> (b & 31)) & 1u;
}

// a wave-uniform u64 in SGPRs (the reductions leave it in every lane)
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// WPE: resident waves per SIMD the kernel is compiled for (VGPR budget)
template <int NCH, int W, int PW, int RG, int EG, bool FULL, int WPE>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE)))
ngt_graph_search_la_kernel(SearchArgs a) {
  constexpr int P = W * PW;
  constexpr int E = 4 * NCH;  // filter-code bytes per lane of a quad
  constexpr int NW = E / 8;   // 8-byte code words per lane
  static_assert((NCH & 1) == 0, "whole 8-byte code words per lane");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const LaLayout lay(a, P);
  LaCtl* ctl = reinterpret_cast<LaCtl*>(smem);
  uint64_t* tkey = reinterpret_cast<uint64_t*>(smem + lay.off_tkey);
  uint32_t* tcnt = reinterpret_cast<uint32_t*>(smem + lay.off_tcnt);
  uint32_t* loff = reinterpret_cast<uint32_t*>(smem + lay.off_loff);
  uint32_t* xoff = reinterpret_cast<uint32_t*>(smem + lay.off_xoff);
  uint32_t* vf = reinterpret_cast<uint32_t*>(smem + lay.off_vf);
  uint64_t* cq = reinterpret_cast<uint64_t*>(smem + lay.off_cq);
  uint64_t* res = reinterpret_cast<uint64_t*>(smem + lay.off_res);
  float* qlds = reinterpret_cast<float*>(smem + lay.off_q);
  uint8_t* qb = smem + lay.off_qb;
  uint32_t* L = reinterpret_cast<uint32_t*>(smem + lay.off_l);
  uint8_t* lfl = smem + lay.off_lfl;
  uint32_t* X = reinterpret_cast<uint32_t*>(smem + lay.off_x);
  uint32_t* Xe = reinterpret_cast<uint32_t*>(smem + lay.off_xe);
  float* Xd = reinterpret_cast<float*>(smem + lay.off_xd);  // by list entry
  uint32_t* sh = reinterpret_cast<uint32_t*>(smem + lay.off_sh);
  uint32_t* nid = reinterpret_cast<uint32_t*>(smem + lay.off_nid);
  float* nd = reinterpret_cast<float*>(smem + lay.off_nd);

  const int lane = lane_id();
  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t NT = 64u * W;
  const uint32_t vf_words = (1u << a.vf_log2) / 32;
  const uint32_t vf_shift = 32 - a.vf_log2;
  const uint32_t sh_n = 1u << a.la_sh_log2;
  const uint32_t lmax = a.la_lmax;
  const float fa = a.fparams[0], fb = a.fparams[1];
  const uint32_t slot = blockIdx.x;
  uint8_t* vis = a.vis + (uint64_t)slot * a.vis_stride;
  uint64_t* spill = a.spill + (uint64_t)slot * a.spill_cap;
  const uint64_t deg_cap = a.adj_stride < a.edge_size ? a.adj_stride : a.edge_size;
  const uint32_t k = a.k;
  const int g = lane & 3, rs = lane >> 2;

  for (;;) {
    if (tid == 0) ctl->qi = atomicAdd(a.work, 1u);
    __syncthreads();
    const uint32_t qi = ctl->qi;
    if (qi >= a.nq) break;

    // ---- per-query init (every wave) -------------------------------------
    for (uint32_t i = tid; i < vf_words; i += NT) vf[i] = 0u;
    {
      const uint4* s = reinterpret_cast<const uint4*>(a.queries + (uint64_t)qi * a.query_bytes);
      uint4* d = reinterpret_cast<uint4*>(qlds);
      for (uint32_t i = tid; i < (uint32_t)a.dp / 4; i += NT) d[i] = s[i];
    }
    uint32_t epoch = a.slot_epoch[slot] + 1;
    if (epoch > 255) {
      uint4* v4 = reinterpret_cast<uint4*>(vis);
      for (uint64_t i = tid; i < a.vis_stride / 16; i += NT) v4[i] = make_uint4(0, 0, 0, 0);
      epoch = 1;
    }
    __syncthreads();
    if (tid == 0) a.slot_epoch[slot] = epoch;

    // wave 0's sequential state
    uint32_t ncq = 0, nspill = 0, nres = 0, maxq = 0;
    uint32_t ndist = 0, nexp = 0, nedge = 0, nexact = 0, ndisc = 0, ns = 0;
    uint32_t sh_used = 0;  // ids inserted into this step's id set
    // wave 0's copy of the step's targets (ascending keys, compile-time indexed)
    // and the commit guard: nblock = the first target j > 0 that a key pushed
    // by this step's earlier commits precedes (that key, not t_j, is then the
    // reference's next pop)
    uint64_t tk[P];
#pragma unroll
    for (int j = 0; j < P; j++) tk[j] = ~0ull;
    uint32_t nblock = P, cur_j = 0;
    // diagnostic build only: shader-clock totals per phase (wave 0's view)
    uint64_t t_a = 0, t_b = 0, t_c = 0, t_e = 0, t_f = 0, t_last = 0, nsteps = 0;
    (void)t_a; (void)t_b; (void)t_c; (void)t_e; (void)t_f; (void)t_last; (void)nsteps;
    // diagnostic build only (NGT_AMD_LACOUNT): where a query's lines come from
    // -- spill keys written / read, refills, visited-epoch probes, code rows of
    // every list entry read (committed or not), exact rows
    uint64_t n_spw = 0, n_spr = 0, n_refill = 0, n_probe = 0, n_codes = 0, n_rows = 0;
    (void)n_spw; (void)n_spr; (void)n_refill; (void)n_probe; (void)n_codes; (void)n_rows;
    float radius = a.radius;
    float expr = 0.f;
    double frq = 0.0;
    // ---- the unchecked set: three levels with key thresholds B and T -------
    // head (wave 0's registers, sorted: lane i = i-th smallest, hn keys) < B
    // <= tail (LDS, unsorted, ncq keys) < T <= spill (HBM, per slot), so the
    // smallest keys are always in the head while it is non-empty: a step's
    // targets are its first lanes and a pop is a lane shift.  A full head
    // sends its largest key to the tail (B drops); an emptying head takes the
    // smallest tail keys (histogram threshold + bitonic sort, B rises).  A full
    // tail is compacted (keys beyond the exploration radius can never be
    // popped, Graph.cpp:433-435) and, if still over half full, its larger half
    // moves to the spill (T drops); an empty tail refills with the smallest
    // spill keys (T rises).  Exact throughout.
    uint64_t hk = ~0ull, B = ~0ull;
    uint32_t hn = 0;
    uint64_t T = ~0ull;
    auto spill_push = [&](uint64_t key) {
      if (nspill >= a.spill_cap) {
        if (lane == 0) atomicOr(a.error, 1);
      } else {
        if (lane == 0) spill[nspill] = key;
        nspill++;
#ifdef NGT_AMD_LACOUNT
        n_spw++;
#endif
      }
    };
    // move the LDS keys >= t to the spill (t lowers T)
    auto lds_to_spill = [&](uint64_t t) {
      uint32_t out = 0;
      for (uint32_t b = 0; b < ncq; b += 64) {
        const uint32_t i = b + (uint32_t)lane;
        const uint64_t key = i < ncq ? cq[i] : ~0ull;
        const bool mv = i < ncq && key >= t;
        const bool keep = i < ncq && key < t;
        const uint64_t mm = ballot64(mv), km = ballot64(keep);
        const uint32_t nm = (uint32_t)__popcll(mm);
        if (nspill + nm > a.spill_cap) {
          if (lane == 0) atomicOr(a.error, 1);
        } else if (mv) {
          spill[nspill + mbcnt(mm)] = key;
        }
        if (nspill + nm <= a.spill_cap) nspill += nm;
#ifdef NGT_AMD_LACOUNT
        n_spw += nm;
#endif
        __builtin_amdgcn_wave_barrier();
        if (keep) cq[out + mbcnt(km)] = key;
        __builtin_amdgcn_wave_barrier();
        out += (uint32_t)__popcll(km);
      }
      ncq = out;
      T = t;
    };
    auto make_room = [&]() {
      ncq = compact(cq, ncq, expr);
      const uint32_t keep = a.cq_cap / 2;
      if (ncq > keep) {
        // bisect for the threshold t that keeps between keep/2 and keep keys
        uint64_t lo = ~0ull, hi = 0;
        for (uint32_t i = lane; i < ncq; i += 64) {
          const uint64_t v = cq[i];
          lo = v < lo ? v : lo;
          hi = v > hi ? v : hi;
        }
        lo = wave_min_u64(lo);
        hi = ~wave_min_u64(~hi);  // max
        // the largest t with count(keys < t) <= keep (keys are distinct, so
        // the count rises by one per key): l is always such a t
        uint64_t l = lo, h = hi;
        for (int it = 0; it < 64 && l < h; it++) {
          const uint64_t mid = l + ((h - l) >> 1) + 1;
          uint32_t c = 0;
          for (uint32_t i = lane; i < ncq; i += 64) c += cq[i] < mid ? 1u : 0u;
          c = wave_sum_u32(c);
          if (c <= keep) {
            l = mid;
            if (c >= keep / 2) break;
          } else {
            h = mid - 1;
          }
        }
        lds_to_spill(l);
      }
    };
    // refill an empty LDS with the smallest spill keys within the radius
    auto refill = [&]() {
      const uint32_t want = a.cq_cap / 2;
      uint32_t* hist = nid;  // 64 counters (free outside the accept staging)
#ifdef NGT_AMD_LACOUNT
      n_refill++;
      n_spr += 2 * nspill;  // the range pass and the move pass
#endif
      // key distances as ordered 32-bit values; the spill keys within the radius
      const uint32_t lim = ord_of(expr);
      uint32_t lo = 0xffffffffu, hi = 0;
      for (uint32_t i = lane; i < nspill; i += 64) {
        const uint32_t o = (uint32_t)(spill[i] >> 32);
        if (o <= lim) {
          lo = o < lo ? o : lo;
          hi = o > hi ? o : hi;
        }
      }
      lo = (uint32_t)(wave_min_u64(lo) & 0xffffffffu);
      hi = (uint32_t)(~wave_min_u64(~(uint64_t)hi) & 0xffffffffu);
      uint32_t bound = 0;  // spill keys with ord < bound move to LDS
      if (lo > hi) {
        nspill = 0;  // nothing within the radius: the search ends
        T = ~0ull;
        return;
      }
      for (;;) {
        const uint64_t span = (uint64_t)hi - lo + 1;
        const uint64_t width = (span + 63) / 64;
        hist[lane] = 0u;
        __builtin_amdgcn_wave_barrier();
#ifdef NGT_AMD_LACOUNT
        n_spr += nspill;
#endif
        for (uint32_t i = lane; i < nspill; i += 64) {
          const uint32_t o = (uint32_t)(spill[i] >> 32);
          if (o >= lo && o <= hi) atomicAdd(hist + (uint32_t)(((uint64_t)o - lo) / width), 1u);
        }
        __builtin_amdgcn_wave_barrier();
        // largest b with sum(hist[0..b)) <= want
        const uint32_t h = hist[lane];
        uint32_t incl = h;  // inclusive prefix over lanes
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t v = __shfl_up(incl, o, 64);
          if (lane >= o) incl += v;
        }
        const uint64_t okm = ballot64(incl <= want);
        const uint32_t b = (uint32_t)__popcll(okm);  // bins [0, b) fit (prefix is monotone)
        if (b >= 1 || width == 1) {
          bound = b >= 1 ? (uint32_t)std::min<uint64_t>((uint64_t)lo + b * width, 0xffffffffull) : lo + 1;
          if (b == 0 && lane == 0) atomicOr(a.error, 8);  // > want keys share one distance: never expected
          break;
        }
        hi = (uint32_t)(lo + width - 1);  // the first bin alone is too big: refine it
      }
      // move: ord < bound (and within the radius) to LDS; keep ord >= bound
      // (within the radius) in the spill, compacted in place
      uint32_t out = 0;
      for (uint32_t b0 = 0; b0 < nspill; b0 += 64) {
        const uint32_t i = b0 + (uint32_t)lane;
        const uint64_t key = i < nspill ? spill[i] : ~0ull;
        const uint32_t o = (uint32_t)(key >> 32);
        const bool in = i < nspill && o <= lim;
        // (the histogram bounds the moved keys by want <= cq_cap / 2; the
        // flagged degenerate bound above keeps any excess in the spill)
        const bool fits = ncq + mbcnt(ballot64(in && o < bound)) < a.cq_cap;
        const bool mv = in && o < bound && fits;
        const bool stay = in && !mv;
        const uint64_t mm = ballot64(mv), sm = ballot64(stay);
        __builtin_amdgcn_wave_barrier();
        if (mv) cq[ncq + mbcnt(mm)] = key;
        if (stay) spill[out + mbcnt(sm)] = key;
        __builtin_amdgcn_wave_barrier();
        ncq += (uint32_t)__popcll(mm);
        out += (uint32_t)__popcll(sm);
      }
      nspill = out;
      T = nspill ? ((uint64_t)bound << 32) : ~0ull;
      __builtin_amdgcn_wave_barrier();
    };
    auto tail_insert = [&](uint64_t key) {
      if (key >= T) {
        spill_push(key);
      } else {
        if (ncq >= a.cq_cap) make_room();
        if (key >= T) {
          spill_push(key);
        } else {
          if (lane == 0) cq[ncq] = key;
          ncq++;
        }
      }
      __builtin_amdgcn_wave_barrier();
    };
    auto insert_key = [&](uint64_t key) {
      if (key < B) {
        const uint32_t pos = (uint32_t)__popcll(ballot64((uint32_t)lane < hn && hk < key));
        const uint64_t uk = wave_up1_u64(hk);
        if (hn == 64u) {
          // the head is full: its largest key (or this one) moves to the tail
          if (pos == 64u) {
            B = key;
            tail_insert(key);
          } else {
            const uint64_t e = readlane_u64(hk, 63);
            if ((uint32_t)lane > pos) hk = uk;
            if ((uint32_t)lane == pos) hk = key;
            B = e;
            tail_insert(e);
          }
        } else {
          if ((uint32_t)lane > pos && (uint32_t)lane <= hn) hk = uk;
          if ((uint32_t)lane == pos) hk = key;
          hn++;
        }
      } else {
        tail_insert(key);
      }
      if (hn + ncq + nspill > maxq) maxq = hn + ncq + nspill;
    };
    // fill the head up with the smallest tail keys (the tail takes the
    // smallest spill keys first when it is empty): at most 64 - hn keys, all
    // above the head's, move in; then a bitonic sort across the lanes
    auto refill_head = [&]() {
      if (ncq == 0 && nspill != 0) refill();
      if (ncq == 0) return;
      const uint32_t room = 64u - hn;
      const uint64_t t = lat_select(cq, ncq, room, ~0ull, nid);
      uint64_t* st64 = reinterpret_cast<uint64_t*>(nid);  // 64 x u64 staged through nid/nd (adjacent)
      uint32_t got = 0, out = 0;
      for (uint32_t b0 = 0; b0 < ncq; b0 += 64) {
        const uint32_t i = b0 + (uint32_t)lane;
        const uint64_t key = i < ncq ? cq[i] : ~0ull;
        const bool mv = i < ncq && key < t;
        const bool kp = i < ncq && !mv;
        const uint64_t mm = ballot64(mv), km = ballot64(kp);
        __builtin_amdgcn_wave_barrier();
        if (mv && got + mbcnt(mm) < room) st64[got + mbcnt(mm)] = key;
        if (kp) cq[out + mbcnt(km)] = key;
        __builtin_amdgcn_wave_barrier();
        got += (uint32_t)__popcll(mm);
        out += (uint32_t)__popcll(km);
      }
      if (got == 0u || got > room) {
        if (lane == 0) atomicOr(a.error, 8);  // selection check: never expected
        got = got > room ? room : got;
      }
      ncq = out;
      uint64_t v = (uint32_t)lane < hn ? hk : ((uint32_t)lane < hn + got ? st64[lane - hn] : ~0ull);
      __builtin_amdgcn_wave_barrier();
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
      hn += got;
      B = (ncq + nspill) ? readlane_u64(hk, (int)hn - 1) + 1 : ~0ull;
    };
    // the head's first key leaves (the commit of a target)
    auto pop_head = [&]() {
      const uint64_t dk = wave_down1_u64(hk);
      hk = (uint32_t)lane + 1 < hn ? dk : ~0ull;
      hn--;
    };
    // keys entering the unchecked set during the commit of target cur_j: the
    // first later target they precede can no longer be the reference's next
    // pop (targets ascend, so every later one is blocked too)
    auto note_pushed = [&](bool mine, uint64_t key) {
#pragma unroll
      for (int jj = 1; jj < P; jj++)
        if ((uint32_t)jj > cur_j && (uint32_t)jj < nblock && ballot64(mine && key < tk[jj]) != 0ull)
          nblock = (uint32_t)jj;
    };
    auto tk_at = [&](uint32_t j) -> uint64_t {
      uint64_t r = tk[0];
#pragma unroll
      for (int jj = 1; jj < P; jj++)
        if ((uint32_t)jj == j) r = tk[jj];
      return r;
    };
    // Push the candidates of `bm` (lanes of cid/cd, all within the
    // exploration radius and none within the result radius, so none changes
    // either radius) into the unchecked set at once -- what the sequential
    // accept would do for each of them.
    auto push_batch = [&](uint64_t bm, uint32_t cid, float cd) {
      const uint32_t cnt = (uint32_t)__popcll(bm);
      if (cnt == 0) return;
      const bool mine = (bm >> lane) & 1ull;
      const uint32_t id = mine ? cid : 0u;
      const uint64_t key = mine ? make_key(cd, id) : ~0ull;
      if constexpr (!FULL) {
        if (mine) {
          vf_set(vf, vf_shift, id);
          vis[id] = (uint8_t)epoch;
          sh_insert(sh, a.la_sh_log2, id);
        }
        sh_used += cnt;
      }
      note_pushed(mine, key);
      // keys below B enter the head one at a time (sorted insert); the rest
      // go to the tail, in one append when they all lie below T and fit
      const uint64_t hm = ballot64(mine && key < B);
      const uint64_t tm = bm & ~hm;
      uint64_t r = hm;
      while (r) {
        const int j = __ffsll((long long)r) - 1;
        r &= r - 1;
        insert_key(readlane_u64(key, j));
      }
      const uint32_t tc = (uint32_t)__popcll(tm);
      if (tc) {
        const bool tmine = (tm >> lane) & 1ull;
        const bool below = ballot64(tmine && key >= T) == 0ull;
        if (below && ncq + tc <= a.cq_cap) {
          if (tmine) cq[ncq + mbcnt(tm)] = key;
          ncq += tc;
          __builtin_amdgcn_wave_barrier();
        } else {
          r = tm;
          while (r) {
            const int j = __ffsll((long long)r) - 1;
            r &= r - 1;
            tail_insert(readlane_u64(key, j));
          }
        }
        if (hn + ncq + nspill > maxq) maxq = hn + ncq + nspill;
      }
    };
    // wave 0: accept the evaluated neighbours of the lanes in km (lane order
    // = neighbour order; id and distance in cid / cd) as Graph.cpp:471-483
    // does.  Only a candidate within the RESULT radius changes the state the
    // next candidates see (it enters the results and may shrink both radii),
    // so the candidates before the next such one are pushed as one batch,
    // that one alone, and the rest re-tested against the new exploration
    // radius -- the sequential order's outcome exactly.
    auto accept = [&](uint64_t km, uint32_t cid, float cd) {
      const bool inl = (km >> lane) & 1ull;
      uint64_t okmask = ballot64(inl && cd <= expr);
      while (okmask) {
        const uint64_t rmask = okmask & ballot64(inl && cd <= radius);
        if (rmask == 0ull) {
          push_batch(okmask, cid, cd);
          break;
        }
        const int j = __ffsll((long long)rmask) - 1;
        push_batch(okmask & ((1ull << j) - 1ull), cid, cd);
        // candidate j: d <= radius <= explorationRadius
        const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cd), j));
        const uint32_t id = (uint32_t)__builtin_amdgcn_readlane((int)cid, j);
        const uint64_t key = make_key(d, id);
        if constexpr (!FULL) {
          if (lane == 0) {
            vf_set(vf, vf_shift, id);
            vis[id] = (uint8_t)epoch;
            sh_insert(sh, a.la_sh_log2, id);
          }
          sh_used++;
        }
        note_pushed(true, key);
        insert_key(key);
        res_insert(res, nres, k, key);
        if (nres >= k) {
          radius = key_dist(res[k - 1]);
          expr = __fmul_rn(a.coef, radius);
        }
        __builtin_amdgcn_wave_barrier();
        okmask &= ~((2ull << j) - 1ull);  // the candidates after j ...
        okmask &= ballot64(inl && cd <= expr);  // ... within the (possibly smaller) radius
      }
    };

    uint32_t fsq = 0;  // wave 0's copy (W == 1 reads it from registers)
    if (wave == 0) {
      filter_query(qlds, a.dp, fa, fb, qb, fsq, frq);
      if (lane == 0) {
        ctl->fe = (double)a.fparams[2];
        ctl->finv_b = 1.0 / (double)a.fparams[1];
        ctl->frq = frq;
      }
      if (lane == 0) ctl->fsq = fsq;
      // ---- setupDistances + setupSeeds (Graph.cpp:293-367) --------------
      const uint64_t sb = a.seed_off ? a.seed_off[qi] : (uint64_t)qi * a.seed_stride;
      ns = a.seed_off ? (uint32_t)(a.seed_off[qi + 1] - sb) : a.seed_count[qi];
      for (uint32_t base = 0; base < ns; base += 64) {
        const uint32_t m = ns - base < 64 ? (uint32_t)(ns - base) : 64u;
        if ((uint32_t)lane < m) nid[lane] = a.seeds[sb + base + lane];
        __builtin_amdgcn_wave_barrier();
        eval_l2f_fast<NCH, 1>(qlds, a.rows, a.row_bytes, nid, nd, (int)m);
        __builtin_amdgcn_wave_barrier();
        if ((uint32_t)lane < m) {
          const uint32_t id = nid[lane];
          vf_set(vf, vf_shift, id);
          vis[id] = (uint8_t)epoch;
        }
        __builtin_amdgcn_wave_barrier();
        // every seed enters the unchecked set (Graph.cpp:355-366), the first
        // k within the radius the results
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
    }

    // ---- best-first loop (Graph.cpp:430-486), P expansions per step --------
#ifdef NGT_AMD_STAMPS
    t_last = stamp();
#endif
    for (;;) {
      // wave 0's step control; with one wave it never goes through LDS
      uint32_t s_done = 0, s_nt = 0, s_fthr = 0;
      // A. wave 0: the reference's next pop and the keys in line after it --
      // the nt <= P smallest keys of the unchecked set within the
      // exploration radius: the head's first lanes (refilled from the tail
      // when it holds fewer than P keys).  They stay in the head; each
      // committed target leaves it at its commit (phase F).
      if (wave == 0) {
        if (hn < (uint32_t)P && (ncq | nspill) != 0u) refill_head();
        const uint32_t lim = hn < (uint32_t)P ? hn : (uint32_t)P;
        const uint32_t nt = (uint32_t)__popcll(ballot64((uint32_t)lane < lim && key_dist(hk) <= expr));
#pragma unroll
        for (int j = 0; j < P; j++) tk[j] = (uint32_t)j < nt ? readlane_u64(hk, j) : ~0ull;
        const uint32_t done = nt == 0 ? 1u : 0u;  // empty, or the minimum is beyond the radius (Graph.cpp:433-435)
        if (lane == 0) {
#pragma unroll
          for (int j = 0; j < P; j++)
            if ((uint32_t)j < nt) tkey[j] = tk[j];
        }
        s_done = done;
        s_nt = nt;
        s_fthr = filter_threshold(expr, ctl->fe, ctl->finv_b, ctl->frq);
        if (W > 1 && lane == 0) {
          ctl->done = done;
          ctl->nt = nt;
          ctl->fthr = s_fthr;
        }
      }
      __syncthreads();
      NGT_MARK(t_a);
      nsteps++;
      if (W == 1 ? s_done != 0u : ctl->done != 0u) break;
      const uint32_t nt = W == 1 ? s_nt : ctl->nt;

      // B. adjacency rows of the targets (target j on wave j mod W), one round trip
      uint32_t r[PW][4];
      uint32_t cnt[PW];
#pragma unroll
      for (int jj = 0; jj < PW; jj++) {
        const uint32_t j = (uint32_t)(wave + W * jj);
        cnt[jj] = 0;
        // one wave: the targets are in its registers (no LDS round trip)
        const uint64_t tkj = W == 1 ? tk[jj] : tkey[j < nt ? j : 0u];
        if (j < nt) load_adj_row(a.adj + (uint64_t)key_id(tkj) * a.adj_stride, deg_cap, r[jj][0], r[jj][1],
                                 r[jj][2], r[jj][3]);
        else r[jj][0] = r[jj][1] = r[jj][2] = r[jj][3] = 0u;
      }
#pragma unroll
      for (int jj = 0; jj < PW; jj++) {
        const uint32_t j = (uint32_t)(wave + W * jj);
        // 0-terminated rows: the ids form a prefix
        cnt[jj] = (uint32_t)(__popcll(ballot64(r[jj][0] != 0u)) + __popcll(ballot64(r[jj][1] != 0u)) +
                             __popcll(ballot64(r[jj][2] != 0u)) + __popcll(ballot64(r[jj][3] != 0u)));
        if (j < nt && lane == 0) tcnt[j] = cnt[jj];
      }
      // the step hash starts empty
      if (sh_n % (4u * NT) == 0u) {
        for (uint32_t i = 4u * tid; i < sh_n; i += 4u * NT) *reinterpret_cast<uint4*>(sh + i) = make_uint4(0, 0, 0, 0);
      } else {
        for (uint32_t i = tid; i < sh_n; i += NT) sh[i] = 0u;
      }
      if constexpr (W > 1) __syncthreads();
      // list offsets: the targets whose lists fit the list capacity (t0 always does)
      uint32_t ntl = nt, tot = 0;
      uint32_t myoff[PW];
#pragma unroll
      for (int jj = 0; jj < PW; jj++) myoff[jj] = 0xffffffffu;
      if constexpr (W == 1) {
        // every target's count is in this wave's registers
        bool fits = true;
#pragma unroll
        for (int jj = 0; jj < PW; jj++) {
          if ((uint32_t)jj < nt && fits) {
            if (tot + cnt[jj] > lmax) {
              ntl = (uint32_t)jj;
              fits = false;
            } else {
              myoff[jj] = tot;
              if (tid == 0) loff[jj] = tot;
              tot += cnt[jj];
            }
          }
        }
      } else {
        for (uint32_t j = 0; j < nt; j++) {
          const uint32_t c = tcnt[j];
          if (tot + c > lmax) { ntl = j; break; }
#pragma unroll
          for (int jj = 0; jj < PW; jj++)
            if (j == (uint32_t)(wave + W * jj)) myoff[jj] = tot;
          if (tid == 0) loff[j] = tot;
          tot += c;
        }
      }
      if (tid == 0) {
        loff[ntl] = tot;
        ctl->ntl = ntl;
        ctl->nl = tot;
      }
#pragma unroll
      for (int jj = 0; jj < PW; jj++) {
        if (myoff[jj] == 0xffffffffu) continue;
        const uint32_t o = myoff[jj], c = cnt[jj];
        if ((uint32_t)lane < c) L[o + lane] = r[jj][0];
        if ((uint32_t)lane + 64 < c) L[o + 64 + lane] = r[jj][1];
        if ((uint32_t)lane + 128 < c) L[o + 128 + lane] = r[jj][2];
        if ((uint32_t)lane + 192 < c) L[o + 192 + lane] = r[jj][3];
      }
      __syncthreads();
      NGT_MARK(t_b);
      const uint32_t nl = tot;

      uint32_t xrun = 0;  // W == 1: survivors so far, entry order
      // C. visited-at-step-start test + filter codes of every list entry:
      // quad per entry, RG groups of 16 entries in flight per wave
      {
        const uint32_t fthr = W == 1 ? s_fthr : ctl->fthr;
        const uint32_t qsq = W == 1 ? fsq : ctl->fsq;
        uint2 q[NW];
        const uint2* qp = reinterpret_cast<const uint2*>(qb + g * E);
#pragma unroll
        for (int w = 0; w < NW; w++) q[w] = qp[w];
        for (uint32_t base = (uint32_t)wave * 16u * RG; base < nl; base += 16u * RG * W) {
          uint2 c[RG][NW];
          uint32_t ids[RG], pw[RG];
          bool bit[RG];
#pragma unroll
          for (int j = 0; j < RG; j++) {
            const uint32_t e = base + 16u * j + (uint32_t)rs;
            const uint32_t lv = L[e < nl ? e : 0u];  // unconditional: the reads issue together
            const uint32_t id = e < nl ? lv : 0u;
            ids[j] = id;
            pw[j] = 0u;
            bit[j] = false;
            if constexpr (FULL) {
              bit[j] = id != 0u && vf_test(vf, vf_shift, id);
              if (bit[j] && g == 0)
                pw[j] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(vis + (id & ~3u)), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
            }
            // unconditional too (an empty entry reads object 0's codes)
            load_code_words<NW>(a.fcodes + (uint64_t)id * (4 * E) + g * (8 * NW), c[j]);
          }
#pragma unroll
          for (int j = 0; j < RG; j++) {
            if (base + 16u * j >= nl) continue;
            uint32_t qc = 0u, cc = 0u;
#pragma unroll
            for (int w = 0; w < NW; w++) {
              qc = __builtin_amdgcn_udot4(q[w].x, c[j][w].x, qc, false);
              qc = __builtin_amdgcn_udot4(q[w].y, c[j][w].y, qc, false);
              cc = __builtin_amdgcn_udot4(c[j][w].x, c[j][w].x, cc, false);
              cc = __builtin_amdgcn_udot4(c[j][w].y, c[j][w].y, cc, false);
            }
            const uint32_t S = qsq + quad_sum_u32(cc - 2u * qc);
            const uint32_t e = base + 16u * j + (uint32_t)rs;
            const uint32_t id = ids[j];
#ifdef NGT_AMD_LACOUNT
            n_codes += (uint64_t)__popcll(ballot64(g == 0 && e < nl));
            if constexpr (FULL) n_probe += (uint64_t)__popcll(ballot64(g == 0 && e < nl && bit[j]));
#endif
            bool fresh = true;
            if constexpr (FULL) fresh = !bit[j] || ((pw[j] >> (8 * (id & 3))) & 0xffu) != epoch;
            // accepted-only set: only a survivor can be accepted, so only
            // survivors need the visited test -- it rides with their exact
            // rows (phase E) instead of an epoch probe per list entry
            const bool sv = g == 0 && e < nl && fresh && S <= fthr;
            if (g == 0 && e < nl) lfl[e] = (uint8_t)((fresh ? 1u : 0u) | (sv ? 2u : 0u));
            if constexpr (W == 1) {
              const uint64_t sm = ballot64(sv);
              if (sv) {
                X[xrun + mbcnt(sm)] = id;
                Xe[xrun + mbcnt(sm)] = e;
              }
              xrun += (uint32_t)__popcll(sm);
            }
          }
        }
      }
      __syncthreads();

      // D. survivors (keep bits) of every target, in target then neighbour
      // order (one wave: collected in phase C already)
      const uint32_t ntl_s = ntl;  // every wave computed it from the same counts
      uint32_t xtot = 0;
      if constexpr (W == 1) {
        xtot = xrun;
      } else {
      uint32_t xc[PW];
#pragma unroll
      for (int jj = 0; jj < PW; jj++) {
        const uint32_t j = (uint32_t)(wave + W * jj);
        xc[jj] = 0;
        if (j >= ntl_s) continue;
        const uint32_t lb = loff[j], le = loff[j + 1];
        for (uint32_t e0 = lb; e0 < le; e0 += 64) {
          const uint32_t e = e0 + (uint32_t)lane;
          xc[jj] += (uint32_t)__popcll(ballot64(e < le && (lfl[e] & 2u)));
        }
        if (lane == 0) xoff[j] = xc[jj];  // count; prefix below
      }
      __syncthreads();
      uint32_t xo[PW];
#pragma unroll
      for (int jj = 0; jj < PW; jj++) xo[jj] = 0;
      for (uint32_t j = 0; j < ntl_s; j++) {
        const uint32_t c = xoff[j];
#pragma unroll
        for (int jj = 0; jj < PW; jj++)
          if (j == (uint32_t)(wave + W * jj)) xo[jj] = xtot;
        xtot += c;
      }
      __syncthreads();  // every wave has read the counts
#pragma unroll
      for (int jj = 0; jj < PW; jj++) {
        const uint32_t j = (uint32_t)(wave + W * jj);
        if (j >= ntl_s) continue;
        if (lane == 0) xoff[j] = xo[jj];
        const uint32_t lb = loff[j], le = loff[j + 1];
        uint32_t o = xo[jj];
        for (uint32_t e0 = lb; e0 < le; e0 += 64) {
          const uint32_t e = e0 + (uint32_t)lane;
          const bool kp = e < le && (lfl[e] & 2u);
          const uint64_t km = ballot64(kp);
          if (kp) {
            X[o + mbcnt(km)] = L[e];
            Xe[o + mbcnt(km)] = e;
          }
          o += (uint32_t)__popcll(km);
        }
      }
      __syncthreads();
      }

      NGT_MARK(t_c);
      // E. exact comparator distances of the survivors (bit-identical to
      // PrimitiveComparator::compareL2 through l2_fold_rows)
      {
        const float4* qq = reinterpret_cast<const float4*>(qlds) + g;
        for (uint32_t r0 = (uint32_t)wave * 16u * EG; r0 < xtot; r0 += 16u * EG * W) {
          float4 v[EG][NCH];
          uint32_t xid[EG], xpw[EG];
          bool xchk[EG];
#pragma unroll
          for (int j = 0; j < EG; j++) {
            const uint32_t rr = r0 + 16u * j + (uint32_t)rs;
            const uint32_t id = rr < xtot ? X[rr] : 0u;
            xid[j] = id;
            xpw[j] = 0u;
            xchk[j] = false;
            const float4* x = reinterpret_cast<const float4*>(a.rows + (uint64_t)id * a.row_bytes) + g;
            if (j == 0 || r0 + 16u * j < xtot) {
#pragma unroll
              for (int i = 0; i < NCH; i++) v[j][i] = x[4 * i];
            }
            if constexpr (!FULL) {
              // the survivor's visited test: LDS filter, then its HBM epoch
              // (after the row loads: they need not wait for the filter read)
              xchk[j] = g == 0 && rr < xtot && vf_test(vf, vf_shift, id);
              if (xchk[j])
                xpw[j] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(vis + (id & ~3u)), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
          }
#pragma unroll
          for (int j = 0; j < EG; j++) {
            if (j != 0 && r0 + 16u * j >= xtot) continue;
            const uint32_t rr = r0 + 16u * j + (uint32_t)rs;
            const float d = l2_fold_rows<NCH>(qq, v[j]);
            // accepted-only set: a visited survivor is marked by a negative
            // distance (an L2 distance is never below +0)
            const bool seen = xchk[j] && ((xpw[j] >> (8 * (xid[j] & 3))) & 0xffu) == epoch;
            if (g == 0 && rr < xtot) Xd[Xe[rr]] = seen ? -1.f : d;
#ifdef NGT_AMD_LACOUNT
            n_probe += (uint64_t)__popcll(ballot64(xchk[j]));
#endif
          }
        }
      }
      __syncthreads();
      NGT_MARK(t_e);
#ifdef NGT_AMD_LACOUNT
      n_rows += xtot;
#endif

      // F. wave 0 commits in the reference's pop order.  After commits
      // 0..j-1 the unchecked set is the step-start set minus t_0..t_{j-1}
      // plus the keys those commits pushed; its minimum is t_j unless one of
      // the pushed keys precedes it (nblock <= j: speculation ends, that key
      // is the next pop), and the reference stops when that minimum lies
      // beyond the exploration radius (Graph.cpp:433-435).
      if (wave == 0) {
        uint32_t done = 0, ncommit = 0;
        sh_used = 0;
        nblock = P;
        for (uint32_t j = 0; j < ntl_s; j++) {
          cur_j = j;
          if (j > 0) {
            // the step's id set must never fill: stop before a target whose
            // every entry could be inserted would pass half its capacity
            if (sh_used + (loff[j + 1] - loff[j]) > sh_n / 2) break;
            if (nblock <= j) break;
            if (key_dist(tk_at(j)) > expr) {
              done = 1;
              break;
            }
          }
          // t_j is the head's first key here: t_0..t_{j-1} left it and no
          // key pushed since precedes t_j (nblock > j)
          if (readlane_u64(hk, 0) != tk_at(j) && lane == 0) atomicOr(a.error, 8);
          pop_head();
          ncommit++;
          nexp++;
          const uint32_t lb = loff[j], le = loff[j + 1];
          nedge += le - lb;
          for (uint32_t e0 = lb; e0 < le; e0 += 64) {
            const uint32_t e = e0 + (uint32_t)lane;
            const bool in = e < le;
            const uint32_t ec = in ? e : lb;  // unconditional reads, issued together
            const uint32_t lv = L[ec], fv = lfl[ec];
            const uint32_t id = in ? lv : 0u;
            const uint32_t fl = in ? fv : 0u;
            bool keep;
            float xd = 0.f;
            if constexpr (FULL) {
              const bool fresh = (fl & 1u) && (j == 0 ? true : !sh_contains(sh, a.la_sh_log2, id));
              const uint32_t nfresh = (uint32_t)__popcll(ballot64(fresh));
              if (fresh) {
                vf_set(vf, vf_shift, id);
                vis[id] = (uint8_t)epoch;
                sh_insert(sh, a.la_sh_log2, id);
              }
              sh_used += nfresh;
              ndist += nfresh;
              keep = fresh && (fl & 2u);
              if (keep) xd = Xd[e];
            } else {
              // survivors carry their visited test (negative distance =
              // accepted before this step; the step's id set = accepted by
              // its earlier commits); every other entry counts as evaluated
              const bool surv = (fl & 2u) != 0u;
              xd = Xd[in ? e : lb];  // read for every lane: no dependent LDS round trip
              keep = surv && !(xd < 0.f) && (j == 0 ? true : !sh_contains(sh, a.la_sh_log2, id));
              ndist += (uint32_t)__popcll(ballot64(in && (!surv || keep)));
            }
            const uint64_t km = ballot64(keep);
            nexact += (uint32_t)__popcll(km);
            if (km) accept(km, id, xd);
            __builtin_amdgcn_wave_barrier();
          }
        }
        ndisc += ntl_s - ncommit;
        // the targets the commit did not reach are still in the head
        s_done = done;
        if (W > 1 && done && lane == 0) ctl->done = 1;
      }
      __syncthreads();
      NGT_MARK(t_f);
      if (W == 1 ? s_done != 0u : ctl->done != 0u) break;
    }

    // ---- results (moveFrom: ascending (distance, id), ObjectSpace.h:49-57)
    if (wave == 0) {
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
          c[3] = ndisc;   // speculative expansions discarded
          c[4] = nedge;
          c[5] = maxq;
          c[6] = nexact;  // exact neighbour distances of the committed expansions
          c[7] = ns;
#ifdef NGT_AMD_LACOUNT
          // line accounting: [1] spill keys written, [3] spill keys read,
          // [5] refills, [6] epoch probes, [7] list entries' code rows;
          // [4] exact rows (committed or not)
          c[1] = n_spw;
          c[3] = n_spr;
          c[5] = n_refill;
          c[6] = n_probe;
          c[7] = n_codes;
          c[4] = n_rows;
#endif
#ifdef NGT_AMD_STAMPS
          // phase cycles: [5] pop + targets, [6] adjacency + lists, [1] filter
          // + survivors, [7] exact rows, [3] commit; [4] steps
          c[5] = t_a;
          c[6] = t_b;
          c[1] = t_c;
          c[7] = t_e;
          c[3] = t_f;
          c[4] = nsteps;
#endif
        }
      }
    }
    __syncthreads();
  }
}

uint32_t search_la_lds_bytes(const SearchArgs& a, int P) { return LaLayout(a, P).total; }

// mode 0: throughput (W = 1), mode 1: latency (W = 8)
hipError_t launch_graph_search_la(const SearchArgs& a, int mode, bool full, uint32_t slots, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  if (a.dp != 128 && a.dp != 96) return hipErrorNotSupported;
  const uint32_t P = la_targets(mode);
  const size_t lds = search_la_lds_bytes(a, (int)P);
#define LA(NCH, W, PW, RG, EG, F, WPE)                                                                         \
  do {                                                                                                          \
    auto kern = ngt_graph_search_la_kernel<NCH, W, PW, RG, EG, F, WPE>;                                         \
    if (lds > 64 * 1024) {                                                                                       \
      hipError_t e_ = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
      if (e_ != hipSuccess) return e_;                                                                          \
    }                                                                                                           \
    hipLaunchKernelGGL(kern, dim3(slots), dim3(64 * W), lds, s, a);                                             \
  } while (0)
  if (mode == 0) {
    // P = 2 targets per step, 4 resident waves per SIMD (ngt_kernels.h)
    if (P != 2 || la_wpe() != 4) return hipErrorNotSupported;
    if (a.dp == 128) {
      if (full) LA(8, 1, 2, 3, 1, true, 4); else LA(8, 1, 2, 3, 1, false, 4);
    } else {
      if (full) LA(6, 1, 2, 3, 1, true, 4); else LA(6, 1, 2, 3, 1, false, 4);
    }
  } else {
    // latency form: one workgroup per CU, 2 waves per SIMD -> room for 192
    // filter rows in flight per wave (1,536 per step's round trip)
    if (a.dp == 128) {
      if (full) LA(8, 8, 1, 12, 1, true, 2); else LA(8, 8, 1, 12, 1, false, 2);
    } else {
      if (full) LA(6, 8, 1, 12, 1, true, 2); else LA(6, 8, 1, 12, 1, false, 2);
    }
  }
#undef LA
  return hipGetLastError();
}

}  // namespace ngt_amd
