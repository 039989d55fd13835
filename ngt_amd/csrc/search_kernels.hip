// search_kernels.hip -- gfx950 kernels for the NGT distance hot path.
//
//  * ngt_distances_kernel   : batched comparator (query x candidate-id list),
//                             the batch form of PrimitiveComparator::*::compare.
//  * ngt_tree_seed_kernel   : GraphAndTreeIndex::getSeedsFromTree
//                             (lib/NGT/Index.h:1524-1567) -- DVP-tree leaf
//                             descent + srand(leafID) thinning, one wave/query.
//  * ngt_graph_search_kernel: NeighborhoodGraph::searchReadOnlyGraph
//                             (lib/NGT/Graph.cpp:398-495), one wave per query,
//                             persistent over a query work counter.
//  * ngt_linear_search_kernel + merge: ObjectSpaceRepository::linearSearch
//                             (lib/NGT/ObjectSpaceRepository.h:466-502).
//
// All per-query state of the best-first search lives in LDS:
//   visited set   : open-addressing hash of object ids (exact; spills to a
//                   per-slot HBM bitmap when it fills),
//   unchecked set : unsorted array of (dist,id) keys; pop = wave min-reduce;
//                   entries farther than the exploration radius are dead and
//                   are dropped on compaction (they could only terminate the
//                   loop, Graph.cpp:433-435); spills to HBM when full,
//   results       : sorted array of the k best keys.
// The accept step runs in neighbour order with wave-uniform radius updates,
// so the traversal is the reference's, not an approximation of it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "ngt_device.h"
#include "ngt_kernels.h"
#include "search_common.h"

namespace ngt_amd {



// ---------------------------------------------------------------------------
// Batched comparator.  pair i: (query qidx[i], object oid[i]) -> out[i].
// ---------------------------------------------------------------------------
template <int M, typename T>
__global__ void __launch_bounds__(256) ngt_distances_kernel(DistanceArgs a) {
  const int lane = threadIdx.x & 63;
  const int g = lane & 3;
  const uint64_t quad = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const uint64_t nquads = ((uint64_t)gridDim.x * blockDim.x) >> 2;
  for (uint64_t i = quad; i < a.npairs; i += nquads) {
    const T* q = reinterpret_cast<const T*>(a.queries + (uint64_t)a.qidx[i] * a.query_bytes);
    const T* x = row_ptr<T>(a.rows, a.row_bytes, a.oid[i]);
    const float d = quad_distance<M, T>(q, x, a.dp, g);
    if (g == 0) a.out[i] = d;
  }
}

// ---------------------------------------------------------------------------
// Tree seeds: one wave per query.
// ---------------------------------------------------------------------------
template <int M, typename T>
__global__ void __launch_bounds__(64) ngt_tree_seed_kernel(TreeSeedArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  T* qlds = reinterpret_cast<T*>(smem);
  const int lane = lane_id();
  for (uint32_t qi = blockIdx.x; qi < a.nq; qi += gridDim.x) {
    load_query<T>(qlds, a.queries + (uint64_t)qi * a.query_bytes, a.dp);
    __syncthreads();
    uint32_t node = a.root;
    uint32_t ndist = 0;
    // DVPTree::search leaf mode, radius 0 (Tree.cpp:400-480, 531-563)
    while (!(node & 0x80000000u)) {
      const uint32_t iid = node & 0x7fffffffu;
      float d = 0.f;
      if (lane < 4) d = quad_distance<M, T>(qlds, row_ptr<T>(a.in_pivot, a.row_bytes, iid), a.dp, lane);
      d = __shfl(d, 0, 64);
      ndist++;
      const float* borders = a.in_border + (uint64_t)iid * (a.children - 1);
      uint32_t mid = 0;
      for (; mid < a.children - 1; mid++)
        if (d < borders[mid]) break;
      node = a.in_child[(uint64_t)iid * a.children + mid];
    }
    const uint32_t lid = node & 0x7fffffffu;
    // leaves as CSR (a loaded index) or fixed-stride rows (the tree under construction)
    const uint64_t b = a.leaf_count ? (uint64_t)lid * a.leaf_stride : a.leaf_off[lid];
    uint32_t n = a.leaf_count ? a.leaf_count[lid] : (uint32_t)(a.leaf_off[lid + 1] - b);
    if (a.out_leaf) {
      float pd = 0.f;
      if (n != 0 && lane < 4) pd = quad_distance<M, T>(qlds, row_ptr<T>(a.leaf_pivot, a.row_bytes, lid), a.dp, lane);
      if (lane == 0) {
        a.out_leaf[qi] = lid;
        a.out_count[qi] = n;
        a.out_pdist[qi] = pd;
      }
    }
    uint32_t* out = a.seeds + (uint64_t)qi * a.seed_stride;
    if (n > a.seed_stride) n = a.seed_stride;
    for (uint32_t i = lane; i < n; i += 64) out[i] = a.leaf_ids[b + i];
    __syncthreads();
    uint32_t ss = a.seed_size == 0 ? a.k : a.seed_size;
    if (ss > a.k) ss = a.k;
    if (a.all_leaf_nodes) ss = n;
    if (lane == 0) {
      if (n > ss) {
        // thinning (Index.h:1555-1562)
        GlibcRand rnd;
        rnd.seed(lid);
        for (uint32_t i = n; i > ss; i--) {
          double random = ((double)rnd.next() + 1.0) / ((double)2147483647 + 2.0);
          uint32_t idx = (uint32_t)floor((double)i * random);
          out[idx] = out[i - 1];
        }
        n = ss;
      }
      a.seed_count[qi] = n;
      if (a.tree_ndist) a.tree_ndist[qi] = ndist;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Graph search.
// ---------------------------------------------------------------------------

// NCH > 0: L2 over float rows of exactly 16*NCH elements held in registers;
// NCH == -1: long float rows streamed in stages (eval_stream, L2/cosine/angle);
// NCH == 0: the generic comparator of any metric.
template <int M, typename T, int NCH, int G>
__device__ __forceinline__ void eval_any(const T* qlds, const SearchArgs& a, float qfold, const uint32_t* ids,
                                         float* dists, int m) {
  if constexpr (NCH > 0 && M == kL2 && sizeof(T) == 4) {
    eval_l2f_fast<NCH, G>(reinterpret_cast<const float*>(qlds), a.rows, a.row_bytes, ids, dists, m);
  } else if constexpr (NCH < 0 && sizeof(T) == 4) {
    eval_stream<M>(reinterpret_cast<const float*>(qlds), a.rows, a.row_bytes, a.dp, qfold, ids, dists, m);
  } else {
    eval_batch<M, T>(qlds, a.rows, a.row_bytes, a.dp, ids, dists, m);
  }
}

// Chunk minima of the unchecked array: cmin[c] = the smallest key of
// cq[64c, 64c + 64) (~0 when the chunk is empty), so a pop reads one minimum
// per chunk and one chunk instead of every key -- the long searches of a
// construction batch keep thousands of unchecked keys, and their pops were
// most of the batch time.
__device__ __forceinline__ void cq_chunk_min(const uint64_t* cq, uint64_t* cmin, uint32_t ncq, uint32_t c) {
  const uint32_t i = 64 * c + (uint32_t)lane_id();
  const uint64_t m = wave_min_u64(i < ncq ? cq[i] : ~0ull);
  if (lane_id() == 0) cmin[c] = m;
}

// Probe-and-resume schedule (SearchArgs::pause_after): a paused query's
// state to and from its record (PauseLayout).
__device__ __forceinline__ void pause_save(uint8_t* prec, const PauseLayout& play, const SearchState& st,
                                          const uint64_t* spill, uint32_t ncq, uint32_t nspill, uint32_t nres,
                                          float expr, float* prio, uint32_t* qflag) {
  const int lane = lane_id();
  uint64_t* rres = reinterpret_cast<uint64_t*>(prec + play.off_res);
  uint64_t* rcq = reinterpret_cast<uint64_t*>(prec + play.off_cq);
  uint64_t* rsp = reinterpret_cast<uint64_t*>(prec + play.off_spill);
  for (uint32_t i = lane; i < nres; i += 64) rres[i] = st.res[i];
  float live = 0.f;
  auto score = [&](float d) -> float { return d <= expr ? 1.f : 0.f; };
  for (uint32_t i = lane; i < ncq; i += 64) {
    const uint64_t key = st.cq[i];
    rcq[i] = key;
    live += score(key_dist(key));
  }
  for (uint32_t i = lane; i < nspill; i += 64) {
    const uint64_t key = spill[i];
    rsp[i] = key;
    live += score(key_dist(key));
  }
  // the predicted rest of the search: unchecked keys within the exploration
  // radius (rank correlation 0.81 with the remaining work)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) live += __shfl_xor(live, o, 64);
  if (lane == 0) {
    *prio = live;
    *qflag = 1u;
  }
}

__device__ __forceinline__ void pause_restore(const uint8_t* prec, const PauseLayout& play, SearchState& st,
                                           uint64_t* spill, uint8_t* vis, uint32_t epoch, PauseHdr& hv) {
  const int lane = lane_id();
  hv = *reinterpret_cast<const PauseHdr*>(prec);
  const uint64_t* rres = reinterpret_cast<const uint64_t*>(prec + play.off_res);
  const uint64_t* rcq = reinterpret_cast<const uint64_t*>(prec + play.off_cq);
  const uint64_t* rsp = reinterpret_cast<const uint64_t*>(prec + play.off_spill);
  const uint32_t* rpop = reinterpret_cast<const uint32_t*>(prec + play.off_pop);
  auto remark = [&](uint32_t id) {
    const uint32_t b = (id * 0x85EBCA77u) >> st.vf_shift;
    atomicOr(st.vf + (b >> 5), 1u << (b & 31));
    vis[id] = (uint8_t)epoch;
  };
  for (uint32_t i = lane; i < hv.nres; i += 64) st.res[i] = rres[i];
  for (uint32_t i = lane; i < hv.ncq; i += 64) {
    const uint64_t key = rcq[i];
    st.cq[i] = key;
    remark(key_id(key));
  }
  for (uint32_t i = lane; i < hv.nspill; i += 64) {
    const uint64_t key = rsp[i];
    spill[i] = key;
    remark(key_id(key));
  }
  for (uint32_t i = lane; i < hv.npop; i += 64) remark(rpop[i]);
  __syncthreads();
}

// Waves per SIMD: 4 (128 VGPRs) for the register-row L2 form and long L2
// rows; 3 (168 VGPRs) for long cosine/angle rows (C3), whose filter bound and
// comparator want ~214 and spilled 260 B per lane at 128 -- 758-761 ms per
// C3 launch against 824-828 at 4 and 857-859 at 2 (profiles/r5zc, one box)
#ifndef NGT_AMD_C2_WPE
#define NGT_AMD_C2_WPE 4
#endif
template <int M, int NCH, int G>
constexpr int search_waves_per_simd() {
  return (NCH > 0 && G == 1) ? NGT_AMD_C2_WPE : (NCH < 0 ? (M == kL2 ? 4 : 3) : 2);
}
template <int M, typename T, int NCH, int G>
__global__ void __launch_bounds__(64, (search_waves_per_simd<M, NCH, G>())) ngt_graph_search_kernel(SearchArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = lane_id();
  SearchState st;
  uint8_t* p = smem;
  const bool use_hash = a.ht_log2 != 0;
  st.ht = reinterpret_cast<uint32_t*>(p);
  if (use_hash) p += (size_t)4 << a.ht_log2;
  st.vf = a.vf_log2 ? reinterpret_cast<uint32_t*>(p) : nullptr;
  st.vf_shift = 32 - a.vf_log2;
  const uint32_t vf_words = a.vf_log2 ? (1u << a.vf_log2) / 32 : 0u;
  p += (size_t)4 * vf_words;
  st.cq = reinterpret_cast<uint64_t*>(p);
  p += (size_t)8 * a.cq_cap;
  uint64_t* cmin = reinterpret_cast<uint64_t*>(p);
  p += ((size_t)8 * ((a.cq_cap + 63) / 64) + 15) & ~(size_t)15;
  st.res = reinterpret_cast<uint64_t*>(p);
  p += ((size_t)8 * (a.k + 1) + 15) & ~(size_t)15;
  st.nid = reinterpret_cast<uint32_t*>(p);
  p += 256;
  st.nd = reinterpret_cast<float*>(p);
  p += 256;
  T* qlds = reinterpret_cast<T*>(p);
  p += ((size_t)a.dp * sizeof(T) + 15) & ~(size_t)15;
  // 1-byte filter copy (filter_kernels.hip): L2 float rows of dp = 16 * NCH
  constexpr bool kFilterable = NCH > 0 && (NCH & 1) == 0 && M == kL2 && sizeof(T) == 4;
  // cosine / angle bounds for long float rows (streamed comparator)
  constexpr bool kFilterCos = NCH < 0 && (M == kCosine || M == kAngle) && sizeof(T) == 4;
  uint8_t* qb = p;  // the query's filter bytes q'', when filtering
  // neighbours of the current expansion whose exact distance is pending, in
  // neighbour order (64 ids; allocated when filtering)
  uint32_t* surv = reinterpret_cast<uint32_t*>(p + (size_t)a.dp);
  bool use_filter = false;
  float fa = 0.f, fb = 0.f, fe = 0.f, fx = 0.f;
  if constexpr (kFilterable || kFilterCos) {
    if (a.fcodes != nullptr && a.fparams[4] != 0.0f) {
      use_filter = true;
      fa = a.fparams[0];
      fb = a.fparams[1];
      fe = a.fparams[2];
      fx = a.fparams[3];
      use_filter = fb > 0.0f;  // b = 0: every element equals a, nothing to reject
    }
  }
  (void)qb; (void)surv; (void)fa; (void)fb; (void)fe; (void)fx;

  const uint32_t slot = blockIdx.x;
  uint8_t* vis = a.vis + (uint64_t)slot * a.vis_stride;
  uint64_t* spill = a.spill + (uint64_t)slot * a.spill_cap;
  const uint32_t hcap = use_hash ? 1u << a.ht_log2 : 0u;
  const uint32_t hlimit = hcap - (hcap >> 2);  // 75 % load factor

  // launch schedule (SearchArgs::order / nwork_dev / pause_after)
  const uint32_t nwork = a.nwork_dev ? *a.nwork_dev : a.nq;
  for (;;) {
    uint32_t w = 0;
    if (lane == 0) w = atomicAdd(a.work, 1u);
    w = (uint32_t)__builtin_amdgcn_readfirstlane((int)w);
    if (w >= nwork) break;
    const uint32_t qi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(a.order ? a.order[w] : w));
    // a query the probe launch paused: its saved state, not the seeds
    const bool resume = a.qflag != nullptr && __builtin_amdgcn_readfirstlane((int)a.qflag[qi]) == 1;

    // ---- per-query init -----------------------------------------------
    for (uint32_t i = lane; i < hcap; i += 64) st.ht[i] = 0u;
    for (uint32_t i = lane; i < vf_words; i += 64) st.vf[i] = 0u;
    load_query<T>(qlds, a.queries + (uint64_t)qi * a.query_bytes, a.dp);
    // next epoch of this slot's visited bytes; wipe the array every 255 queries
    uint32_t epoch = a.slot_epoch[slot] + 1;
    if (epoch > 255) {
      uint4* v4 = reinterpret_cast<uint4*>(vis);
      for (uint64_t i = lane; i < a.vis_stride / 16; i += 64) v4[i] = make_uint4(0, 0, 0, 0);
      epoch = 1;
    }
    __syncthreads();
    if (lane == 0) a.slot_epoch[slot] = epoch;
    float qfold = 0.f;
    if constexpr (NCH < 0 && (M == kCosine || M == kAngle))
      qfold = query_sq_fold(reinterpret_cast<const float*>(qlds), a.dp);
    // filter bytes of the query, sum q''^2 and r_q (search_common.h, filter_l2u8)
    uint32_t fsq = 0u;
    double frq = 0.0, finv_b = 0.0;
    (void)fsq; (void)frq; (void)finv_b;
    if constexpr (kFilterable) {
      if (use_filter) {
        filter_query(reinterpret_cast<const float*>(qlds), a.dp, fa, fb, qb, fsq, frq);
        finv_b = 1.0 / (double)fb;
        __syncthreads();
      }
    }
    CosFilterQuery fcq{};
    (void)fcq;
    if constexpr (kFilterCos) {
      if (use_filter) {
        filter_query_cos(reinterpret_cast<const float*>(qlds), a.dp, fa, fb, qb, fcq);
        __syncthreads();
      }
    }

    bool bitmap_mode = !use_hash;
    const bool lazy = a.accepted_only && !use_hash && st.vf;
    uint32_t nvisited = 0;
    uint32_t ncq = 0, nspill = 0, nres = 0, maxq = 0;
    uint64_t ndist = 0, nvisit = 0, nexp = 0, nedge = 0, nexact = 0;
    uint64_t t_pop = 0, t_adj = 0, t_filt = 0, t_eval = 0, t_last = 0, t_rest = 0;
    (void)t_pop; (void)t_adj; (void)t_filt; (void)t_eval; (void)t_last; (void)t_rest;
#ifdef NGT_AMD_STAMPS
    t_last = stamp();
#endif
    float radius = a.radius;
    const uint32_t k = a.k;

    // ---- setupDistances + setupSeeds (Graph.cpp:293-367) ----------------
    const uint64_t sb = a.seed_off ? a.seed_off[qi] : (uint64_t)qi * a.seed_stride;
    const uint32_t ns = a.seed_off ? (uint32_t)(a.seed_off[qi + 1] - sb) : a.seed_count[qi];
    if (resume) {
      // the paused query's state: counters, results, unchecked keys (LDS and
      // this slot's spill), and its accepted-only visited set rebuilt from
      // the popped ids and the unchecked keys in this slot's new epoch
      PauseHdr h;
      pause_restore(a.qstate + (uint64_t)qi * a.qstate_stride, PauseLayout(a.k, a.cq_cap, 0), st, spill, vis, epoch,
                    h);
      ncq = h.ncq;
      nspill = h.nspill;
      nres = h.nres;
      maxq = h.maxq;
      ndist = h.ndist;
      nvisit = h.nvisit;
      nexp = h.nexp;
      nedge = h.nedge;
      nexact = h.nexact;
      for (uint32_t c = 0; c < ((ncq + 63) >> 6); c++) cq_chunk_min(st.cq, cmin, ncq, c);
      __syncthreads();
    }
    for (uint32_t base = 0; base < (resume ? 0u : ns); base += 64) {
      const uint32_t m = ns - base < 64 ? ns - base : 64;
      if ((uint32_t)lane < m) st.nid[lane] = a.seeds[sb + base + lane];
      __syncthreads();
      eval_any<M, T, NCH, G>(qlds, a, qfold, st.nid, st.nd, (int)m);
      __syncthreads();
      if ((uint32_t)lane < m) {
        const uint32_t id = st.nid[lane];
        const uint64_t key = make_key(st.nd[lane], id);
        visit(a.ht_log2, st, id, bitmap_mode, vis, epoch);
        if (ncq + lane < a.cq_cap) st.cq[ncq + lane] = key;
        else spill[nspill + (ncq + lane - a.cq_cap)] = key;
      }
      __syncthreads();
      // results take the k best seeds with d <= radius (sorted order, :347-353)
      for (uint32_t j = 0; j < m; j++) {
        const float d = st.nd[j];
        if (d <= a.radius) res_insert(st.res, nres, k, make_key(d, st.nid[j]));
      }
      const uint32_t ncq0 = ncq;
      if (ncq + m <= a.cq_cap) {
        ncq += m;
      } else {
        nspill += ncq + m - a.cq_cap;
        ncq = a.cq_cap;
      }
      for (uint32_t c = ncq0 >> 6; c < ((ncq + 63) >> 6); c++) cq_chunk_min(st.cq, cmin, ncq, c);
      ndist += m;
      nvisited += m;
      __syncthreads();
      if (!bitmap_mode && nvisited > hlimit) {
        ht_to_vis(a.ht_log2, st, vis, epoch);
        bitmap_mode = true;
        __syncthreads();
      }
    }
    if (nres >= k) radius = key_dist(st.res[k - 1]);
    float expr = __fmul_rn(a.coef, radius);

    // Accept `me` evaluated neighbours (ids[j], distances st.nd[j]) in
    // neighbour order (Graph.cpp:471-483); only candidates within the radius
    // at batch start can be accepted.
    auto accept_batch = [&](const uint32_t* ids, uint32_t me) {
      uint64_t okmask = ballot64((uint32_t)lane < me && st.nd[lane] <= expr);
      while (okmask) {
        const int j = __ffsll((long long)okmask) - 1;
        okmask &= okmask - 1;
        const float d = st.nd[j];
        if (!(d <= expr)) continue;
        const uint64_t key = make_key(d, ids[j]);
        if (lazy && lane == 0) mark_accepted(st, ids[j], vis, epoch);
        if (ncq >= a.cq_cap) {
          ncq = compact(st.cq, ncq, expr);
          if (nspill) nspill = compact(spill, nspill, expr);
          for (uint32_t c = 0; c < ((ncq + 63) >> 6); c++) cq_chunk_min(st.cq, cmin, ncq, c);
          __builtin_amdgcn_wave_barrier();
        }
        if (ncq < a.cq_cap) {
          if (lane == 0) {
            st.cq[ncq] = key;
            const uint32_t c = ncq >> 6;
            cmin[c] = (ncq & 63) == 0 ? key : (key < cmin[c] ? key : cmin[c]);
          }
          ncq++;
        } else {
          if (nspill >= a.spill_cap) {
            if (lane == 0) atomicOr(a.error, 1);
          } else {
            if (lane == 0) spill[nspill] = key;
            nspill++;
          }
        }
        if (ncq + nspill > maxq) maxq = ncq + nspill;  // the largest unchecked set
        if (d <= radius) {
          res_insert(st.res, nres, k, key);
          if (nres >= k) {
            radius = key_dist(st.res[k - 1]);
            expr = __fmul_rn(a.coef, radius);
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      __syncthreads();
      // exact overflow of the visited set into the HBM bitmap
      if (!bitmap_mode && nvisited > hlimit) {
        ht_to_vis(a.ht_log2, st, vis, epoch);
        bitmap_mode = true;
        __syncthreads();
      }
    };

    // Adjacency row prefetch (filtered accepted-only mode): after each pop the
    // row of the next key in line is loaded under the current expansion and
    // used when that key is the next pop (nothing closer was accepted).
    uint32_t pf_node = 0, pf0 = 0, pf1 = 0, pf2 = 0, pf3 = 0;
    (void)pf_node; (void)pf0; (void)pf1; (void)pf2; (void)pf3;

    // ---- best-first loop (Graph.cpp:430-486) ----------------------------
    bool paused = false;
    for (;;) {
      NGT_MARK(t_rest);
      // probe launch: stop here; the state is saved after the loop
      // (only while the popped-id log is complete: a query whose spill held
      // it past the budget runs to its end)
      if (a.pause_after && nexp >= a.pause_after && nexp <= a.pause_after + kPauseStepMax &&
          nspill <= kPauseSpillMax) {
        paused = true;
        break;
      }
      // pop the minimum key
      // best chunk minimum (<= 128 chunks: two per lane), then the spill
      uint64_t best = ~0ull;
      uint32_t bidx = 0xffffffffu;
      const uint32_t nch = (ncq + 63) >> 6;
      if ((uint32_t)lane < nch) { best = cmin[lane]; bidx = (uint32_t)lane; }
      if ((uint32_t)lane + 64 < nch) {
        const uint64_t v = cmin[lane + 64];
        if (v < best) { best = v; bidx = (uint32_t)lane + 64; }
      }
      for (uint32_t i = lane; i < nspill; i += 64) {
        const uint64_t key = spill[i];
        if (key < best) { best = key; bidx = i | 0x80000000u; }
      }
      const uint64_t wbest = wave_min_u64(best);
      if (wbest == ~0ull) break;
      if (key_dist(wbest) > expr) break;
      const uint64_t owner = ballot64(best == wbest);
      const int olane = __ffsll((long long)owner) - 1;
      bidx = __shfl(bidx, olane, 64);
      if (!(bidx & 0x80000000u)) {
        // the key's slot inside its chunk (keys are distinct)
        const uint32_t i = 64 * bidx + (uint32_t)lane;
        const uint64_t in = ballot64(i < ncq && st.cq[i] == wbest);
        if (in == 0) {  // stale chunk minimum: never expected; stop this query loudly
          if (lane == 0) atomicOr(a.error, 4);
          break;
        }
        bidx = 64 * bidx + (uint32_t)(__ffsll((long long)in) - 1);
      }
      if (lane == 0) {
        if (bidx & 0x80000000u) spill[bidx & 0x7fffffffu] = spill[nspill - 1];
        else st.cq[bidx] = st.cq[ncq - 1];
      }
      if (bidx & 0x80000000u) {
        nspill--;
        __syncthreads();
      } else {
        ncq--;
        __syncthreads();
        // the popped slot's chunk took the last key; the last chunk lost it
        cq_chunk_min(st.cq, cmin, ncq, bidx >> 6);
        if ((ncq >> 6) != (bidx >> 6)) cq_chunk_min(st.cq, cmin, ncq, ncq >> 6);
        __syncthreads();
      }
      nexp++;
      NGT_MARK(t_pop);

      const uint32_t target = key_id(wbest);
      // probe launch: the popped ids (the accepted-only visited set of a resume)
      if (a.pause_after && lane == 0 && nexp <= a.pause_after + kPauseStepMax)
        reinterpret_cast<uint32_t*>(a.qstate + (uint64_t)qi * a.qstate_stride +
                                    PauseLayout(a.k, a.cq_cap, 0).off_pop)[nexp - 1] = target;
      // adjacency: padded fixed-stride rows (one load, 0-terminated) or CSR
      uint64_t eb, deg;
      const bool padded = a.adj != nullptr;
      if (padded) {
        eb = (uint64_t)target * a.adj_stride;
        deg = a.adj_stride < a.edge_size ? a.adj_stride : a.edge_size;
      } else {
        eb = a.edge_off[target];
        deg = a.edge_off[target + 1] - eb;
        if (deg > a.edge_size) deg = a.edge_size;
      }

      if constexpr (kFilterable) {
        if (use_filter && lazy && padded && deg <= 256) {
          // Pipelined expansion.  Round trips: the row's ids (none when
          // prefetched), then the filter codes of a 64-id chunk together with
          // the epoch bytes of its filter-positive ids, then one exact-row
          // batch for the survivors of every chunk.  Deferring the exact
          // distances past later chunks only widens the filter threshold
          // those chunks see (the radius never grows), and the survivors are
          // accepted in neighbour order with the current radius: the
          // traversal is the same.
          const uint32_t nchk = (uint32_t)((deg + 63) >> 6);
          uint32_t a0, a1, a2, a3;
          if (pf_node == target) {
            a0 = pf0; a1 = pf1; a2 = pf2; a3 = pf3;
          } else {
            load_adj_row(a.adj + eb, deg, a0, a1, a2, a3);
          }
          // the next key in line: the minimum left after this pop
          {
            uint64_t nb = ~0ull;
            const uint32_t nc2 = (ncq + 63) >> 6;
            if ((uint32_t)lane < nc2) nb = cmin[lane];
            if ((uint32_t)lane + 64 < nc2) { const uint64_t v = cmin[lane + 64]; nb = v < nb ? v : nb; }
            for (uint32_t i = lane; i < nspill; i += 64) { const uint64_t v = spill[i]; nb = v < nb ? v : nb; }
            nb = wave_min_u64(nb);
            pf_node = (nb != ~0ull && key_dist(nb) <= expr) ? key_id(nb) : 0u;
            if (pf_node) load_adj_row(a.adj + (uint64_t)pf_node * a.adj_stride, deg, pf0, pf1, pf2, pf3);
          }
          NGT_MARK(t_adj);
          uint32_t ns = 0;
          for (uint32_t c = 0; c < nchk; c++) {
            const uint32_t id = c == 0 ? a0 : (c == 1 ? a1 : (c == 2 ? a2 : a3));
            const uint64_t vmask = ballot64(id != 0u);
            const uint32_t cnt = (uint32_t)__popcll(vmask);  // 0-terminated: a prefix
            nedge += cnt;
            if (cnt == 0) break;
            // accepted-only visited test: a clear filter bit proves the id
            // fresh; a set bit needs its epoch byte, loaded with the codes
            bool bit = false;
            uint32_t pw = 0;
            if (id != 0u) {
              const uint32_t b = (id * 0x85EBCA77u) >> st.vf_shift;
              bit = ((st.vf[b >> 5] >> (b & 31)) & 1u) != 0u;
              if (bit)
                pw = __hip_atomic_load(reinterpret_cast<const uint32_t*>(vis + (id & ~3u)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            st.nid[lane] = id;
            __syncthreads();
            filter_l2u8<NCH>(qb, fsq, a.fcodes, st.nid, reinterpret_cast<uint32_t*>(st.nd), (int)cnt);
            __syncthreads();
            const bool fresh = id != 0u && (!bit || ((pw >> (8 * (id & 3))) & 0xffu) != epoch);
            const uint32_t m = (uint32_t)__popcll(ballot64(fresh));
            ndist += m;
            nvisit += m;
            nvisited += m;
            const uint32_t fthr = filter_threshold(expr, (double)fe, finv_b, frq);
            const bool keep = fresh && reinterpret_cast<const uint32_t*>(st.nd)[lane] <= fthr;
            const uint64_t km = ballot64(keep);
            const uint32_t me = (uint32_t)__popcll(km);
            nexact += me;
            NGT_MARK(t_filt);
            if (ns + me > 64) {
              eval_any<M, T, NCH, G>(qlds, a, qfold, surv, st.nd, (int)ns);
              __syncthreads();
              NGT_MARK(t_eval);
              accept_batch(surv, ns);
              ns = 0;
            }
            if (keep) surv[ns + mbcnt(km)] = id;
            ns += me;
            __syncthreads();
            if (cnt < 64) break;
          }
          if (ns != 0) {
            eval_any<M, T, NCH, G>(qlds, a, qfold, surv, st.nd, (int)ns);
            __syncthreads();
            NGT_MARK(t_eval);
            accept_batch(surv, ns);
          }
          continue;
        }
      }

      for (uint64_t base = 0; base < deg; base += 64) {
        const uint32_t cnt = (uint32_t)(deg - base < 64 ? deg - base : 64);
        uint32_t id = 0;
        if ((uint32_t)lane < cnt) id = padded ? a.adj[eb + base + lane] : a.edges[eb + base + lane];
        const uint64_t vmask = ballot64(id != 0u);
        nedge += (uint64_t)__popcll(vmask);
        const bool fresh = id != 0u && (lazy ? not_accepted(st, id, vis, epoch)
                                             : visit(a.ht_log2, st, id, bitmap_mode, vis, epoch));
        const uint64_t fmask = ballot64(fresh);
        const uint32_t m = (uint32_t)__popcll(fmask);
        if (fresh) st.nid[mbcnt(fmask)] = id;
        nvisited += m;
        __syncthreads();
        NGT_MARK(t_adj);
        // ids whose exact distance is needed: all fresh ones, or the ones the
        // filter bound cannot place outside the exploration radius (kept in
        // neighbour order)
        uint32_t me = m;
        if constexpr (kFilterable) {
          if (use_filter && m != 0) {
            filter_l2u8<NCH>(qb, fsq, a.fcodes, st.nid, reinterpret_cast<uint32_t*>(st.nd), (int)m);
            __syncthreads();
            const uint32_t fthr = filter_threshold(expr, (double)fe, finv_b, frq);
            const bool keep = (uint32_t)lane < m && reinterpret_cast<const uint32_t*>(st.nd)[lane] <= fthr;
            const uint32_t myid = (uint32_t)lane < m ? st.nid[lane] : 0u;
            const uint64_t km = ballot64(keep);
            __syncthreads();
            if (keep) st.nid[mbcnt(km)] = myid;
            me = (uint32_t)__popcll(km);
            __syncthreads();
          }
        }
        if constexpr (kFilterCos) {
          if (use_filter && m != 0) {
            filter_cos_u8<M>(qb, a.fcodes, a.fstride, a.dp, st.nid, st.nd, (int)m, fa, fb, fe, fcq);
            __syncthreads();
            const bool keep = (uint32_t)lane < m && !(st.nd[lane] > expr);
            const uint32_t myid = (uint32_t)lane < m ? st.nid[lane] : 0u;
            const uint64_t km = ballot64(keep);
            __syncthreads();
            if (keep) st.nid[mbcnt(km)] = myid;
            me = (uint32_t)__popcll(km);
            __syncthreads();
          }
        }
        NGT_MARK(t_filt);
        ndist += m;
        nvisit += m;
        nexact += me;
        if (me != 0) {
          eval_any<M, T, NCH, G>(qlds, a, qfold, st.nid, st.nd, (int)me);
          __syncthreads();
          NGT_MARK(t_eval);
          accept_batch(st.nid, me);
        }
        if (padded && vmask != ~0ull) break;  // 0-terminated list ended in this chunk
      }
    }

    if (paused) {
      // save the state, predict the rest of the search by the unchecked keys
      // within the exploration radius, and take the next query
      uint8_t* prec = a.qstate + (uint64_t)qi * a.qstate_stride;
      if (lane == 0) {
        PauseHdr* h = reinterpret_cast<PauseHdr*>(prec);
        h->ncq = ncq;
        h->nspill = nspill;
        h->nres = nres;
        h->npop = (uint32_t)nexp;
        h->maxq = maxq;
        h->ndist = ndist;
        h->nvisit = nvisit;
        h->nexp = nexp;
        h->nedge = nedge;
        h->nexact = nexact;
      }
      pause_save(prec, PauseLayout(a.k, a.cq_cap, 0), st, spill, ncq, nspill, nres, expr, a.prio + qi,
                 a.qflag + qi);
      __syncthreads();
      continue;
    }
    // ---- results (moveFrom: ascending (distance, id), ObjectSpace.h:49-57)
    for (uint32_t i = lane; i < nres; i += 64) {
      a.out_ids[(uint64_t)qi * a.k + i] = key_id(st.res[i]);
      a.out_dists[(uint64_t)qi * a.k + i] = key_dist(st.res[i]);
    }
    if (lane == 0) {
      a.out_n[qi] = nres;
      if (a.qflag) a.qflag[qi] = 2u;
      if (a.stat) {
        atomicAdd(a.stat, (unsigned long long)nexp);
        atomicAdd(a.stat + 1, 1ull);
      }
      if (a.counters) {
        uint64_t* c = a.counters + (uint64_t)qi * 8;
        c[0] = ndist;
        c[1] = nvisit;
        c[2] = nexp;
        c[3] = (bitmap_mode && use_hash) ? 1 : 0;
        c[4] = nedge;
#ifdef NGT_AMD_STAMPS
        c[5] = t_pop;
        c[6] = t_adj;
        c[7] = t_eval;
        c[3] = t_rest;  // accept + loop overhead
        c[1] = t_filt;  // filter codes + bound (0 without the filter)
#else
        c[5] = maxq;
        c[6] = use_filter ? nexact : ndist - (ns < ndist ? ns : ndist);  // exact distances of neighbours
        c[7] = ns;                                                        // seed distances
#endif
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Linear search: block (slice s, query q) keeps a sorted top-k of its slice;
// a merge kernel combines the slices.
// ---------------------------------------------------------------------------
template <int M, typename T>
__global__ void __launch_bounds__(64) ngt_linear_search_kernel(LinearArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = lane_id();
  uint64_t* res = reinterpret_cast<uint64_t*>(smem);
  uint8_t* p = smem + (((size_t)8 * (a.k + 1) + 15) & ~(size_t)15);
  uint32_t* nid = reinterpret_cast<uint32_t*>(p);
  float* nd = reinterpret_cast<float*>(p + 256);
  T* qlds = reinterpret_cast<T*>(p + 512);
  const uint32_t qi = blockIdx.y;
  const uint32_t slice = blockIdx.x;
  load_query<T>(qlds, a.queries + (uint64_t)qi * a.query_bytes, a.dp);
  __syncthreads();
  const uint64_t per = (a.nrows + gridDim.x - 1) / gridDim.x;
  uint64_t b = (uint64_t)slice * per, e = b + per;
  if (b < 1) b = 1;
  if (e > a.nrows) e = a.nrows;
  uint32_t nres = 0;
  float thr = __int_as_float(0x7f800000);  // +inf: nothing to beat yet
  for (uint64_t base = b; base < e; base += 64) {
    const uint32_t cnt = (uint32_t)(e - base < 64 ? e - base : 64);
    const uint32_t id = (uint32_t)(base + lane);
    const bool ok = (uint32_t)lane < cnt && (a.valid == nullptr || a.valid[id]);
    const uint64_t mask = ballot64(ok);
    const uint32_t m = (uint32_t)__popcll(mask);
    if (ok) nid[mbcnt(mask)] = id;
    __syncthreads();
    eval_batch<M, T>(qlds, a.rows, a.row_bytes, a.dp, nid, nd, (int)m);
    __syncthreads();
    // (radius < 0 || d <= radius), then bounded max-heap == k best (d, id)
    uint64_t cand = ballot64((uint32_t)lane < m && (a.radius < 0.0 || (double)nd[lane] <= a.radius) &&
                            (nres < a.k || nd[lane] <= thr));
    while (cand) {
      const int j = __ffsll((long long)cand) - 1;
      cand &= cand - 1;
      const uint64_t key = make_key(nd[j], nid[j]);
      if (nres >= a.k && key > res[a.k - 1]) continue;
      res_insert(res, nres, a.k, key);
      if (nres >= a.k) thr = key_dist(res[a.k - 1]);
    }
    __syncthreads();
  }
  uint64_t* out = a.partial + ((uint64_t)qi * gridDim.x + slice) * a.k;
  for (uint32_t i = lane; i < a.k; i += 64) out[i] = i < nres ? res[i] : ~0ull;
}

__global__ void __launch_bounds__(64) ngt_linear_merge_kernel(LinearArgs a, uint32_t nslices) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t* res = reinterpret_cast<uint64_t*>(smem);
  const int lane = lane_id();
  const uint32_t qi = blockIdx.x;
  uint32_t nres = 0;
  const uint64_t* part = a.partial + (uint64_t)qi * nslices * a.k;
  for (uint64_t base = 0; base < (uint64_t)nslices * a.k; base += 64) {
    const uint64_t i = base + lane;
    const uint64_t key = i < (uint64_t)nslices * a.k ? part[i] : ~0ull;
    uint64_t cand = ballot64(key != ~0ull && (nres < a.k || key < res[a.k - 1]));
    while (cand) {
      const int j = __ffsll((long long)cand) - 1;
      cand &= cand - 1;
      const uint64_t kj = __shfl(key, j, 64);
      if (nres >= a.k && kj > res[a.k - 1]) continue;
      res_insert(res, nres, a.k, kj);
    }
  }
  for (uint32_t i = lane; i < nres; i += 64) {
    a.out_ids[(uint64_t)qi * a.k + i] = key_id(res[i]);
    a.out_dists[(uint64_t)qi * a.k + i] = key_dist(res[i]);
  }
  if (lane == 0) a.out_n[qi] = nres;
}

// ---------------------------------------------------------------------------
// Shard merge (repository sharded over GPUs): per query, the
// k best (distance, global id) keys of nparts sorted per-shard result lists
// gathered from every rank -- ObjectDistance ordering (Common.h:1946-1959),
// so ties across shards resolve by id exactly as one index would.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) ngt_merge_results_kernel(MergeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t* keys = reinterpret_cast<uint64_t*>(smem);
  const int lane = lane_id();
  const uint32_t total = a.nparts * a.k;
  for (uint32_t qi = blockIdx.x; qi < a.nq; qi += gridDim.x) {
    for (uint32_t i = lane; i < total; i += 64) {
      const uint32_t s = i / a.k, j = i - s * a.k;
      const uint64_t at = ((uint64_t)s * a.nq + qi) * a.k + j;
      const uint32_t n = a.in_n[(uint64_t)s * a.nq + qi];
      keys[i] = j < n ? make_key(a.in_dists[at], a.in_ids[at] + a.id_offsets[s]) : ~0ull;
    }
    __syncthreads();
    uint32_t valid = 0;
    for (uint32_t i = lane; i < total; i += 64) {
      const uint64_t key = keys[i];
      if (key == ~0ull) continue;
      valid++;
      uint32_t rank = 0;
      for (uint32_t j = 0; j < total; j++) rank += keys[j] < key ? 1u : 0u;
      if (rank < a.k) {
        a.out_ids[(uint64_t)qi * a.k + rank] = key_id(key);
        a.out_dists[(uint64_t)qi * a.k + rank] = key_dist(key);
      }
    }
    valid = wave_sum_u32(valid);
    if (lane == 0) a.out_n[qi] = valid < a.k ? valid : a.k;
    __syncthreads();
  }
}

// Packed shard messages: one uint64 per result slot, the NGT::ObjectDistance
// pair {uint32 id, float distance} (Common.h:1937-1992) as (distance bits << 32
// | shard-local id); 0 = empty (ids are 1-based, ObjectRepository.h:37-40).
// One all-gather of these [nq][k] words is the whole shard exchange.
__global__ void __launch_bounds__(256) ngt_pack_results_kernel(const uint32_t* ids, const float* dists,
                                                               const uint32_t* n, uint32_t nq, uint32_t k,
                                                               uint64_t* out) {
  const uint64_t total = (uint64_t)nq * k;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t q = (uint32_t)(i / k), j = (uint32_t)(i - (uint64_t)q * k);
    const uint32_t id = j < n[q] ? ids[i] : 0u;
    out[i] = id ? ((uint64_t)__float_as_uint(dists[i]) << 32) | id : 0ull;
  }
}

__global__ void __launch_bounds__(64) ngt_merge_packed_kernel(MergeArgs a, const uint64_t* packed) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t* keys = reinterpret_cast<uint64_t*>(smem);
  const int lane = lane_id();
  const uint32_t total = a.nparts * a.k;
  const uint64_t stride = a.part_stride ? a.part_stride : (uint64_t)a.nq * a.k;
  if (a.err_out && blockIdx.x == 0 && (uint32_t)lane < a.nparts) {
    const int f = (int)(uint32_t)packed[(uint64_t)lane * stride + (uint64_t)a.nq * a.k];
    if (f) atomicOr(a.err_out, f);
  }
  for (uint32_t qi = blockIdx.x; qi < a.nq; qi += gridDim.x) {
    for (uint32_t i = lane; i < total; i += 64) {
      const uint32_t s = i / a.k, j = i - s * a.k;
      const uint64_t w = packed[(uint64_t)s * stride + (uint64_t)qi * a.k + j];
      const uint32_t id = (uint32_t)w;
      keys[i] = id ? make_key(__uint_as_float((uint32_t)(w >> 32)), id + a.id_offsets[s]) : ~0ull;
    }
    __syncthreads();
    uint32_t valid = 0;
    for (uint32_t i = lane; i < total; i += 64) {
      const uint64_t key = keys[i];
      if (key == ~0ull) continue;
      valid++;
      uint32_t rank = 0;
      for (uint32_t j = 0; j < total; j++) rank += keys[j] < key ? 1u : 0u;
      if (rank < a.k) {
        a.out_ids[(uint64_t)qi * a.k + rank] = key_id(key);
        a.out_dists[(uint64_t)qi * a.k + rank] = key_dist(key);
      }
    }
    valid = wave_sum_u32(valid);
    if (lane == 0) a.out_n[qi] = valid < a.k ? valid : a.k;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Host-side launchers (dispatch on metric x object type).
// ---------------------------------------------------------------------------
#define NGT_DISPATCH(METRIC, OTYPE, LAUNCH)                                    \
  do {                                                                         \
    if ((OTYPE) == kFloat) {                                                   \
      switch (METRIC) {                                                        \
        case kL1: LAUNCH(kL1, float); break;                                   \
        case kL2: LAUNCH(kL2, float); break;                                   \
        case kHamming: LAUNCH(kHamming, float); break;                         \
        case kAngle: LAUNCH(kAngle, float); break;                             \
        case kCosine: LAUNCH(kCosine, float); break;                           \
        case kNormalizedAngle: LAUNCH(kNormalizedAngle, float); break;         \
        case kNormalizedCosine: LAUNCH(kNormalizedCosine, float); break;       \
        case kJaccard: LAUNCH(kJaccard, float); break;                         \
        case kSparseJaccard: LAUNCH(kSparseJaccard, float); break;             \
        case kNormalizedL2: LAUNCH(kNormalizedL2, float); break;               \
        case kPoincare: LAUNCH(kPoincare, float); break;                       \
        case kLorentz: LAUNCH(kLorentz, float); break;                         \
        default: return hipErrorInvalidValue;                                  \
      }                                                                        \
    } else if ((OTYPE) == kUint8) {                                            \
      switch (METRIC) {                                                        \
        case kL1: LAUNCH(kL1, uint8_t); break;                                 \
        case kL2: LAUNCH(kL2, uint8_t); break;                                 \
        case kHamming: LAUNCH(kHamming, uint8_t); break;                       \
        case kAngle: LAUNCH(kAngle, uint8_t); break;                           \
        case kCosine: LAUNCH(kCosine, uint8_t); break;                         \
        case kNormalizedAngle: LAUNCH(kNormalizedAngle, uint8_t); break;       \
        case kNormalizedCosine: LAUNCH(kNormalizedCosine, uint8_t); break;     \
        case kJaccard: LAUNCH(kJaccard, uint8_t); break;                       \
        case kNormalizedL2: LAUNCH(kNormalizedL2, uint8_t); break;             \
        case kPoincare: LAUNCH(kPoincare, uint8_t); break;                     \
        case kLorentz: LAUNCH(kLorentz, uint8_t); break;                       \
        default: return hipErrorInvalidValue;                                  \
      }                                                                        \
    } else {                                                                   \
      return hipErrorInvalidValue;                                             \
    }                                                                          \
  } while (0)

hipError_t launch_distances(const DistanceArgs& a, int metric, int otype, hipStream_t s) {
  if (a.npairs == 0) return hipSuccess;
  uint64_t blocks = (a.npairs * 4 + 255) / 256;
  if (blocks > 65536) blocks = 65536;
#define L_DIST(MM, TT) hipLaunchKernelGGL((ngt_distances_kernel<MM, TT>), dim3((uint32_t)blocks), dim3(256), 0, s, a)
  NGT_DISPATCH(metric, otype, L_DIST);
#undef L_DIST
  return hipGetLastError();
}

hipError_t launch_tree_seeds(const TreeSeedArgs& a, int metric, int otype, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const size_t lds = ((size_t)a.dp * (otype == kFloat ? 4 : 1) + 15) & ~(size_t)15;
  uint32_t blocks = a.nq < 8192 ? a.nq : 8192;
#define L_TREE(MM, TT) hipLaunchKernelGGL((ngt_tree_seed_kernel<MM, TT>), dim3(blocks), dim3(64), lds, s, a)
  NGT_DISPATCH(metric, otype, L_TREE);
#undef L_TREE
  return hipGetLastError();
}

size_t search_lds_bytes(const SearchArgs& a, int otype) {
  size_t b = (a.ht_log2 ? ((size_t)4 << a.ht_log2) : 0) + (size_t)8 * a.cq_cap;
  b += ((size_t)8 * ((a.cq_cap + 63) / 64) + 15) & ~(size_t)15;  // chunk minima
  b += a.vf_log2 ? ((size_t)1 << a.vf_log2) / 8 : 0;
  b += ((size_t)8 * (a.k + 1) + 15) & ~(size_t)15;
  b += 512;
  b += ((size_t)a.dp * (otype == kFloat ? 4 : 1) + 15) & ~(size_t)15;
  if (a.fcodes) b += (size_t)a.dp + 256;  // the query's filter bytes and the pending survivors
  return b;
}

// Launch schedule of the resume launch: the queries the probe launch paused
// (qflag 1), in descending predicted rest of their search (prio: unchecked
// keys within the exploration radius), as a counting sort over 1024
// logarithmic buckets in one workgroup; *n_out = their count.  The order
// inside a bucket is whatever the atomics give: any order gives the same
// results, the schedule only decides when each query runs.
__global__ void __launch_bounds__(1024) ngt_schedule_kernel(const uint32_t* qflag, const float* prio, uint32_t nq,
                                                           uint32_t* order, uint32_t* n_out) {
  constexpr uint32_t NB = 1024;
  __shared__ uint32_t hist[NB];
  __shared__ uint32_t part[NB / 64];
  const uint32_t t = threadIdx.x;
  hist[t] = 0u;
  __syncthreads();
  auto bucket = [&](uint32_t q) -> uint32_t {
    const float p = prio[q];
    const float l = __log2f(1.0f + (p > 0.0f ? p : 0.0f)) * 48.0f;
    const uint32_t b = l < (float)(NB - 1) ? (uint32_t)l : NB - 1;
    return NB - 1 - b;  // descending
  };
  for (uint32_t q = t; q < nq; q += NB)
    if (qflag[q] == 1u) atomicAdd(hist + bucket(q), 1u);
  __syncthreads();
  // exclusive prefix over the buckets: per wave of 64, then over the 16 waves
  const uint32_t lane = t & 63, wv = t >> 6;
  const uint32_t v = hist[t];
  uint32_t incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)incl, o, 64);
    if ((int)lane >= o) incl += u;
  }
  if (lane == 63) part[wv] = incl;
  __syncthreads();
  uint32_t base = 0;
  for (uint32_t i = 0; i < wv; i++) base += part[i];
  __syncthreads();
  hist[t] = base + incl - v;  // the bucket's first position
  if (t == NB - 1) *n_out = base + incl;
  __syncthreads();
  for (uint32_t q = t; q < nq; q += NB)
    if (qflag[q] == 1u) order[atomicAdd(hist + bucket(q), 1u)] = q;
}

hipError_t launch_schedule(const uint32_t* qflag, const float* prio, uint32_t nq, uint32_t* order, uint32_t* n_out,
                           hipStream_t s) {
  hipLaunchKernelGGL(ngt_schedule_kernel, dim3(1), dim3(1024), 0, s, qflag, prio, nq, order, n_out);
  return hipGetLastError();
}

hipError_t launch_graph_search(const SearchArgs& a, int metric, int otype, uint32_t slots,
                               hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const size_t lds = search_lds_bytes(a, otype);
  if (metric == kL2 && otype == kFloat && (a.dp == 128 || a.dp == 96)) {
    // Small launches (construction batches: 200 queries, under one wave per
    // CU) are latency-bound: keep 64 rows per wave in flight instead of 16.
    if (a.dp == 128 && slots < 512)
      hipLaunchKernelGGL((ngt_graph_search_kernel<kL2, float, 8, 4>), dim3(slots), dim3(64), lds, s, a);
    else if (a.dp == 128)
      hipLaunchKernelGGL((ngt_graph_search_kernel<kL2, float, 8, 1>), dim3(slots), dim3(64), lds, s, a);
    else
      hipLaunchKernelGGL((ngt_graph_search_kernel<kL2, float, 6, 1>), dim3(slots), dim3(64), lds, s, a);
    return hipGetLastError();
  }
  // long float rows: streamed comparator (C3: 960-d cosine)
  if (otype == kFloat && a.dp > 128 && ((a.dp >> 4) & 3) == 0 && !ngt_amd::knob("NGT_AMD_NO_STREAM")) {
    if (metric == kL2) {
      hipLaunchKernelGGL((ngt_graph_search_kernel<kL2, float, -1, 1>), dim3(slots), dim3(64), lds, s, a);
      return hipGetLastError();
    }
    if (metric == kCosine) {
      hipLaunchKernelGGL((ngt_graph_search_kernel<kCosine, float, -1, 1>), dim3(slots), dim3(64), lds, s, a);
      return hipGetLastError();
    }
    if (metric == kAngle) {
      hipLaunchKernelGGL((ngt_graph_search_kernel<kAngle, float, -1, 1>), dim3(slots), dim3(64), lds, s, a);
      return hipGetLastError();
    }
  }
#define L_SEARCH(MM, TT) hipLaunchKernelGGL((ngt_graph_search_kernel<MM, TT, 0, 1>), dim3(slots), dim3(64), lds, s, a)
  NGT_DISPATCH(metric, otype, L_SEARCH);
#undef L_SEARCH
  return hipGetLastError();
}

hipError_t launch_linear_search(const LinearArgs& a, int metric, int otype, uint32_t nslices,
                                hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const size_t lds = (((size_t)8 * (a.k + 1) + 15) & ~(size_t)15) + 512 +
                     (((size_t)a.dp * (otype == kFloat ? 4 : 1) + 15) & ~(size_t)15);
#define L_LIN(MM, TT) hipLaunchKernelGGL((ngt_linear_search_kernel<MM, TT>), dim3(nslices, a.nq), dim3(64), lds, s, a)
  NGT_DISPATCH(metric, otype, L_LIN);
#undef L_LIN
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_linear_merge(a, nslices, s);
}

hipError_t launch_linear_merge(const LinearArgs& a, uint32_t nslices, hipStream_t s) {
  const size_t lds2 = ((size_t)8 * (a.k + 1) + 15) & ~(size_t)15;
  hipLaunchKernelGGL(ngt_linear_merge_kernel, dim3(a.nq), dim3(64), lds2, s, a, nslices);
  return hipGetLastError();
}

hipError_t launch_pack_results(const uint32_t* ids, const float* dists, const uint32_t* n, uint32_t nq, uint32_t k,
                               uint64_t* out, hipStream_t s) {
  const uint64_t total = (uint64_t)nq * k;
  if (total == 0) return hipSuccess;
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(ngt_pack_results_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, ids, dists, n, nq, k, out);
  return hipGetLastError();
}

hipError_t launch_merge_packed(const MergeArgs& a, const uint64_t* packed, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const size_t lds = (size_t)a.nparts * a.k * sizeof(uint64_t);
  const uint32_t blocks = a.nq < 16384 ? a.nq : 16384;
  hipLaunchKernelGGL(ngt_merge_packed_kernel, dim3(blocks), dim3(64), lds, s, a, packed);
  return hipGetLastError();
}

hipError_t launch_merge_results(const MergeArgs& a, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const size_t lds = (size_t)a.nparts * a.k * sizeof(uint64_t);
  const uint32_t blocks = a.nq < 16384 ? a.nq : 16384;
  hipLaunchKernelGGL(ngt_merge_results_kernel, dim3(blocks), dim3(64), lds, s, a);
  return hipGetLastError();
}

}  // namespace ngt_amd
