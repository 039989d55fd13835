// search_common.h -- device building blocks shared by the exact graph search
// (search_kernels.hip) and the quantized-graph search (qg_kernels.hip): query
// staging, batched row distances, and the per-query search state of
// NeighborhoodGraph::search / NGTQG::Index::searchQuantizedGraph kept in LDS
// (visited set, unchecked set, sorted results).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ngt_device.h"

namespace ngt_amd {

// Diagnostic build only (-DNGT_AMD_STAMPS, libngt_amd_stamps.so): per-query
// shader-clock totals of the search phases land in counters [5..7]; the
// product build compiles these to nothing.
#ifdef NGT_AMD_STAMPS
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define NGT_MARK(dst)              \
  do {                             \
    const uint64_t now_ = stamp(); \
    dst += now_ - t_last;          \
    t_last = now_;                 \
  } while (0)
#else
#define NGT_MARK(dst)
#endif

// glibc random(3) TYPE_3, for srand(leafID) (lib/NGT/Index.h:1555-1559): the
// tree-seed thinning of ngt_tree_seed_kernel and of the serving kernel.
struct GlibcRand {
  uint32_t s[31];
  int f, r;
  __device__ void seed(uint32_t sd) {
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
  __device__ int next() {
    s[f] += s[r];
    int res = (int)((s[f] >> 1) & 0x7fffffff);
    f = f == 30 ? 0 : f + 1;
    r = r == 30 ? 0 : r + 1;
    return res;
  }
};


// a wave-uniform double kept in SGPRs (the shuffle reductions leave the same
// value in every lane, which the compiler cannot see)
__device__ __forceinline__ double uniform_f64(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

template <typename T>
__device__ __forceinline__ const T* row_ptr(const uint8_t* rows, uint64_t row_bytes, uint32_t id) {
  return reinterpret_cast<const T*>(rows + (uint64_t)id * row_bytes);
}

// Copy a padded query row (dp elements) into LDS with 16-byte stores.
template <typename T>
__device__ __forceinline__ void load_query(T* qlds, const uint8_t* src, int dp) {
  const int n16 = (dp * (int)sizeof(T)) >> 4;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(qlds);
  for (int i = lane_id(); i < n16; i += 64) d[i] = s[i];
}

// Distances for `m` candidate ids staged in LDS; 16 rows per wave step,
// 4 lanes per row.  Results land in dists[0..m).
template <int M, typename T>
__device__ __forceinline__ void eval_batch(const T* qlds, const uint8_t* rows, uint64_t row_bytes,
                                           int dp, const uint32_t* ids, float* dists, int m) {
  const int lane = lane_id();
  const int g = lane & 3;
  for (int r0 = 0; r0 < m; r0 += 16) {
    const int r = r0 + (lane >> 2);
    if (r < m) {
      const float d = quad_distance<M, T>(qlds, row_ptr<T>(rows, row_bytes, ids[r]), dp, g);
      if (g == 0) dists[r] = d;
    }
  }
}

// One adjacency row of the padded fixed-stride copy, all chunks in one round
// trip: lane l holds ids l, l + 64, l + 128, l + 192 (0 past `deg`).
__device__ __forceinline__ void load_adj_row(const uint32_t* row, uint64_t deg, uint32_t& r0, uint32_t& r1,
                                             uint32_t& r2, uint32_t& r3) {
  const uint32_t l = (uint32_t)lane_id();
  r0 = l < deg ? row[l] : 0u;
  r1 = l + 64 < deg ? row[l + 64] : 0u;
  r2 = l + 128 < deg ? row[l + 128] : 0u;
  r3 = l + 192 < deg ? row[l + 192] : 0u;
}

// ---------------------------------------------------------------------------
// Graph search.
// ---------------------------------------------------------------------------
struct SearchState {
  uint32_t* ht;      // visited hash (LDS)
  uint32_t* vf;      // visited filter bits (LDS) in front of the HBM epochs, or null
  uint32_t vf_shift; // 32 - log2(filter bits)
  uint64_t* cq;      // unchecked keys (LDS)
  uint64_t* res;     // sorted results (LDS)
  uint32_t* nid;     // staged candidate ids (LDS, 64)
  float* nd;         // staged distances (LDS, 64)
};

__device__ __forceinline__ uint32_t ht_hash(uint32_t id, uint32_t shift) {
  return (id * 0x9E3779B1u) >> shift;
}

// Insert `id` into the visited set; true if it was not present.  Two exact
// forms: an LDS open-addressing hash (small searches), or the slot's HBM
// byte array of query epochs (vis[id] == epoch <=> visited).  The byte form
// needs no read-modify-write: the test is a plain L2 load (sc1, so this CU's
// L1 cannot serve a stale line) and the mark is a plain byte store -- no
// scattered device atomics (MI355X_MICROARCH.md, Global float atomics: 64 lanes
// in 64 rows run ~17x slower than contiguous).
__device__ __forceinline__ bool visit(uint32_t ht_log2, SearchState& st, uint32_t id, bool vis_mode,
                                      uint8_t* vis, uint32_t epoch) {
  if (vis_mode) {
    // LDS filter: one bit per hash of every visited id.  A clear bit proves
    // the id unvisited, so the HBM probe (a 128-B line fetch for one byte) is
    // skipped and only the mark is stored; a set bit falls through to the probe.
    if (st.vf) {
      const uint32_t b = (id * 0x85EBCA77u) >> st.vf_shift;
      const uint32_t m = 1u << (b & 31);
      const uint32_t old = atomicOr(st.vf + (b >> 5), m);
      if (!(old & m)) {
        if (ht_log2) st.ht[ht_hash(id, 32 - ht_log2)] = id;
        vis[id] = (uint8_t)epoch;
        return true;
      }
    }
    // With an LDS table (ht_log2 != 0) it stays on as a direct-mapped cache of
    // visited ids in front of the epoch bytes: only visited ids are ever
    // written to it, so a hit is exact and a miss falls through to HBM.
    uint32_t h = 0;
    if (ht_log2) {
      h = ht_hash(id, 32 - ht_log2);
      if (st.ht[h] == id) return false;
    }
    const uint32_t* w = reinterpret_cast<const uint32_t*>(vis + (id & ~3u));
    const uint32_t word = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t old = (word >> (8 * (id & 3))) & 0xffu;
    if (ht_log2) st.ht[h] = id;
    if (old == epoch) return false;
    vis[id] = (uint8_t)epoch;
    return true;
  }
  const uint32_t mask = (1u << ht_log2) - 1;
  uint32_t h = ht_hash(id, 32 - ht_log2);
  for (;;) {
    const uint32_t old = atomicCAS(st.ht + h, 0u, id);
    if (old == 0u) return true;
    if (old == id) return false;
    h = (h + 1) & mask;
  }
}

// Accepted-only visited set (SearchArgs::accepted_only).  The filter and the
// epoch bytes hold only ids that entered the unchecked set (the seeds and every
// neighbour with d <= explorationRadius).  A neighbour outside that set is
// evaluated even if it was evaluated before: it was rejected then with
// d > explorationRadius, the radius only shrinks, so it is rejected again and
// the traversal and results are the reference's (Graph.cpp:462-483); only the
// distance count grows by the re-evaluations.  True <=> evaluate `id`.
__device__ __forceinline__ bool not_accepted(const SearchState& st, uint32_t id, const uint8_t* vis,
                                             uint32_t epoch) {
  const uint32_t b = (id * 0x85EBCA77u) >> st.vf_shift;
  if (!(st.vf[b >> 5] & (1u << (b & 31)))) return true;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(vis + (id & ~3u));
  const uint32_t word = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ((word >> (8 * (id & 3))) & 0xffu) != epoch;
}

__device__ __forceinline__ void mark_accepted(SearchState& st, uint32_t id, uint8_t* vis, uint32_t epoch) {
  const uint32_t b = (id * 0x85EBCA77u) >> st.vf_shift;
  st.vf[b >> 5] |= 1u << (b & 31);
  vis[id] = (uint8_t)epoch;
}

// Move the LDS hash contents into the slot's epoch array (exact overflow path).
__device__ inline void ht_to_vis(uint32_t ht_log2, SearchState& st, uint8_t* vis, uint32_t epoch) {
  const uint32_t n = 1u << ht_log2;
  for (uint32_t i = lane_id(); i < n; i += 64) {
    const uint32_t id = st.ht[i];
    if (id) {
      vis[id] = (uint8_t)epoch;
      if (st.vf) {
        const uint32_t b = (id * 0x85EBCA77u) >> st.vf_shift;
        atomicOr(st.vf + (b >> 5), 1u << (b & 31));
      }
    }
  }
  __threadfence_block();
}

// Sorted insert of `key` into res[0..nres) keeping at most k entries.
__device__ __forceinline__ void res_insert(uint64_t* res, uint32_t& nres, uint32_t k, uint64_t key) {
  const int lane = lane_id();
  uint32_t lt = 0;
  for (uint32_t i = lane; i < nres; i += 64) lt += res[i] < key ? 1u : 0u;
  const uint32_t pos = wave_sum_u32(lt);
  if (pos >= k) return;
  const uint32_t last = nres < k - 1 ? nres : k - 1;  // [pos, last) moves up one
  if (last > pos) {
    for (int c = (int)((last - 1) >> 6); c >= (int)(pos >> 6); c--) {
      const uint32_t i = (uint32_t)c * 64 + lane;
      uint64_t v = 0;
      const bool mv = i >= pos && i < last;
      if (mv) v = res[i];
      __builtin_amdgcn_wave_barrier();
      if (mv) res[i + 1] = v;
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (lane == 0) res[pos] = key;
  __builtin_amdgcn_wave_barrier();
  nres = nres + 1 < k ? nres + 1 : k;
}

// Drop unchecked entries farther than expR (they can never be expanded).
__device__ __forceinline__ uint32_t compact(uint64_t* v, uint32_t n, float expr) {
  const int lane = lane_id();
  uint32_t out = 0;
  for (uint32_t b = 0; b < n; b += 64) {
    const uint32_t i = b + lane;
    uint64_t key = i < n ? v[i] : ~0ull;
    const bool keep = i < n && key_dist(key) <= expr;
    const uint64_t mask = ballot64(keep);
    __builtin_amdgcn_wave_barrier();
    if (keep) v[out + mbcnt(mask)] = key;
    __builtin_amdgcn_wave_barrier();
    out += (uint32_t)__popcll(mask);
  }
  return out;
}

// L2 over float rows with a compile-time chunk count (dp = 16 * NCH): the
// query lives in registers and the loads of two 16-row groups (32 rows,
// 16 KiB at dp = 128) are all issued before the first FMA, so one batch costs
// one memory round trip.  Same quad mapping and folds as dist_f32<kL2>, hence
// bit-identical results.  Out-of-range lanes read the dummy row 0.
template <int NCH>
__device__ __forceinline__ float l2_fold_rows(const float4* qq, const float4 (&v)[NCH]) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < NCH; i++) {
    const float4 q = qq[4 * i];  // query stays in LDS: ds_read_b128, saves 4*NCH VGPRs
    const float vx = q.x - v[i].x, vy = q.y - v[i].y, vz = q.z - v[i].z, vw = q.w - v[i].w;
    acc.x = __builtin_fmaf(vx, vx, acc.x);
    acc.y = __builtin_fmaf(vy, vy, acc.y);
    acc.z = __builtin_fmaf(vz, vz, acc.z);
    acc.w = __builtin_fmaf(vw, vw, acc.w);
  }
  return (float)sqrt((double)fold16(acc));
}

// G = 16-row groups whose loads are in flight together (G=1: 16 rows / 8 KiB
// per round trip at dp=128, low VGPR count, more resident waves; G=2: 32 rows).
template <int NCH, int G>
__device__ __forceinline__ void eval_l2f_fast(const float* qlds, const uint8_t* rows, uint64_t row_bytes,
                                              const uint32_t* ids, float* dists, int m) {
  const int lane = lane_id();
  const int g = lane & 3, rs = lane >> 2;
  const float4* qq = reinterpret_cast<const float4*>(qlds) + g;
  for (int r0 = 0; r0 < m; r0 += 16 * G) {
    float4 v[G][NCH];
#pragma unroll
    for (int j = 0; j < G; j++) {
      if (j == 0 || r0 + 16 * j < m) {
        const int r = r0 + 16 * j + rs;
        const uint32_t id = r < m ? ids[r] : 0u;
        const float4* x = reinterpret_cast<const float4*>(rows + (uint64_t)id * row_bytes) + g;
#pragma unroll
        for (int i = 0; i < NCH; i++) v[j][i] = x[4 * i];
      }
    }
#pragma unroll
    for (int j = 0; j < G; j++) {
      if (j == 0 || r0 + 16 * j < m) {
        const int r = r0 + 16 * j + rs;
        const float d = l2_fold_rows<NCH>(qq, v[j]);
        if (g == 0 && r < m) dists[r] = d;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Long rows (Dp > 128, Dp/16 a multiple of 4; C3: 960 floats = 3,840 B):
// streamed through registers in stages of 4 float4 per lane with the next
// stage's loads issued before the current stage's FMAs, so a 16-row wave
// step keeps 16 rows x 256 B per lane group in flight instead of waiting on
// each unrolled chunk.  Same quad mapping and per-lane FMA order over the
// chunks as dist_f32 (chunk i strictly in order), hence bit-identical.
// Cosine/angle: the query's sum of squares (compareCosine's first
// accumulator, PrimitiveComparator.h:487-553) depends on the query only, so
// it is folded once per query (query_sq_fold) and reused.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float query_sq_fold(const float* qlds, int dp) {
  const int g = lane_id() & 3;
  const float4* qq = reinterpret_cast<const float4*>(qlds) + g;
  float4 na = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = 0; i < (dp >> 4); i++) {
    const float4 qv = qq[4 * i];
    na.x = __builtin_fmaf(qv.x, qv.x, na.x); na.y = __builtin_fmaf(qv.y, qv.y, na.y);
    na.z = __builtin_fmaf(qv.z, qv.z, na.z); na.w = __builtin_fmaf(qv.w, qv.w, na.w);
  }
  return fold16(na);
}

template <int M>
__device__ __forceinline__ void stream_stage(const float4* qq, int c, const float4 (&b)[4], float4& a0, float4& a1) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const float4 qv = qq[4 * (c + k)];
    const float4 xv = b[k];
    if constexpr (M == kL2) {
      const float vx = qv.x - xv.x, vy = qv.y - xv.y, vz = qv.z - xv.z, vw = qv.w - xv.w;
      a0.x = __builtin_fmaf(vx, vx, a0.x); a0.y = __builtin_fmaf(vy, vy, a0.y);
      a0.z = __builtin_fmaf(vz, vz, a0.z); a0.w = __builtin_fmaf(vw, vw, a0.w);
    } else {  // kCosine / kAngle: a0 = sum x^2, a1 = sum x*q
      a0.x = __builtin_fmaf(xv.x, xv.x, a0.x); a0.y = __builtin_fmaf(xv.y, xv.y, a0.y);
      a0.z = __builtin_fmaf(xv.z, xv.z, a0.z); a0.w = __builtin_fmaf(xv.w, xv.w, a0.w);
      a1.x = __builtin_fmaf(xv.x, qv.x, a1.x); a1.y = __builtin_fmaf(xv.y, qv.y, a1.y);
      a1.z = __builtin_fmaf(xv.z, qv.z, a1.z); a1.w = __builtin_fmaf(xv.w, qv.w, a1.w);
    }
  }
}

template <int M>
__device__ __forceinline__ void eval_stream(const float* qlds, const uint8_t* rows, uint64_t row_bytes, int dp,
                                            float qfold, const uint32_t* ids, float* dists, int m) {
  const int lane = lane_id();
  const int g = lane & 3, rs = lane >> 2;
  const float4* qq = reinterpret_cast<const float4*>(qlds) + g;
  const int nch = dp >> 4;  // float4 per lane, a multiple of 4
  for (int r0 = 0; r0 < m; r0 += 16) {
    const int r = r0 + rs;
    const uint32_t id = r < m ? ids[r] : 0u;  // out-of-range lanes read the dummy row
    const float4* x = reinterpret_cast<const float4*>(rows + (uint64_t)id * row_bytes) + g;
    float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
    float4 b0[4], b1[4];
#pragma unroll
    for (int k = 0; k < 4; k++) b0[k] = x[4 * k];
    for (int c = 0; c < nch; c += 8) {
      const bool more = c + 4 < nch;
      if (more) {
#pragma unroll
        for (int k = 0; k < 4; k++) b1[k] = x[4 * (c + 4 + k)];
      }
      stream_stage<M>(qq, c, b0, a0, a1);
      if (!more) break;
      if (c + 8 < nch) {
#pragma unroll
        for (int k = 0; k < 4; k++) b0[k] = x[4 * (c + 8 + k)];
      }
      stream_stage<M>(qq, c + 4, b1, a0, a1);
    }
    float d;
    if constexpr (M == kL2) {
      d = (float)sqrt((double)fold16(a0));
    } else {
      const double dnb = fold16(a0), ds = fold16(a1);
      const double cs = ds / sqrt((double)qfold * dnb);
      if constexpr (M == kCosine) d = (float)(1.0 - cs);
      else d = (float)angle_of(cs);
    }
    if (g == 0 && r < m) dists[r] = d;
  }
}


// ---------------------------------------------------------------------------
// Lower bounds from the 1-byte filter copy (filter_kernels.hip), in exact
// integer arithmetic.  With x~ = a + b c (codes c in [0,255]), q' = (q - a)/b,
// its clamp to [0,255] q^ and the per-query byte vector q'' = rint(q^):
//   ||q - x|| >= ||q - x~|| - E = b ||q' - c|| - E >= b ||q^ - c|| - E
//             >= b (||q'' - c|| - r_q) - E,      r_q = ||q^ - q''||
// (clamping moves q' closer to every code vector; triangle inequality twice).
// out[r] = S = ||q'' - c(r)||^2 = sum q''^2 + sum c^2 - 2 sum q'' c, exact in
// u32 via v_dot4_u32_u8; the caller rejects when S exceeds the square of
// (radius + E)/b + r_q, rounded up.  Quad per row: lane g of a quad takes
// bytes [g E, g E + E), E = dp / 4; 64 rows' codes (4 x 16 rows) are in
// flight before the first dot product.  Not bit-matched to anything: a bound.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t quad_sum_u32(uint32_t s) {
  s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0xb1, 0xf, 0xf, false);  // lane ^ 1
  s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x4e, 0xf, 0xf, false);  // lane ^ 2
  return s;
}

// A lane's NW 8-byte code words of one row, fetched in 16-byte loads when
// they are whole pairs (the row's lanes start 16-B aligned: 128-B code rows,
// 32 B per lane): half the vector-memory instructions of 8-byte loads, each
// touching the same rows' lines -- the per-instruction address work of the
// texture unit, not the bytes, is what these gathers spend (TA busy 0.74 on
// the C2 headline, profiles/r6t).
template <int NW>
__device__ __forceinline__ void load_code_words(const uint8_t* rowp, uint2 (&c)[NW]) {
  if constexpr (NW % 2 == 0) {
    const uint4* p = reinterpret_cast<const uint4*>(rowp);
#pragma unroll
    for (int w = 0; w < NW / 2; w++) {
      const uint4 v = p[w];
      c[2 * w] = make_uint2(v.x, v.y);
      c[2 * w + 1] = make_uint2(v.z, v.w);
    }
  } else {
    const uint2* p = reinterpret_cast<const uint2*>(rowp);
#pragma unroll
    for (int w = 0; w < NW; w++) c[w] = p[w];
  }
}

template <int NCH>
__device__ __forceinline__ void filter_l2u8(const uint8_t* qb, uint32_t sq, const uint8_t* codes,
                                            const uint32_t* ids, uint32_t* out, int m) {
  static_assert((NCH & 1) == 0, "whole 8-byte code words per lane");
  constexpr int E = 4 * NCH;   // bytes per lane
  constexpr int NW = E / 8;    // 8-byte code words per lane
  const int lane = lane_id();
  const int g = lane & 3, rs = lane >> 2;
  uint2 q[NW];
  const uint2* qp = reinterpret_cast<const uint2*>(qb + g * E);
#pragma unroll
  for (int w = 0; w < NW; w++) q[w] = qp[w];
  for (int r0 = 0; r0 < m; r0 += 64) {
    uint2 c[4][NW];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int r = r0 + 16 * j + rs;
      const uint32_t id = r < m ? ids[r] : 0u;
      if (j == 0 || r0 + 16 * j < m) {
        load_code_words<NW>(codes + (uint64_t)id * (4 * E) + g * (8 * NW), c[j]);
      } else {
#pragma unroll
        for (int w = 0; w < NW; w++) c[j][w] = make_uint2(0u, 0u);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (j == 0 || r0 + 16 * j < m) {
        uint32_t qc = 0u, cc = 0u;
#pragma unroll
        for (int w = 0; w < NW; w++) {
          qc = __builtin_amdgcn_udot4(q[w].x, c[j][w].x, qc, false);
          qc = __builtin_amdgcn_udot4(q[w].y, c[j][w].y, qc, false);
          cc = __builtin_amdgcn_udot4(c[j][w].x, c[j][w].x, cc, false);
          cc = __builtin_amdgcn_udot4(c[j][w].y, c[j][w].y, cc, false);
        }
        const uint32_t s = quad_sum_u32(cc - 2u * qc);  // modulo 2^32: the total below is exact
        const int r = r0 + 16 * j + rs;
        if (g == 0 && r < m) out[r] = sq + s;
      }
    }
  }
}

// Per-query filter state: q'' bytes into qb (LDS), sum q''^2 and the
// rounding radius r_q (rounded up); wave-uniform results.
__device__ __forceinline__ void filter_query(const float* qf, int dp, float fa, float fb, uint8_t* qb, uint32_t& sq,
                                             double& rq) {
  uint32_t s = 0u;
  double r2 = 0.0;
  for (int i = lane_id(); i < dp; i += 64) {
    float c = rintf((qf[i] - fa) / fb);
    c = c >= 0.0f ? (c <= 255.0f ? c : 255.0f) : 0.0f;  // NaN -> 0 (r_q is then NaN: no rejection)
    qb[i] = (uint8_t)c;
    s += (uint32_t)c * (uint32_t)c;
    double t = ((double)qf[i] - (double)fa) / (double)fb;
    t = t < 0.0 ? 0.0 : (t > 255.0 ? 255.0 : t);
    r2 += (t - (double)c) * (t - (double)c);
  }
  sq = wave_sum_u32(s);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) r2 += __shfl_xor(r2, o, 64);
  rq = sqrt(r2) * (1.0 + 1e-9) + 1e-9;
}

// The largest S a neighbour may have and still lie within `expr`: the square
// of (expr (1 + 2^-15) + E) / b + r_q, rounded up (the 2^-15 covers the
// comparator's own float rounding); all ones (keep everything) when that is
// not finite or beyond u32.
__device__ __forceinline__ uint32_t filter_threshold(float expr, double fe, double inv_b, double rq) {
  const double t = ((double)expr * (1.0 + 0x1p-15) + fe) * inv_b + rq;
  const double t2 = t * t * (1.0 + 1e-12) + 1e-6;
  if (!(t2 < 4294967295.0)) return 0xffffffffu;
  return (uint32_t)t2;  // floor: S > t2 <=> S > floor(t2) for integer S
}

// ---------------------------------------------------------------------------
// Cosine / angle lower bounds from the 1-byte filter copy (long rows, Dp a
// multiple of 64).  With x = x~ + e, |e| <= E, x~ = a + b c, and the query
// split as q = a + b q'' + r (q'' = rint(clamp((q - a)/b)), r the residual):
//   q.x  <= q.x~ + |q| E,   |x| >= |x~| - E,
//   q.x~ =  a sum q + b (a sum c + b sum q''c + r.c),  r.c <= |r| |c|,
//   |x~|^2 = Dp a^2 + 2ab sum c + b^2 sum c^2,
// so cos(q, x) <= U = (q.x~ + |q| E) / (|q| (|x~| - E)) (1 when |x~| <= E).
// The comparator's float sums (PrimitiveComparator.h:487-553: 16 lanes of
// Dp/16 FMAs and a 16->1 fold) sit within 8e-6 of the real cosine; with 2e-5
// of slack the distance is at least 1 - (U + 2e-5) (cosine) or
// acos(min(1, U + 2e-5)) (angle), stored rounded down.  sum c, sum c^2 and
// sum q''c are exact u32 sums of v_dot4_u32_u8; 16 lanes per row, dword d of
// a row on lane d mod 16 (64 contiguous bytes per row per load instruction),
// 8 rows per wave step.  A bound, not bit-matched to anything.
// ---------------------------------------------------------------------------
struct CosFilterQuery {
  double sum_q;  // sum q_i
  double qn;     // |q|
  double rn;     // |q - a - b q''|
};

__device__ __forceinline__ void filter_query_cos(const float* qf, int dp, float fa, float fb, uint8_t* qb,
                                                 CosFilterQuery& fq) {
  double sq = 0.0, qq = 0.0, rr = 0.0;
  for (int i = lane_id(); i < dp; i += 64) {
    float c = rintf((qf[i] - fa) / fb);
    c = c >= 0.0f ? (c <= 255.0f ? c : 255.0f) : 0.0f;  // NaN -> 0 (the sums are then NaN: no rejection)
    qb[i] = (uint8_t)c;
    const double q = (double)qf[i];
    const double r = q - ((double)fa + (double)fb * (double)c);
    sq += q;
    qq += q * q;
    rr += r * r;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    sq += __shfl_xor(sq, o, 64);
    qq += __shfl_xor(qq, o, 64);
    rr += __shfl_xor(rr, o, 64);
  }
  fq.sum_q = uniform_f64(sq);
  fq.qn = uniform_f64(sqrt(qq));
  fq.rn = uniform_f64(sqrt(rr) * (1.0 + 1e-9) + 1e-12);
}

template <int M>
__device__ __forceinline__ float cos_filter_bound(uint32_t sc, uint32_t scc, uint32_t sqc, int dp, float fa, float fb,
                                                  float fe, const CosFilterQuery& fq) {
  const double a = fa, b = fb, e = fe;
  const double cn = sqrt((double)scc);
  const double qx = a * fq.sum_q + b * (a * (double)sc + b * (double)sqc + fq.rn * cn);
  const double x2 = (double)dp * a * a + 2.0 * a * b * (double)sc + b * b * (double)scc;
  const double xn = sqrt(x2 > 0.0 ? x2 : 0.0);
  double u = 1.0;
  if (xn > e * (1.0 + 1e-9) && fq.qn > 0.0) {
    const double num = qx * (1.0 + 1e-12) + fabs(qx) * 1e-12 + fq.qn * e;
    u = num >= 0.0 ? num / (fq.qn * (xn - e) * (1.0 - 1e-12)) : num / (fq.qn * (xn + e) * (1.0 + 1e-12));
    u += 2e-5;
  }
  if (!(u < 1.0)) u = 1.0;  // NaN included
  if (u < -1.0) u = -1.0;
  const double lb = M == kCosine ? 1.0 - u : acos(u);
  return __double2float_rd(lb * (1.0 - 1e-12));
}

template <int M>
__device__ __forceinline__ void filter_cos_u8(const uint8_t* qb, const uint8_t* codes, uint64_t stride, int dp,
                                              const uint32_t* ids,
                                              float* out, int m, float fa, float fb, float fe,
                                              const CosFilterQuery& fq) {
  const int lane = lane_id();
  const int g = lane & 15, rs = lane >> 4;  // 4 rows per 64 lanes
  const int nw = dp >> 6;                   // dwords per lane per row
  const uint32_t* qw = reinterpret_cast<const uint32_t*>(qb);
  for (int r0 = 0; r0 < m; r0 += 8) {
    const int ra = r0 + rs, rb = r0 + 4 + rs;
    const uint32_t* xa = reinterpret_cast<const uint32_t*>(codes + (uint64_t)(ra < m ? ids[ra] : 0u) * stride);
    const uint32_t* xb = reinterpret_cast<const uint32_t*>(codes + (uint64_t)(rb < m ? ids[rb] : 0u) * stride);
    uint32_t sca = 0u, scca = 0u, sqca = 0u, scb = 0u, sccb = 0u, sqcb = 0u;
    // blocks of 16 dwords per lane: every load of both rows issued before
    // the first dot product (Dp = 960: one block, one round trip)
    for (int kb = 0; kb < nw; kb += 16) {
      uint32_t ca[16], cb[16];
#pragma unroll
      for (int t = 0; t < 16; t++) {
        const int w = g + 16 * (kb + t);
        ca[t] = kb + t < nw ? xa[w] : 0u;
        cb[t] = kb + t < nw ? xb[w] : 0u;
      }
#pragma unroll
      for (int t = 0; t < 16; t++) {
        const uint32_t q = kb + t < nw ? qw[g + 16 * (kb + t)] : 0u;
        sca = __builtin_amdgcn_udot4(ca[t], 0x01010101u, sca, false);
        scca = __builtin_amdgcn_udot4(ca[t], ca[t], scca, false);
        sqca = __builtin_amdgcn_udot4(q, ca[t], sqca, false);
        scb = __builtin_amdgcn_udot4(cb[t], 0x01010101u, scb, false);
        sccb = __builtin_amdgcn_udot4(cb[t], cb[t], sccb, false);
        sqcb = __builtin_amdgcn_udot4(q, cb[t], sqcb, false);
      }
    }
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
      sca += __shfl_xor(sca, o, 16);
      scca += __shfl_xor(scca, o, 16);
      sqca += __shfl_xor(sqca, o, 16);
      scb += __shfl_xor(scb, o, 16);
      sccb += __shfl_xor(sccb, o, 16);
      sqcb += __shfl_xor(sqcb, o, 16);
    }
    // lane 0 of a 16-lane group bounds its row a, lane 1 its row b
    const bool isb = g == 1;
    const int r = isb ? rb : ra;
    if (g < 2 && r < m)
      out[r] = cos_filter_bound<M>(isb ? scb : sca, isb ? sccb : scca, isb ? sqcb : sqca, dp, fa, fb, fe, fq);
  }
}

// ---------------------------------------------------------------------------
// Sorted register heads (lane i = i-th smallest key) and threshold selection
// over LDS/HBM key arrays: the latency kernel's and the lookahead kernel's
// unchecked sets (search_lat.hip, search_la.hip).
// ---------------------------------------------------------------------------
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

}  // namespace ngt_amd
