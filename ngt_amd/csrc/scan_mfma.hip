// scan_mfma.hip -- the exact batch scan of ObjectSpaceRepository::linearSearch
// (lib/NGT/ObjectSpaceRepository.h:466-502) for float L2 and Cosine as a
// matrix-core filter plus a bit-exact recompute.
//
// Every (row, query) pair gets a dot product from bf16 MFMAs
// (v_mfma_f32_32x32x16_bf16): rows and queries are split into bf16 hi + lo
// parts, and hi*hi + hi*lo + lo*hi carries ~16 mantissa bits, so the filter
// value v' is within a PROVEN bound of the real-number distance (DESIGN.md
// 4d: kappa terms below).  A pair is a candidate only when v' says its
// distance may beat the query's current k-th key; candidates (a handful per
// query and tile once the lists fill) get the reference comparator's own
// distance (quad_distance: the 16-lane FMA order, folds and double sqrt of
// PrimitiveComparator.h) and enter the query's k-best list by (distance, id).
// A pair the filter rejects has a reference distance strictly above the k-th
// key at that moment, so the lists end exactly as the comparator-order scan's.
//
//  * L2: v' = q.x - xnk/2 with xnk = |x|^2 (1 - kappa) folded into the MFMA
//    as one extra k-step (three bf16 terms of xnk against -0.5);
//    candidate iff v' >= H_q = hb_q - thr_s (1 + rho) / 2, hb_q =
//    |q|^2 (1 - kappa) / 2 - kappa |q| Xmax, thr_s the squared-sum bound of
//    the k-th distance.
//  * Cosine: rows and queries are normalized first; v' ~ cos;
//    candidate iff v' >= H_q = (1 - kappa_c) - kth.
//  * rows that are removed / padding carry NaN in the extra column (never
//    candidates), rows with non-finite values (or zero norm for Cosine) -inf
//    (always candidates, the comparator decides); queries likewise through
//    hb = NaN / -inf.
//
// Work: a workgroup (4 waves, one per SIMD) owns 256 queries x one
// contiguous part of the rows and walks it in 128-row tiles; wave (wr, wq)
// computes 64 rows x 128 queries (2 x 4 MFMA tiles, 128 accumulator
// registers).  Operands are stored
// in HBM in fragment order ([32-row tile][k-step][lane][8 bf16]), so a wave
// stages one 1 KiB block per load and reads its fragments conflict-free.
// Workgroups of the same part run on the same XCD (blockIdx -> (xcd, slot))
// and share the part's rows through that XCD's L2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ngt_device.h"
#include "ngt_kernels.h"
#include "search_common.h"

namespace ngt_amd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMxQ = 128;    // queries per workgroup
constexpr int kMxR = 256;    // rows per tile
constexpr int kMxW = kMxR / 32;  // candidate bitmap words per query
constexpr int kMxPend = 16;  // pending candidates per query between processing rounds
constexpr int kMxNst = 4;    // staging ring depth (k-steps in flight: kMxNst - 1)
constexpr int kMxStage = 24576;  // one k-step: rows hi/lo 8 KiB each, queries hi/lo 4 KiB each

__device__ __forceinline__ uint16_t bf16_bits(float v) {
  const __bf16 b = (__bf16)v;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bf16_val(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }

// squared-sum bound of a distance d (as in scan_kernels.hip): any sum whose
// (float)sqrt((double)sum) is <= d is below it
__device__ __forceinline__ float scan_sq_bound(float d) {
  if (!(d >= 0.0f) || d >= 3.0e38f) return __builtin_huge_valf();
  const double dn = (double)__uint_as_float(__float_as_uint(d) + 1u);
  const float s2 = (float)(dn * dn);
  return __uint_as_float(__float_as_uint(s2) + 1u);
}

// The comparator on one lane: PrimitiveComparator's 16 AVX-512 accumulator
// lanes as 16 registers (lane l: dims l, l+16, ...), the 16 -> 8 -> 4 folds
// and (x0 + x1) + (x2 + x3) exactly as fold16 (ngt_device.h), double sqrt /
// double cosine -- bit for bit dist_f32<M>.
__device__ __forceinline__ float fold16_lane(const float* v) {
  float t8[8], t4[4];
#pragma unroll
  for (int j = 0; j < 8; j++) t8[j] = v[j + 8] + v[j];
#pragma unroll
  for (int j = 0; j < 4; j++) t4[j] = t8[j + 4] + t8[j];
  return (t4[0] + t4[1]) + (t4[2] + t4[3]);
}
template <int M>
__device__ __forceinline__ float dist_lane(const float* __restrict__ q, const float* __restrict__ x, int dp) {
  const float4* q4 = reinterpret_cast<const float4*>(q);
  const float4* x4 = reinterpret_cast<const float4*>(x);
  if constexpr (M == kL2) {
    float acc[16];
#pragma unroll
    for (int l = 0; l < 16; l++) acc[l] = 0.0f;
#pragma unroll 2
    for (int i = 0; i < (dp >> 4); i++) {
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const float4 qv = q4[4 * i + c], xv = x4[4 * i + c];
        const float d0 = qv.x - xv.x, d1 = qv.y - xv.y, d2 = qv.z - xv.z, d3 = qv.w - xv.w;
        acc[4 * c + 0] = __builtin_fmaf(d0, d0, acc[4 * c + 0]);
        acc[4 * c + 1] = __builtin_fmaf(d1, d1, acc[4 * c + 1]);
        acc[4 * c + 2] = __builtin_fmaf(d2, d2, acc[4 * c + 2]);
        acc[4 * c + 3] = __builtin_fmaf(d3, d3, acc[4 * c + 3]);
      }
    }
    return (float)sqrt((double)fold16_lane(acc));
  } else {  // kCosine
    float na[16], nb[16], sv[16];
#pragma unroll
    for (int l = 0; l < 16; l++) na[l] = nb[l] = sv[l] = 0.0f;
#pragma unroll 2
    for (int i = 0; i < (dp >> 4); i++) {
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const float4 qv = q4[4 * i + c], xv = x4[4 * i + c];
        const float qa[4] = {qv.x, qv.y, qv.z, qv.w}, xa[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          na[4 * c + e] = __builtin_fmaf(qa[e], qa[e], na[4 * c + e]);
          nb[4 * c + e] = __builtin_fmaf(xa[e], xa[e], nb[4 * c + e]);
          sv[4 * c + e] = __builtin_fmaf(xa[e], qa[e], sv[4 * c + e]);
        }
      }
    }
    const double dna = fold16_lane(na), dnb = fold16_lane(nb), ds = fold16_lane(sv);
    const double cs = ds / sqrt(dna * dnb);
    return (float)(1.0 - cs);
  }
}

// ---------------------------------------------------------------------------
// Operand preparation: one wave per 32-object tile.  Lane (h = l >> 5,
// r = l & 31) writes, per k-step s, dims 16s + 8h .. +7 of object 32t + r.
// ---------------------------------------------------------------------------
template <bool COS, bool QUERY>
__global__ void __launch_bounds__(64) ngt_scan_prep_kernel(ScanPrepArgs a) {
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const int nk = a.dp >> 4;
  for (uint64_t t = blockIdx.x; t < a.ntiles32; t += gridDim.x) {
    const uint64_t id = t * 32 + r;
    const bool ok = id < a.n && (QUERY || a.valid == nullptr || a.valid[id]);
    const float* x = reinterpret_cast<const float*>(a.src + (ok ? id : 0) * a.stride);
    float ss = 0.0f;
    bool fin = true;
    if (ok) {
      for (int s = 0; s < nk; s++) {
        const float4 u = *reinterpret_cast<const float4*>(x + 16 * s + 8 * h);
        const float4 v = *reinterpret_cast<const float4*>(x + 16 * s + 8 * h + 4);
        const float e[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 8; j++) {
          ss = __builtin_fmaf(e[j], e[j], ss);
          fin = fin && __builtin_isfinite(e[j]);
        }
      }
    }
    ss += __shfl_xor(ss, 32, 64);
    fin = __shfl_xor((int)fin, 32, 64) != 0 && fin;
    fin = fin && __builtin_isfinite(ss);
    const bool forced = ok && (!fin || (COS && !(ss > 0.0f)));
    const bool use = ok && !forced;
    const float scale = COS && use ? 1.0f / sqrtf(ss) : 1.0f;
    uint16_t* oh = a.out_h + (t * a.ks) * 512 + lane * 8;
    uint16_t* ol = a.out_l + (t * a.ks) * 512 + lane * 8;
    for (int s = 0; s < nk; s++) {
      uint16_t hv[8], lv[8];
      float e[8];
      if (use) {
        const float4 u = *reinterpret_cast<const float4*>(x + 16 * s + 8 * h);
        const float4 v = *reinterpret_cast<const float4*>(x + 16 * s + 8 * h + 4);
        e[0] = u.x; e[1] = u.y; e[2] = u.z; e[3] = u.w; e[4] = v.x; e[5] = v.y; e[6] = v.z; e[7] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) e[j] = 0.0f;
      }
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const float v = e[j] * scale;
        hv[j] = bf16_bits(v);
        lv[j] = bf16_bits(v - bf16_val(hv[j]));
      }
      uint4 ph, pl;
      ph.x = hv[0] | (uint32_t)hv[1] << 16; ph.y = hv[2] | (uint32_t)hv[3] << 16;
      ph.z = hv[4] | (uint32_t)hv[5] << 16; ph.w = hv[6] | (uint32_t)hv[7] << 16;
      pl.x = lv[0] | (uint32_t)lv[1] << 16; pl.y = lv[2] | (uint32_t)lv[3] << 16;
      pl.z = lv[4] | (uint32_t)lv[5] << 16; pl.w = lv[6] | (uint32_t)lv[7] << 16;
      *reinterpret_cast<uint4*>(oh + s * 512) = ph;
      *reinterpret_cast<uint4*>(ol + s * 512) = pl;
    }
    // the extra k-step: rows carry -2 * (their share of the filter value)
    // as three bf16 terms, queries the matching -0.5 weights
    uint16_t ev[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (h == 0) {
      if (QUERY) {
        if (ok) ev[0] = ev[1] = ev[2] = bf16_bits(-0.5f);
      } else if (!ok) {
        ev[0] = 0x7fc0;  // NaN: never a candidate
      } else if (forced) {
        ev[0] = 0xff80;  // -inf: v' = +inf, always a candidate
      } else if (!COS) {
        const float xnk = ss * a.one_minus_kappa;
        ev[0] = bf16_bits(xnk);
        const float r1 = xnk - bf16_val(ev[0]);
        ev[1] = bf16_bits(r1);
        ev[2] = bf16_bits(r1 - bf16_val(ev[1]));
      }
    }
    uint4 pe;
    pe.x = ev[0] | (uint32_t)ev[1] << 16; pe.y = ev[2] | (uint32_t)ev[3] << 16;
    pe.z = ev[4] | (uint32_t)ev[5] << 16; pe.w = ev[6] | (uint32_t)ev[7] << 16;
    *reinterpret_cast<uint4*>(oh + nk * 512) = pe;
    *reinterpret_cast<uint4*>(ol + nk * 512) = make_uint4(0u, 0u, 0u, 0u);
    if (!QUERY) {
      if (!COS) {
        // Xmax: an upper bound of every row's |x| (rounded up twice)
        float nx = use ? sqrtf(ss) * 1.0000005f : 0.0f;
        for (int o = 32; o >= 1; o >>= 1) nx = fmaxf(nx, __shfl_xor(nx, o, 64));
        if (lane == 0 && nx > 0.0f) atomicMax(a.xmax_bits, __float_as_uint(nx));
      }
    } else if (h == 0 && t * 32 + r < a.n_pad) {
      // hb: the filter base; hm: the margin of a threshold taken from the
      // filter values themselves (the first tile's bootstrap)
      float hb, hm = __builtin_huge_valf();
      if (!ok) {
        hb = __builtin_nanf("");
      } else if (forced) {
        hb = -__builtin_huge_valf();
      } else if (COS) {
        hb = 1.0f - a.kappa;
        hm = a.kappa_boot;
      } else {
        const float xmax = __uint_as_float(*a.xmax_bits);
        const float nq = sqrtf(ss) * 1.0000005f;
        hb = 0.5f * ss * a.one_minus_kappa - a.kappa * nq * xmax - a.slack;
        hm = a.kappa_boot * (nq + xmax) * (nq + xmax) + 2.0f * a.slack;
      }
      a.hb[t * 32 + r] = hb;
      a.hm[t * 32 + r] = hm;
    }
  }
}

// ---------------------------------------------------------------------------
// The scan.
// ---------------------------------------------------------------------------
// Workgroup barrier for LDS only.  __syncthreads() would also drain the
// staging ring's LDS-DMA loads (vmcnt(0)); the ring is waited for by count.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int M, int P>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
ngt_scan_mfma_kernel(MfmaScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t k = a.k;
  uint8_t* stage = smem;                                              // [4][24 KiB] ring
  uint64_t* lists = reinterpret_cast<uint64_t*>(smem + kMxNst * kMxStage);  // [256][k]
  uint64_t* thr = lists + (size_t)kMxQ * k;                            // [256] k-th key or ~0
  uint32_t* pend = reinterpret_cast<uint32_t*>(thr + kMxQ);           // [128][16] pending rows
  float* boot = reinterpret_cast<float*>(pend);                        // [128][16] (first tile, before any pending)
  float* pdist = reinterpret_cast<float*>(pend + kMxQ * kMxPend);      // [128][16] their distances
  float* H = pdist + kMxQ * kMxPend;                                   // [128]
  float* HB = H + kMxQ;                                                // [256]
  float* HM = HB + kMxQ;                                               // [256]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(HM + kMxQ);             // [256] list sizes
  uint32_t* pc = cnt + kMxQ;                                           // [256] pending counts
  uint32_t* bits = pc + kMxQ;                                          // [256][4]
  uint32_t* flags = bits + kMxQ * kMxW;                                // [4]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w & 1, wq = w >> 1;
  // the launch covers query blocks mb0 .. mb0 + mblocks - 1; its parts are
  // a multiple of 8 and part p runs on XCD p % 8 (blockIdx % 8 picks the
  // XCD), so the workgroups streaming one part share that XCD's L2
  const uint32_t slot = a.xcd ? blockIdx.x >> 3 : blockIdx.x;
  const uint32_t mb = a.mb0 + slot % a.mblocks;
  const uint32_t part = a.xcd ? (slot / a.mblocks) * 8 + (blockIdx.x & 7) : slot / a.mblocks;
  const uint32_t q0 = mb * kMxQ;
  const uint32_t t0 = part * a.tiles_per_part;
  uint32_t t1 = t0 + a.tiles_per_part;
  if (t1 > a.ntiles) t1 = a.ntiles;
  const uint32_t ks = a.ks;
  const uint64_t row0 = (uint64_t)t0 * kMxR;  // pending rows are offsets from here

  for (int i = tid; i < kMxQ; i += 256) {
    thr[i] = ~0ull;
    cnt[i] = 0;
    pc[i] = 0;
    HB[i] = a.hb[q0 + i];
    HM[i] = a.hm[q0 + i];
    H[i] = HB[i] - a.scale * a.t_init;
  }
  for (int i = tid; i < kMxQ * kMxW; i += 256) bits[i] = 0;
  if (tid < 4) flags[tid] = 0;

  // The comparator's distances of every pending (query, row), then their
  // insertion into the k-lists (one thread per query) and the new filter
  // thresholds.  Called by the whole workgroup.
  auto process = [&]() {
    {  // the comparator's distances: two threads per query
      const uint32_t q = tid & (kMxQ - 1);
      const uint32_t n = min(pc[q], (uint32_t)kMxPend);
      if (n) {
        const float* qp = reinterpret_cast<const float*>(a.queries + (uint64_t)(q0 + q) * a.query_bytes);
        for (uint32_t ci = tid >> 7; ci < n; ci += 2) {
          const uint64_t row = row0 + pend[q * kMxPend + ci];
          pdist[q * kMxPend + ci] =
              dist_lane<M>(qp, reinterpret_cast<const float*>(a.rows + row * a.row_bytes), a.dp);
        }
      }
    }
    lds_barrier();
    if (tid < kMxQ && pc[tid]) {
      const uint32_t n = min(pc[tid], (uint32_t)kMxPend);
      uint32_t c = cnt[tid];
      uint64_t* L = lists + (size_t)tid * k;
      uint64_t th = thr[tid];
      for (uint32_t ci = 0; ci < n; ci++) {
        const float d = pdist[tid * kMxPend + ci];
        if (!(a.radius < 0.0 || (double)d <= a.radius)) continue;
        const uint64_t key = make_key(d, (uint32_t)(row0 + pend[tid * kMxPend + ci]));
        if (key >= th) continue;
        bool dup = false;  // a pair seen again on the bitmap path
        for (uint32_t j = 0; j < c; j++) dup = dup || L[j] == key;
        if (dup) continue;
        uint32_t p = c < k ? c : k - 1;  // the k-th entry drops out when full
        while (p > 0 && L[p - 1] > key) {
          L[p] = L[p - 1];
          p--;
        }
        L[p] = key;
        if (c < k) c++;
        if (c >= k) th = L[k - 1];
      }
      if (a.stats) atomicAdd(&a.stats[0], (unsigned long long)n);
      pc[tid] = 0;
      thr[tid] = th;
      cnt[tid] = c;
    }
    if (tid < kMxQ && q0 + tid < a.nq) {
      // every part's k-th key bounds the query's global k-th key: publish
      // this part's, take the smallest over the parts for the filter
      const uint64_t th = thr[tid];
      const uint64_t g = __hip_atomic_fetch_min(a.gthr + q0 + tid, (unsigned long long)th, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t best = g < th ? g : th;
      if (best != ~0ull) {
        const float kd = key_dist(best);
        const float tv = M == kL2 ? fminf(a.t_init, scan_sq_bound(kd)) : fminf(a.t_init, kd);
        H[tid] = fmaxf(H[tid], HB[tid] - a.scale * tv);
      }
    }
    if (a.stats && tid == 0) atomicAdd(&a.stats[1], 1ull);
    lds_barrier();
  };

  // staging ring: k-step g of the part (tile t0 + g / ks, k-step g % ks)
  // goes to slot g % 4 by LDS-DMA; wave w moves blocks w, 4 + w, ... of the
  // 24 1-KiB blocks (rows hi, rows lo: 8 tiles each; queries hi, lo: 4
  // tiles each), so the image is the fragment order of the HBM arrays
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const uint32_t G = (t1 > t0 ? t1 - t0 : 0) * ks;
  auto issue = [&](uint32_t g) {
    uint8_t* base = stage + (g % kMxNst) * kMxStage + w * 1024;
    const uint32_t gg = g < G ? g : G - 1;  // past the end: a harmless reload
    const uint32_t rt = t0 + gg / ks, s = gg - (gg / ks) * ks;
    const size_t ro0 = (((size_t)rt * 8 + w) * ks + s) * 512 + (size_t)lane * 8;
    const size_t ro1 = ro0 + (size_t)4 * ks * 512;
    const size_t qo = (((size_t)mb * 4 + w) * ks + s) * 512 + (size_t)lane * 8;
    __builtin_amdgcn_global_load_lds((const void*)(a.rh + ro0), (lds_ptr)(base), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(a.rh + ro1), (lds_ptr)(base + 4096), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(a.qh + qo), (lds_ptr)(base + 16384), 16, 0, 0);
    if (P == 3) {  // the lo parts
      __builtin_amdgcn_global_load_lds((const void*)(a.rl + ro0), (lds_ptr)(base + 8192), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(a.rl + ro1), (lds_ptr)(base + 12288), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(a.ql + qo), (lds_ptr)(base + 20480), 16, 0, 0);
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; mt++)
#pragma unroll
    for (int nt = 0; nt < 2; nt++) acc[mt][nt] = (f32x16){};

  __syncthreads();
  if (G) {
    issue(0);
    issue(1);
    issue(2);
  }
  const int ql0 = wq * 64 + (lane & 31);  // this lane's query in n-tile 0
  const int rsh = 4 * (lane >> 5);
  for (uint32_t g = 0; g < G; g++) {
    const uint32_t rt = t0 + g / ks, s = g - (g / ks) * ks;
    // k-step g has landed once at most k-steps g+1, g+2 (2P loads each) are
    // outstanding; the barrier publishes every wave's blocks and retires the
    // reads of slot (g + 3) % 4, which is refilled right after
    if (P == 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    lds_barrier();
    issue(g + 3);
    // hi x hi + hi x lo + lo x hi (the norm column's lo parts are 0)
    {
      const uint8_t* sb = stage + (g % kMxNst) * kMxStage + lane * 16;
      bf16x8 ah[4], al[4], bh[2], bl[2];
#pragma unroll
      for (int mt = 0; mt < 4; mt++) {
        ah[mt] = *reinterpret_cast<const bf16x8*>(sb + (wr * 4 + mt) * 1024);
        if (P == 3) al[mt] = *reinterpret_cast<const bf16x8*>(sb + 8192 + (wr * 4 + mt) * 1024);
      }
#pragma unroll
      for (int nt = 0; nt < 2; nt++) {
        bh[nt] = *reinterpret_cast<const bf16x8*>(sb + 16384 + (wq * 2 + nt) * 1024);
        if (P == 3) bl[nt] = *reinterpret_cast<const bf16x8*>(sb + 20480 + (wq * 2 + nt) * 1024);
      }
#pragma unroll
      for (int mt = 0; mt < 4; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
          if (P == 3) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[mt], bh[nt], acc[mt][nt], 0, 0, 0);
          }
        }
    }
    if (s + 1 < ks) continue;

    if (a.dbg & 1) {
#pragma unroll
      for (int mt = 0; mt < 4; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++) acc[mt][nt] = (f32x16){};
      continue;
    }
    if (rt == t0) {
      // bootstrap: the k-th largest of 16 filter values of distinct rows
      // (each lane's 4 largest finite ones of its 32) bounds the k-th
      // distance from above; rows more than the margin HM below it cannot
      // make the top k
#pragma unroll
      for (int nt = 0; nt < 2; nt++) {
        float t4[4] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf(),
                       -__builtin_huge_valf()};
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
#pragma unroll
          for (int e = 0; e < 16; e++) {
            float v = acc[mt][nt][e];
            if (!(v < __builtin_huge_valf())) v = -__builtin_huge_valf();  // NaN, +inf
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const float hi = fmaxf(t4[j], v), lo = fminf(t4[j], v);
              t4[j] = hi;
              v = lo;
            }
          }
        float* bp = boot + (ql0 + nt * 32) * 16 + (wr * 2 + (lane >> 5)) * 4;
#pragma unroll
        for (int j = 0; j < 4; j++) bp[j] = t4[j];
      }
      lds_barrier();
      if (tid < kMxQ && q0 + tid < a.nq) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = boot[tid * 16 + j];
        // k-th largest: k - 1 passes of removing the maximum
        float kth = -__builtin_huge_valf();
        for (uint32_t r = 0; r < k; r++) {
          float mx = -__builtin_huge_valf();
          int at = 0;
#pragma unroll
          for (int j = 0; j < 16; j++)
            if (v[j] > mx) {
              mx = v[j];
              at = j;
            }
          kth = mx;
#pragma unroll
          for (int j = 0; j < 16; j++)
            if (j == at) v[j] = -__builtin_huge_valf();
        }
        const float hb = kth - HM[tid];
        if (hb > H[tid]) H[tid] = hb;
      }
      lds_barrier();
    }

    // ---- filter: lane holds queries ql0 + 32 nt x 64 rows of the tile.
    // Fast path: a 16-value block whose maximum is below the threshold is
    // done in 8 VALU operations; passing values go straight into the query's
    // pending slots (LDS atomics).  A full slot array falls back to the
    // candidate bitmap below.
    float hq[2];
#pragma unroll
    for (int nt = 0; nt < 2; nt++) hq[nt] = H[ql0 + nt * 32];
    const uint32_t rbase = (rt - t0) * kMxR + wr * 128 + rsh;
#pragma unroll
    for (int mt = 0; mt < 4; mt++)
#pragma unroll
      for (int nt = 0; nt < 2; nt++) {
        float mx = acc[mt][nt][0];
#pragma unroll
        for (int e = 1; e < 16; e++) mx = fmaxf(mx, acc[mt][nt][e]);
        const bool hit = mx >= hq[nt];
        if (__ballot(hit)) {
          if (hit) {
            const uint32_t q = ql0 + nt * 32;
#pragma unroll
            for (int e = 0; e < 16; e++)
              if (acc[mt][nt][e] >= hq[nt]) {
                const uint32_t n = atomicAdd(&pc[q], 1u);
                if (n < (uint32_t)kMxPend) pend[q * kMxPend + n] = rbase + mt * 32 + (e & 3) + 8 * (e >> 2);
                if (n + 4 >= (uint32_t)kMxPend) flags[1] = 1;  // process after this tile
                if (n >= (uint32_t)kMxPend) flags[2] = 1;      // overflow: bitmap path
              }
          }
        }
      }
    lds_barrier();
    const uint32_t now = flags[1], over = flags[2];
    lds_barrier();
    if (tid == 0) flags[1] = flags[2] = 0;
    if (a.stats && tid == 0 && now) atomicAdd(&a.stats[2], 1ull);
    if (now && !(a.dbg & 2)) {
      if (tid < kMxQ && pc[tid] > (uint32_t)kMxPend) pc[tid] = kMxPend;
      lds_barrier();
      process();
      if (over) {
        // some passing pairs found no slot: redo the tile through the
        // candidate bitmap with the tightened thresholds (pairs already
        // processed are skipped at insertion, every round takes new bits)
#pragma unroll
        for (int nt = 0; nt < 2; nt++) hq[nt] = H[ql0 + nt * 32];
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
#pragma unroll
          for (int nt = 0; nt < 2; nt++) {
            uint32_t mask = 0;
#pragma unroll
            for (int e = 0; e < 16; e++)
              mask |= (acc[mt][nt][e] >= hq[nt] ? 1u : 0u) << ((e & 3) + 8 * (e >> 2) + rsh);
            if (mask) atomicOr(&bits[(ql0 + nt * 32) * kMxW + wr * 4 + mt], mask);
          }
        lds_barrier();
        for (;;) {
          if (tid < kMxQ) {
            uint32_t n = 0;
            bool rest = false;
#pragma unroll
            for (int wd = 0; wd < kMxW; wd++) {
              uint32_t b = bits[tid * kMxW + wd];
              while (b && n < (uint32_t)kMxPend) {
                pend[tid * kMxPend + n++] = (uint32_t)((rt - t0) * kMxR) + wd * 32 + (__ffs(b) - 1);
                b &= b - 1;
              }
              bits[tid * kMxW + wd] = b;
              rest = rest || b != 0;
            }
            pc[tid] = n;
            if (rest) flags[2] = 1;
          }
          lds_barrier();
          const uint32_t more = flags[2];
          lds_barrier();
          if (tid == 0) flags[2] = 0;
          process();
          if (!more) break;
          // drop the bits the tightened thresholds now exclude
#pragma unroll
          for (int nt = 0; nt < 2; nt++) hq[nt] = H[ql0 + nt * 32];
#pragma unroll
          for (int mt = 0; mt < 4; mt++)
#pragma unroll
            for (int nt = 0; nt < 2; nt++) {
              uint32_t fail = 0;
#pragma unroll
              for (int e = 0; e < 16; e++)
                fail |= (acc[mt][nt][e] >= hq[nt] ? 0u : 1u) << ((e & 3) + 8 * (e >> 2) + rsh);
              if (fail) atomicAnd(&bits[(ql0 + nt * 32) * kMxW + wr * 4 + mt], ~fail);
            }
          lds_barrier();
        }
      }
    }
#pragma unroll
    for (int mt = 0; mt < 4; mt++)
#pragma unroll
      for (int nt = 0; nt < 2; nt++) acc[mt][nt] = (f32x16){};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  process();  // what is still pending at the part's end
  for (uint32_t i = tid; i < (uint32_t)kMxQ * k; i += 256) {
    const uint32_t ql = i / k, r = i - ql * k;
    const uint32_t qi = q0 + ql;
    if (qi < a.nq)
      a.partial[((uint64_t)(qi - a.mb0 * kMxQ) * a.nparts + part) * k + r] = r < cnt[ql] ? lists[i] : ~0ull;
  }
}

size_t scan_mfma_lds_bytes(uint32_t k) {
  return kMxNst * kMxStage + (size_t)kMxQ * k * 8 + kMxQ * 8 + (size_t)kMxQ * kMxPend * 8 + kMxQ * 4 * 5 +
         kMxQ * kMxW * 4 + 16;
}

hipError_t launch_scan_prep(const ScanPrepArgs& a, bool cosine, bool query, hipStream_t s) {
  const uint64_t blocks = a.ntiles32 < 65536 ? a.ntiles32 : 65536;
  if (blocks == 0) return hipSuccess;
  if (cosine) {
    if (query) hipLaunchKernelGGL((ngt_scan_prep_kernel<true, true>), dim3((uint32_t)blocks), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((ngt_scan_prep_kernel<true, false>), dim3((uint32_t)blocks), dim3(64), 0, s, a);
  } else {
    if (query) hipLaunchKernelGGL((ngt_scan_prep_kernel<false, true>), dim3((uint32_t)blocks), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((ngt_scan_prep_kernel<false, false>), dim3((uint32_t)blocks), dim3(64), 0, s, a);
  }
  return hipGetLastError();
}

template <int M, int P>
static void launch_scan_mfma_t(const MfmaScanArgs& a, size_t lds, uint32_t grid, hipStream_t s) {
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)ngt_scan_mfma_kernel<M, P>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL((ngt_scan_mfma_kernel<M, P>), dim3(grid), dim3(256), lds, s, a);
}

hipError_t launch_scan_mfma(const MfmaScanArgs& a, int metric, int passes, hipStream_t s) {
  const size_t lds = scan_mfma_lds_bytes(a.k);
  const uint32_t grid = a.nparts * a.mblocks;
  if (metric == kL2 && passes == 3) launch_scan_mfma_t<kL2, 3>(a, lds, grid, s);
  else if (metric == kL2 && passes == 1) launch_scan_mfma_t<kL2, 1>(a, lds, grid, s);
  else if (metric == kCosine && passes == 3) launch_scan_mfma_t<kCosine, 3>(a, lds, grid, s);
  else if (metric == kCosine && passes == 1) launch_scan_mfma_t<kCosine, 1>(a, lds, grid, s);
  else return hipErrorNotSupported;
  return hipGetLastError();
}

}  // namespace ngt_amd
