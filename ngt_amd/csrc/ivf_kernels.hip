// ivf_kernels.hip -- NGTQ IVF-ADC search on gfx950: the aggregation half of
// NGTQ::QuantizerInstance::search (lib/NGT/NGTQ/Quantizer.h:2499-2549).
//
// The global-codebook search (:2248-2262) runs before this kernel on the
// existing graph/linear search kernels; this kernel takes its centroid lists
// and, one 64-lane wave per query, walks the inverted lists in centroid
// order exactly as aggregateObjects (:2423-2441) does:
//   * the first non-empty list is aggregated whole (limit INT_MAX while the
//     result set is empty), every later one only while fewer than
//     approximateSearchSize entries have been aggregated;
//   * an entry's distance is the centroid's distance when its localID[0] is 0
//     (the object is the centroid), else by mode
//       'a' AggregationModeApproximateDistance: getL2DistanceFloat (:579-608),
//       'c'/'r' ...WithCache / ExactDistanceThroughApproximateDistance: the
//           AVX per-subspace residual distances (:1102-1153),
//       'l' ...WithLookupTable: the float LUT (createFloatL2DistanceLookup
//           :683-706) summed by QuantizedObjectDistanceFloat (:942-953),
//       'e' AggregationModeExactDistance: the L2 comparator on the object list;
//   * the ResultSet is popped into ascending (distance, id) order and cut to
//     `size`, so the kernel keeps the `size` smallest keys;
//   * 'r' then recomputes exact distances of those and sorts (refineDistance,
//     :2450-2460).
// A query's residual tables depend only on (query, centroid): they are built
// once per centroid in LDS ([N][17] doubles) with the arithmetic the
// reference's -Ofast -march=native build emits for each function (read from
// its object code and pinned by tests/golden/ngtq_n*): sub = o - (g + l),
// 16-lane zmm FMA accumulators folded 16->8->4->2->1, an 8-lane (o - l) - g
// block, scalar FMA tails; 'c' an 8-lane FMA accumulator folded (x0+x4 ..),
// (s0+s1)+(s3+s2); 'a' double lanes fma(lo, lo, hi * hi).  Entry sums run in
// double in subspace order, the distance is (float)sqrt(sum).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ngt_device.h"
#include "ngt_kernels.h"
#include "search_common.h"

namespace ngt_amd {

// 'l': createFloatL2DistanceLookup's float sum for one (subspace, centroid)
__device__ __forceinline__ float ivf_lut_l(const float* o, const float* g, const float* l, uint32_t dsub) {
  float acc = 0.0f;
  uint32_t i = 0;
  if (dsub >= 16) {
    float a[16];
#pragma unroll
    for (int j = 0; j < 16; j++) a[j] = 0.0f;
    for (; i + 16 <= dsub; i += 16) {
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const float s = o[i + j] - (g[i + j] + l[i + j]);
        a[j] = __builtin_fmaf(s, s, a[j]);
      }
    }
#pragma unroll
    for (int h = 8; h >= 1; h >>= 1)
#pragma unroll
      for (int j = 0; j < h; j++) a[j] = a[j + h] + a[j];
    acc = a[0];
  }
  if (dsub - i >= 8) {
    float b[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const float s = (o[i + j] - l[i + j]) - g[i + j];
      b[j] = s * s;
    }
#pragma unroll
    for (int h = 4; h >= 1; h >>= 1)
#pragma unroll
      for (int j = 0; j < h; j++) b[j] = b[j + h] + b[j];
    acc = acc + b[0];
    i += 8;
  }
  for (; i < dsub; i++) {
    const float s = o[i] - (g[i] + l[i]);
    acc = __builtin_fmaf(s, s, acc);
  }
  return acc;
}

// 'c' / 'r': the 8-lane AVX loop of the cached-distance operator.  The
// reference reads whole 8-float blocks, past the subvector when dsub is not a
// multiple of 8; the host accepts only dsub % 8 == 0 for these modes.
__device__ __forceinline__ double ivf_sub_c(const float* o, const float* g, const float* l, uint32_t dsub) {
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; j++) a[j] = 0.0f;
  for (uint32_t i = 0; i < dsub; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const float s = o[i + j] - (g[i + j] + l[i + j]);
      a[j] = __builtin_fmaf(s, s, a[j]);
    }
  }
  float x[4];
#pragma unroll
  for (int j = 0; j < 4; j++) x[j] = a[j] + a[j + 4];
  return (double)((x[0] + x[1]) + (x[3] + x[2]));
}

// 'a': getL2DistanceFloat's per-subspace double sum.
__device__ __forceinline__ double ivf_sub_a(const float* o, const float* g, const float* l, uint32_t dsub) {
  double d = 0.0;
  uint32_t i = 0;
  if (dsub >= 16) {
    double a[8];
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = 0.0;
    for (; i + 16 <= dsub; i += 16) {
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const double lo = (double)(o[i + j] - (g[i + j] + l[i + j]));
        const double hi = (double)(o[i + j + 8] - (g[i + j + 8] + l[i + j + 8]));
        a[j] = a[j] + __builtin_fma(lo, lo, hi * hi);
      }
    }
#pragma unroll
    for (int h = 4; h >= 1; h >>= 1)
#pragma unroll
      for (int j = 0; j < h; j++) a[j] = a[j + h] + a[j];
    d = a[0];
  }
  if (dsub - i >= 8) {
    double t[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const double lo = (double)(o[i + j] - (g[i + j] + l[i + j]));
      const double hi = (double)(o[i + j + 4] - (g[i + j + 4] + l[i + j + 4]));
      t[j] = __builtin_fma(lo, lo, hi * hi);
    }
    d = d + ((t[3] + t[1]) + (t[2] + t[0]));
    i += 8;
  }
  for (; i < dsub; i++) {
    const double s = (double)(o[i] - (g[i] + l[i]));
    d = __builtin_fma(s, s, d);
  }
  return d;
}

__global__ void __launch_bounds__(64) ngt_ivf_search_kernel(IvfSearchArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = lane_id();
  uint8_t* p = smem;
  float* qlds = reinterpret_cast<float*>(p);
  p += (size_t)4 * a.dp;
  double* tab = reinterpret_cast<double*>(p);  // [N][17]
  p += (((size_t)8 * a.N * 17) + 15) & ~(size_t)15;
  uint64_t* res = reinterpret_cast<uint64_t*>(p);
  p += (((size_t)8 * (a.size + 1)) + 15) & ~(size_t)15;
  uint32_t* nid = reinterpret_cast<uint32_t*>(p);
  p += 4 * 64;
  float* nd = reinterpret_cast<float*>(p);

  const uint32_t ntab = a.N * 16;
  for (uint32_t qi = blockIdx.x; qi < a.nq; qi += gridDim.x) {
    load_query<float>(qlds, a.queries + (uint64_t)qi * a.query_bytes, a.dp);
    __syncthreads();
    uint32_t nres = 0;
    uint64_t count = 0;
    const uint32_t nc = a.cent_n[qi];
    for (uint32_t ci = 0; ci < nc; ci++) {
      const uint32_t gid = a.cent_ids[(uint64_t)qi * a.cent_stride + ci];
      const float gd = a.cent_d[(uint64_t)qi * a.cent_stride + ci];
      if (gid >= a.nlists) continue;  // no inverted list for this centroid
      const uint64_t lo = a.list_off[gid], len = a.list_off[gid + 1] - lo;
      uint64_t m;
      if (count == 0) m = len;
      else m = count < a.ass ? (len < a.ass - count ? len : a.ass - count) : 0;
      if (m == 0) {
        if (count >= a.ass) break;
        continue;
      }
      if (a.mode != kIvfExact) {
        // residual tables of this centroid (entry 0 of each subspace unused)
        const float* g = reinterpret_cast<const float*>(a.grows + (uint64_t)gid * a.grow_bytes);
        for (uint32_t t = lane; t < ntab; t += 64) {
          const uint32_t li = t >> 4, k = (t & 15) + 1;
          const float* o = qlds + li * a.dsub;
          const float* gg = g + li * a.dsub;
          const float* l = a.local + ((uint64_t)li * 17 + k) * a.dsub;
          double v;
          if (a.mode == kIvfLut) v = (double)ivf_lut_l(o, gg, l, a.dsub);
          else if (a.mode == kIvfApprox) v = ivf_sub_a(o, gg, l, a.dsub);
          else v = ivf_sub_c(o, gg, l, a.dsub);
          tab[li * 17 + k] = v;
        }
        __syncthreads();
      }
      for (uint64_t b0 = 0; b0 < m; b0 += 64) {
        const uint64_t e = lo + b0 + lane;
        const bool live = b0 + lane < m;
        const uint32_t id = live ? a.eids[e] : 0u;
        const uint16_t* lid = a.elids + e * a.lid_stride;
        const bool at_centroid = live && lid[0] == 0;
        float d = 0.0f;
        if (a.mode == kIvfExact) {
          nid[lane] = (live && !at_centroid) ? id : 0u;
          __syncthreads();
          const int nb = (int)(m - b0 < 64 ? m - b0 : 64);
          eval_batch<kL2, float>(qlds, a.orows, a.orow_bytes, a.dp, nid, nd, nb);
          __syncthreads();
          d = nd[lane];
        } else if (live && !at_centroid) {
          double s = 0.0;
          for (uint32_t li = 0; li < a.N; li++) s = s + tab[li * 17 + lid[li]];
          d = (float)sqrt(s);
        }
        if (at_centroid) d = gd;
        const uint64_t key = live ? make_key(d, id) : ~0ull;
        // keys that can still enter the `size` smallest, in lane order
        uint64_t cand = ballot64(live && (nres < a.size || key < res[a.size - 1]));
        while (cand) {
          const int j = __ffsll((long long)cand) - 1;
          cand &= cand - 1;
          const uint64_t kj = __shfl(key, j, 64);
          if (nres < a.size || kj < res[a.size - 1]) res_insert(res, nres, a.size, kj);
        }
        __syncthreads();
      }
      count += m;
      if (count >= a.ass) break;
    }
    if (a.mode == kIvfRefine) {
      // exact distances of the kept results, sorted by (distance, id)
      for (uint32_t base = 0; base < nres; base += 64) {
        const uint32_t mm = nres - base < 64 ? nres - base : 64;
        if ((uint32_t)lane < mm) nid[lane] = key_id(res[base + lane]);
        __syncthreads();
        eval_batch<kL2, float>(qlds, a.orows, a.orow_bytes, a.dp, nid, nd, (int)mm);
        __syncthreads();
        uint64_t k2 = (uint32_t)lane < mm ? make_key(nd[lane], nid[lane]) : ~0ull;
        __syncthreads();
        if ((uint32_t)lane < mm) res[base + lane] = k2;
        __syncthreads();
      }
      // rank sort (ids are distinct)
      uint64_t mine[4];
      uint32_t pos[4];
      const uint32_t per = (nres + 63) / 64;
      for (uint32_t r = 0; r < per && r < 4; r++) {
        const uint32_t i = r * 64 + lane;
        mine[r] = i < nres ? res[i] : ~0ull;
        pos[r] = 0;
        if (i < nres)
          for (uint32_t j = 0; j < nres; j++) pos[r] += res[j] < mine[r] ? 1u : 0u;
      }
      __syncthreads();
      for (uint32_t r = 0; r < per && r < 4; r++)
        if (r * 64 + lane < nres) res[pos[r]] = mine[r];
      __syncthreads();
    }
    for (uint32_t i = lane; i < a.size; i += 64) {
      a.out_ids[(uint64_t)qi * a.size + i] = i < nres ? key_id(res[i]) : 0u;
      a.out_dists[(uint64_t)qi * a.size + i] = i < nres ? key_dist(res[i]) : 0.0f;
    }
    if (lane == 0) a.out_n[qi] = nres;
    __syncthreads();
  }
}

size_t ivf_search_lds_bytes(const IvfSearchArgs& a) {
  return (size_t)4 * a.dp + ((((size_t)8 * a.N * 17) + 15) & ~(size_t)15) +
         ((((size_t)8 * (a.size + 1)) + 15) & ~(size_t)15) + 8 * 64;
}

hipError_t launch_ivf_search(const IvfSearchArgs& a, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const size_t lds = ivf_search_lds_bytes(a);
  const uint32_t blocks = a.nq < 65536 ? a.nq : 65536;
  hipLaunchKernelGGL(ngt_ivf_search_kernel, dim3(blocks), dim3(64), lds, s, a);
  return hipGetLastError();
}

}  // namespace ngt_amd
