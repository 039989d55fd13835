// ngt_device.h -- CDNA4 (gfx950) device-side building blocks for the NGT
// distance hot path.  Everything here is wave64-native.
//
// Comparators: a row is evaluated by a *quad* of 4 consecutive lanes.  Lane g
// of the quad owns the reference's AVX-512 accumulator lanes 4g..4g+3, i.e. it
// streams the 16-byte column groups {16i + 4g .. 16i + 4g + 3} of the padded
// row (PrimitiveComparator.h:146-152).  The two quad shuffles then reproduce
// the 16 -> 8 -> 4 lane folds and the final (x0+x1)+(x2+x3), so the float
// result is bit-identical to the reference's compareL2 / compareCosine /
// compareDotProduct, and the L1 / uint8 variants follow their own folds
// (see oracle/ngt_oracle.c for the pinned restatement).  A wave therefore
// evaluates 16 candidate rows per step with fully independent 16-byte loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ngt_amd {

// NGT::ObjectSpace::DistanceType (lib/NGT/ObjectSpace.h:166-180)
enum Metric : int {
  kL1 = 0, kL2 = 1, kHamming = 2, kAngle = 3, kCosine = 4, kNormalizedAngle = 5,
  kNormalizedCosine = 6, kJaccard = 7, kSparseJaccard = 8, kNormalizedL2 = 9,
  kPoincare = 100, kLorentz = 101
};
// NGT::ObjectSpace::ObjectType (lib/NGT/ObjectSpace.h:182-186)
enum ObjType : int { kUint8 = 1, kFloat = 2 };

// ---------------------------------------------------------------------------
// (distance, id) keys.  ObjectDistance orders by distance, then id
// (lib/NGT/Common.h:1946-1959); mapping the float to an order-preserving
// uint32 and packing (dist << 32 | id) makes that a single u64 compare.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ord_of(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float float_of_ord(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}
__device__ __forceinline__ uint64_t make_key(float d, uint32_t id) {
  return ((uint64_t)ord_of(d) << 32) | id;
}
__device__ __forceinline__ float key_dist(uint64_t k) { return float_of_ord((uint32_t)(k >> 32)); }
__device__ __forceinline__ uint32_t key_id(uint64_t k) { return (uint32_t)k; }

// ---------------------------------------------------------------------------
// wave64 helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ float quad_xor(float v, int m) {
  // lanes within a quad: DPP-able swizzle, __shfl_xor lowers to ds_swizzle/dpp
  return __shfl_xor(v, m, 64);
}
__device__ __forceinline__ double quad_xor(double v, int m) { return __shfl_xor(v, m, 64); }
__device__ __forceinline__ uint32_t quad_xor(uint32_t v, int m) {
  return (uint32_t)__shfl_xor((int)v, m, 64);
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
  uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
// Wave-wide reductions without LDS traffic: DPP inside each 16-lane row
// (quad_perm lane^1 / lane^2, row_ror:4, row_ror:8 -- the last two turn quad
// results into row results), then gfx950 v_permlane16_swap / v_permlane32_swap
// across rows (odd rows trade with even rows, upper half with lower half), so
// every lane ends with the wave's result.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t x) {
  return ((uint64_t)dpp_u32<CTRL>((uint32_t)(x >> 32)) << 32) | dpp_u32<CTRL>((uint32_t)x);
}
__device__ __forceinline__ uint64_t min_u64(uint64_t a, uint64_t b) { return b < a ? b : a; }

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  v = min_u64(v, dpp_u64<0xb1>(v));   // quad_perm [1,0,3,2]
  v = min_u64(v, dpp_u64<0x4e>(v));   // quad_perm [2,3,0,1]
  v = min_u64(v, dpp_u64<0x124>(v));  // row_ror:4
  v = min_u64(v, dpp_u64<0x128>(v));  // row_ror:8
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  {
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    v = min_u64(((uint64_t)h[0] << 32) | l[0], ((uint64_t)h[1] << 32) | l[1]);
  }
  lo = (uint32_t)v;
  hi = (uint32_t)(v >> 32);
  {
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    v = min_u64(((uint64_t)h[0] << 32) | l[0], ((uint64_t)h[1] << 32) | l[1]);
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += dpp_u32<0xb1>(v);
  v += dpp_u32<0x4e>(v);
  v += dpp_u32<0x124>(v);
  v += dpp_u32<0x128>(v);
  {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = r[0] + r[1];
  }
  {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = r[0] + r[1];
  }
  return v;
}
__device__ __forceinline__ float wave_sum_f32(float f) {
  uint32_t v = __float_as_uint(f);
  v = __float_as_uint(__uint_as_float(v) + __uint_as_float(dpp_u32<0xb1>(v)));
  v = __float_as_uint(__uint_as_float(v) + __uint_as_float(dpp_u32<0x4e>(v)));
  v = __float_as_uint(__uint_as_float(v) + __uint_as_float(dpp_u32<0x124>(v)));
  v = __float_as_uint(__uint_as_float(v) + __uint_as_float(dpp_u32<0x128>(v)));
  {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = __float_as_uint(__uint_as_float(r[0]) + __uint_as_float(r[1]));
  }
  {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = __float_as_uint(__uint_as_float(r[0]) + __uint_as_float(r[1]));
  }
  return __uint_as_float(v);
}
__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t mbcnt(uint64_t mask) {
  // number of set bits in mask below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// ---------------------------------------------------------------------------
// Quad folds that restate the AVX-512 horizontal reductions.
// ---------------------------------------------------------------------------
// 16 accumulators spread as 4 per lane (lane g holds j = 4g+c).  Returns the
// float of PrimitiveComparator's (x0+x1)+(x2+x3) after 16->8->4 in every lane
// of the quad.
__device__ __forceinline__ float fold16(float4 a) {
  // t8[j] = acc[j+8] + acc[j]: partner lane g^2
  float4 o;
  o.x = quad_xor(a.x, 2); o.y = quad_xor(a.y, 2); o.z = quad_xor(a.z, 2); o.w = quad_xor(a.w, 2);
  a.x = o.x + a.x; a.y = o.y + a.y; a.z = o.z + a.z; a.w = o.w + a.w;
  // t4[j] = t8[j+4] + t8[j]: partner lane g^1
  o.x = quad_xor(a.x, 1); o.y = quad_xor(a.y, 1); o.z = quad_xor(a.z, 1); o.w = quad_xor(a.w, 1);
  a.x = o.x + a.x; a.y = o.y + a.y; a.z = o.z + a.z; a.w = o.w + a.w;
  return (a.x + a.y) + (a.z + a.w);
}
// Same folds, but the last four lanes are summed in double
// (compareDotProduct, PrimitiveComparator.h:473-476).
__device__ __forceinline__ double fold16_dot(float4 a) {
  float4 o;
  o.x = quad_xor(a.x, 2); o.y = quad_xor(a.y, 2); o.z = quad_xor(a.z, 2); o.w = quad_xor(a.w, 2);
  a.x = o.x + a.x; a.y = o.y + a.y; a.z = o.z + a.z; a.w = o.w + a.w;
  o.x = quad_xor(a.x, 1); o.y = quad_xor(a.y, 1); o.z = quad_xor(a.z, 1); o.w = quad_xor(a.w, 1);
  a.x = o.x + a.x; a.y = o.y + a.y; a.z = o.z + a.z; a.w = o.w + a.w;
  return ((double)a.x + (double)a.y) + ((double)a.z + (double)a.w);
}

__device__ __forceinline__ double angle_of(double c) {
  if (c >= 1.0) return 0.0;
  if (c <= -1.0) return acos(-1.0);
  return acos(c);
}

// ---------------------------------------------------------------------------
// float rows.  q: query (padded, in LDS), x: candidate row (global), dp: padded
// dimension (multiple of 16), g: lane within quad.  Every lane of the quad
// returns the same value.
// ---------------------------------------------------------------------------
template <int M>
__device__ __forceinline__ float dist_f32(const float* __restrict__ q,
                                          const float* __restrict__ x, int dp, int g) {
  const float4* xq = reinterpret_cast<const float4*>(x) + g;
  const float4* qq = reinterpret_cast<const float4*>(q) + g;
  const int nchunk = dp >> 4;
  if constexpr (M == kL2 || M == kPoincare) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int i = 0; i < nchunk; i++) {
      float4 xv = xq[4 * i];
      float4 qv = qq[4 * i];
      float vx = qv.x - xv.x, vy = qv.y - xv.y, vz = qv.z - xv.z, vw = qv.w - xv.w;
      acc.x = __builtin_fmaf(vx, vx, acc.x);
      acc.y = __builtin_fmaf(vy, vy, acc.y);
      acc.z = __builtin_fmaf(vz, vz, acc.z);
      acc.w = __builtin_fmaf(vw, vw, acc.w);
    }
    double l2 = sqrt((double)fold16(acc));
    if constexpr (M == kL2) {
      return (float)l2;
    } else {
      // comparePoincareDistance (PrimitiveComparator.h:608-618)
      double a2 = 0.0, b2 = 0.0;
      for (int i = 0; i < nchunk; i++) {
        float4 xv = xq[4 * i];
        float4 qv = qq[4 * i];
        a2 += (double)qv.x * qv.x + (double)qv.y * qv.y + (double)qv.z * qv.z + (double)qv.w * qv.w;
        b2 += (double)xv.x * xv.x + (double)xv.y * xv.y + (double)xv.z * xv.z + (double)xv.w * xv.w;
      }
      a2 += quad_xor(a2, 1); a2 += quad_xor(a2, 2);
      b2 += quad_xor(b2, 1); b2 += quad_xor(b2, 2);
      return (float)acosh(1 + 2.0 * l2 * l2 / (1.0 - a2) / (1.0 - b2));
    }
  } else if constexpr (M == kL1) {
    // compareL1 (PrimitiveComparator.h:269-289): 8 AVX lanes, lane j takes
    // column 8i + j.  Our lane g holds columns 16i+4g..+3 = AVX lanes
    // (4g..4g+3) mod 8, i.e. g and g^2 hold the same AVX lanes, split by
    // parity of the 8-column group -- the per-AVX-lane sum must be formed in
    // column order, so interleave the two partners' partial adds.
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int odd = g >> 1;  // this lane's groups are the odd 8-column halves
    for (int i = 0; i < nchunk; i++) {
      float4 xv = xq[4 * i];
      float4 qv = qq[4 * i];
      float4 v = make_float4(fabsf(qv.x - xv.x), fabsf(qv.y - xv.y), fabsf(qv.z - xv.z),
                             fabsf(qv.w - xv.w));
      // partner holds the other half of the same 16 columns
      float4 pv;
      pv.x = quad_xor(v.x, 2); pv.y = quad_xor(v.y, 2); pv.z = quad_xor(v.z, 2); pv.w = quad_xor(v.w, 2);
      float4 first = odd ? pv : v, second = odd ? v : pv;
      acc.x = (acc.x + first.x) + second.x;
      acc.y = (acc.y + first.y) + second.y;
      acc.z = (acc.z + first.z) + second.z;
      acc.w = (acc.w + first.w) + second.w;
    }
    // lanes g=0,1 now hold AVX lanes 0..7 (g=2,3 duplicates).
    float4 o;
    o.x = quad_xor(acc.x, 1); o.y = quad_xor(acc.y, 1); o.z = quad_xor(acc.z, 1); o.w = quad_xor(acc.w, 1);
    float4 lo = (g & 1) ? o : acc, hi = (g & 1) ? acc : o;  // lo = lanes 0..3, hi = 4..7
    float s = ((lo.x + lo.y) + (lo.z + lo.w)) + ((hi.x + hi.y) + (hi.z + hi.w));
    return (float)(double)s;
  } else if constexpr (M == kCosine || M == kAngle) {
    float4 na = make_float4(0.f, 0.f, 0.f, 0.f), nb = na, s = na;
#pragma unroll 4
    for (int i = 0; i < nchunk; i++) {
      float4 xv = xq[4 * i];
      float4 qv = qq[4 * i];
      na.x = __builtin_fmaf(qv.x, qv.x, na.x); na.y = __builtin_fmaf(qv.y, qv.y, na.y);
      na.z = __builtin_fmaf(qv.z, qv.z, na.z); na.w = __builtin_fmaf(qv.w, qv.w, na.w);
      nb.x = __builtin_fmaf(xv.x, xv.x, nb.x); nb.y = __builtin_fmaf(xv.y, xv.y, nb.y);
      nb.z = __builtin_fmaf(xv.z, xv.z, nb.z); nb.w = __builtin_fmaf(xv.w, xv.w, nb.w);
      s.x = __builtin_fmaf(xv.x, qv.x, s.x); s.y = __builtin_fmaf(xv.y, qv.y, s.y);
      s.z = __builtin_fmaf(xv.z, qv.z, s.z); s.w = __builtin_fmaf(xv.w, qv.w, s.w);
    }
    double dna = fold16(na), dnb = fold16(nb), ds = fold16(s);
    double c = ds / sqrt(dna * dnb);
    if constexpr (M == kCosine) return (float)(1.0 - c);
    else return (float)angle_of(c);
  } else if constexpr (M == kNormalizedAngle || M == kNormalizedCosine || M == kNormalizedL2) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int i = 0; i < nchunk; i++) {
      float4 xv = xq[4 * i];
      float4 qv = qq[4 * i];
      s.x = __builtin_fmaf(xv.x, qv.x, s.x); s.y = __builtin_fmaf(xv.y, qv.y, s.y);
      s.z = __builtin_fmaf(xv.z, qv.z, s.z); s.w = __builtin_fmaf(xv.w, qv.w, s.w);
    }
    double dot = fold16_dot(s);
    if constexpr (M == kNormalizedAngle) {
      return (float)angle_of(dot);
    } else if constexpr (M == kNormalizedCosine) {
      double v = 1.0 - dot;
      return (float)(v < 0.0 ? 0.0 : v);
    } else {
      double v = 2.0 - 2.0 * dot;
      return (float)(v < 0.0 ? 0.0 : sqrt(v));
    }
  } else if constexpr (M == kLorentz) {
    // compareLorentzDistance (PrimitiveComparator.h:630-637)
    double sum = 0.0;
    for (int i = 0; i < nchunk; i++) {
      float4 xv = xq[4 * i];
      float4 qv = qq[4 * i];
      double p0 = (double)qv.x * xv.x;
      if (i == 0 && g == 0) p0 = -p0;  // column 0 is added, the rest subtracted
      sum -= p0 + (double)qv.y * xv.y + (double)qv.z * xv.z + (double)qv.w * xv.w;
    }
    sum += quad_xor(sum, 1);
    sum += quad_xor(sum, 2);
    return (float)acosh(sum);
  } else if constexpr (M == kHamming || M == kJaccard) {
    // compareHammingDistance / compareJaccardDistance on the raw bytes
    const uint4* xb = reinterpret_cast<const uint4*>(x) + g;
    const uint4* qb = reinterpret_cast<const uint4*>(q) + g;
    uint32_t c = 0, de = 0;
    for (int i = 0; i < nchunk; i++) {
      uint4 xv = xb[4 * i], qv = qb[4 * i];
      if constexpr (M == kHamming) {
        c += __popc(xv.x ^ qv.x) + __popc(xv.y ^ qv.y) + __popc(xv.z ^ qv.z) + __popc(xv.w ^ qv.w);
      } else {
        c += __popc(xv.x & qv.x) + __popc(xv.y & qv.y) + __popc(xv.z & qv.z) + __popc(xv.w & qv.w);
        de += __popc(xv.x | qv.x) + __popc(xv.y | qv.y) + __popc(xv.z | qv.z) + __popc(xv.w | qv.w);
      }
    }
    c += quad_xor(c, 1); c += quad_xor(c, 2);
    if constexpr (M == kHamming) return (float)(double)c;
    de += quad_xor(de, 1); de += quad_xor(de, 2);
    return (float)(1.0 - (double)c / (double)de);
  } else if constexpr (M == kSparseJaccard) {
    // compareSparseJaccardDistance (PrimitiveComparator.h:399-418); a
    // sequential merge, evaluated by lane 0 of the quad.
    float r = 0.f;
    if (g == 0) {
      const uint32_t* ai = reinterpret_cast<const uint32_t*>(q);
      const uint32_t* bi = reinterpret_cast<const uint32_t*>(x);
      size_t loca = 0, locb = 0, count = 0, size = (size_t)dp;
      while (locb < size && ai[loca] != 0 && bi[loca] != 0) {
        int64_t sub = (int64_t)ai[loca] - (int64_t)bi[locb];
        count += sub == 0;
        loca += sub <= 0;
        locb += sub >= 0;
      }
      while (ai[loca] != 0) loca++;
      while (locb < size && bi[locb] != 0) locb++;
      const size_t den = loca + locb - count;
      // two empty lists: 1 - 0/0 is x86's default NaN, sign bit set (the
      // reference's bits; a GPU 0/0 would give the positive quiet NaN)
      r = den == 0 ? __uint_as_float(0xFFC00000u) : (float)(1.0 - (double)count / (double)den);
    }
    return __shfl(r, (lane_id() & ~3), 64);
  } else {
    return 0.f;
  }
}

// ---------------------------------------------------------------------------
// uint8 rows: lane g owns bytes 16i+4g..16i+4g+3.  The reference sums
// squares / absolute differences in 4 float lanes (lane c takes element
// e with e mod 4 == c); all partials are exact integers, so we accumulate
// integers per reference lane and rebuild the float folds.
// ---------------------------------------------------------------------------
template <int M>
__device__ __forceinline__ float dist_u8(const uint8_t* __restrict__ q,
                                         const uint8_t* __restrict__ x, int dp, int g) {
  const uint32_t* xw = reinterpret_cast<const uint32_t*>(x) + g;
  const uint32_t* qw = reinterpret_cast<const uint32_t*>(q) + g;
  const int nchunk = dp >> 4;
  if constexpr (M == kL2 || M == kL1 || M == kPoincare) {
    int acc[4] = {0, 0, 0, 0};
    for (int i = 0; i < nchunk; i++) {
      uint32_t xv = xw[4 * i], qv = qw[4 * i];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        int d = (int)((qv >> (8 * c)) & 0xff) - (int)((xv >> (8 * c)) & 0xff);
        acc[c] += (M == kL1) ? abs(d) : d * d;
      }
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
      acc[c] += (int)quad_xor((uint32_t)acc[c], 1);
      acc[c] += (int)quad_xor((uint32_t)acc[c], 2);
    }
    float f0 = (float)acc[0], f1 = (float)acc[1], f2 = (float)acc[2], f3 = (float)acc[3];
    double s = (double)((f0 + f1) + (f2 + f3));
    if constexpr (M == kL1) return (float)s;
    double l2 = sqrt(s);
    if constexpr (M == kL2) return (float)l2;
    double a2 = 0.0, b2 = 0.0;
    for (int i = 0; i < nchunk; i++) {
      uint32_t xv = xw[4 * i], qv = qw[4 * i];
      for (int c = 0; c < 4; c++) {
        double a = (double)((qv >> (8 * c)) & 0xff), b = (double)((xv >> (8 * c)) & 0xff);
        a2 += a * a;
        b2 += b * b;
      }
    }
    a2 += quad_xor(a2, 1); a2 += quad_xor(a2, 2);
    b2 += quad_xor(b2, 1); b2 += quad_xor(b2, 2);
    return (float)acosh(1 + 2.0 * l2 * l2 / (1.0 - a2) / (1.0 - b2));
  } else if constexpr (M == kHamming || M == kJaccard) {
    // popcount over the padded bytes (PrimitiveComparator.h:340-391)
    uint32_t c = 0, de = 0;
    for (int i = 0; i < nchunk; i++) {
      uint32_t xv = xw[4 * i], qv = qw[4 * i];
      if constexpr (M == kHamming) {
        c += __popc(xv ^ qv);
      } else {
        c += __popc(xv & qv);
        de += __popc(xv | qv);
      }
    }
    c += quad_xor(c, 1); c += quad_xor(c, 2);
    if constexpr (M == kHamming) return (float)(double)c;
    de += quad_xor(de, 1); de += quad_xor(de, 2);
    return (float)(1.0 - (double)c / (double)de);
  } else {
    // cosine / angle / dot-product family on uint8: exact integer sums in double
    uint32_t na = 0, nb = 0, s = 0;
    for (int i = 0; i < nchunk; i++) {
      uint32_t xv = xw[4 * i], qv = qw[4 * i];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        uint32_t a = (qv >> (8 * c)) & 0xff, b = (xv >> (8 * c)) & 0xff;
        na += a * a; nb += b * b; s += a * b;
      }
    }
    na += quad_xor(na, 1); na += quad_xor(na, 2);
    nb += quad_xor(nb, 1); nb += quad_xor(nb, 2);
    s += quad_xor(s, 1); s += quad_xor(s, 2);
    if constexpr (M == kCosine || M == kAngle) {
      double c = (double)s / sqrt((double)na * (double)nb);
      if constexpr (M == kCosine) return (float)(1.0 - c);
      else return (float)angle_of(c);
    } else if constexpr (M == kNormalizedAngle) {
      return (float)angle_of((double)s);
    } else if constexpr (M == kNormalizedCosine) {
      double v = 1.0 - (double)s;
      return (float)(v < 0.0 ? 0.0 : v);
    } else if constexpr (M == kNormalizedL2) {
      double v = 2.0 - 2.0 * (double)s;
      return (float)(v < 0.0 ? 0.0 : sqrt(v));
    } else if constexpr (M == kLorentz) {
      // sum = a0*b0 - sum_{i>=1} ai*bi, exact integers
      double a0b0 = (double)((q[0]) * (x[0]));
      return (float)acosh(a0b0 - ((double)s - a0b0));
    } else {
      return 0.f;
    }
  }
}

template <int M, typename T>
__device__ __forceinline__ float quad_distance(const T* __restrict__ q, const T* __restrict__ x,
                                               int dp, int g) {
  if constexpr (sizeof(T) == 4) return dist_f32<M>(q, x, dp, g);
  else return dist_u8<M>(q, x, dp, g);
}

}  // namespace ngt_amd
