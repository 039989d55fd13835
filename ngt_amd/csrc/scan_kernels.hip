// scan_kernels.hip -- the exact scan of ObjectSpaceRepository::linearSearch
// (lib/NGT/ObjectSpaceRepository.h:466-502) for float L2, tiled for CDNA4.
//
// The reference computes every (query, object) distance with compareL2's 16
// AVX-512 accumulator lanes (PrimitiveComparator.h:143-198): lane l sums
// fma((q-x)^2) over dims l, l+16, l+32, ... in order, then the lanes fold
// 16 -> 8 -> 4 and (x0+x1)+(x2+x3), and sqrt runs in double.  Here a group of
// 16 GPU lanes plays those 16 accumulator lanes, and each GPU lane carries
// them for 16 (query, object) pairs at once:
//
//   * queries stay in VGPRs: group g of a 256-thread workgroup owns 8
//     queries; its lane j holds dims j + 16m of each (8 x Dp/16 floats);
//   * objects stream through LDS two rows at a time, stored as float2
//     {row a, row b} per dim, so one ds_read_b64 feeds a packed
//     v_pk_add_f32 / v_pk_fma_f32 for the pairs (q, a) and (q, b): the FMA
//     chain of each pair is the reference's, lane for lane;
//   * the 16 accumulator lanes fold with a reduce-scatter in the reference's
//     order (DPP row_ror:8, xor 4, quad_perm xor 1, then xor 2): every lane
//     ends with the full sum of one of the group's 16 pairs.  Lanes 8..15 see
//     the two rows swapped and every lane j holds its query slots permuted by
//     j & 7, so at each stage the kept / sent registers are the same for all
//     lanes and no select is needed;
//   * each query keeps its k best (distance, id) keys in LDS; a distance is a
//     candidate only when it beats the current k-th key (rare after the first
//     rows), inserted by the whole wave.
//
// One workgroup = 128 queries x one contiguous part of the rows; the parts'
// lists merge in ngt_linear_merge_kernel.  Distances are bit-identical to the
// comparator's, so ids and distances equal the quad-per-row kernel's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ngt_device.h"
#include "ngt_kernels.h"
#include "search_common.h"

namespace ngt_amd {

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kScanQ = 8;        // queries per 16-lane group
constexpr int kScanGroups = 16;  // groups per 256-thread workgroup
constexpr int kScanQB = kScanQ * kScanGroups;  // 128 queries per workgroup
constexpr int kScanPairs = 4;    // row pairs per LDS stage (8 rows)

// Fold steps as single DPP adds (update_dpp with a zero `old` and bound_ctrl
// lets the compiler fold the swizzle into v_add_f32_dpp).  keep + lane (j^8)
// of the 16-lane row:
__device__ __forceinline__ float add_xor8(float keep, float send) {
  return keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x128, 0xf, 0xf, true));
}
// keep + lane j^4: lanes with bit 2 clear take lane j+4 (row_shl:4), the
// others lane j-4 (row_shr:4); both sums are formed, one is selected
__device__ __forceinline__ float add_xor4(float keep, float send, bool up) {
  const float fwd = keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x104, 0xf, 0xf, true));
  const float bwd = keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x114, 0xf, 0xf, true));
  return up ? bwd : fwd;
}
__device__ __forceinline__ float add_xor1(float keep, float send) {  // quad_perm [1,0,3,2]
  return keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0xb1, 0xf, 0xf, true));
}
__device__ __forceinline__ float add_xor2(float keep, float send) {  // quad_perm [2,3,0,1]
  return keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x4e, 0xf, 0xf, true));
}

template <int NCH>
__global__ void __launch_bounds__(256) ngt_linear_scan_l2f_kernel(LinearArgs a, uint32_t rows_per_part) {
  constexpr int DP = 16 * NCH;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t k = a.k;
  uint64_t* lists = reinterpret_cast<uint64_t*>(smem);              // [128][k]
  uint64_t* thr = lists + (size_t)kScanQB * k;                        // [128] k-th key (or ~0)
  uint32_t* cnt = reinterpret_cast<uint32_t*>(thr + kScanQB);         // [128]
  // [128] upper bound of the squared sum a candidate may have: a sum above
  // it cannot round to a distance <= the k-th key's (or the radius)
  float* thr_s = reinterpret_cast<float*>(cnt + kScanQB);
  uint8_t* vflag = reinterpret_cast<uint8_t*>(thr_s + kScanQB);     // [2][8] row valid flags
  // row stages: [2 buffers][2 orders][kScanPairs][NCH][16] float2
  f2* stage = reinterpret_cast<f2*>(vflag + 16);
  constexpr int kStage = 2 * kScanPairs * NCH * 16;                   // float2 per buffer

  const int tid = threadIdx.x;
  const int g = tid >> 4, j = tid & 15, lane = tid & 63;
  const uint32_t qb = blockIdx.x * kScanQB;
  const uint32_t part = blockIdx.y;
  uint64_t r0 = (uint64_t)part * rows_per_part, r1 = r0 + rows_per_part;
  if (r0 < 1) r0 = 1;
  if (r1 > a.nrows) r1 = a.nrows;

  // queries: slot s of lane j holds query qb + 8g + (s ^ (j & 7)), dims j + 16m
  float qv[kScanQ][NCH];
#pragma unroll
  for (int s = 0; s < kScanQ; s++) {
    const uint32_t qi = qb + 8 * g + (s ^ (j & 7));
    const float* qp = reinterpret_cast<const float*>(a.queries + (uint64_t)(qi < a.nq ? qi : 0) * a.query_bytes);
#pragma unroll
    for (int m = 0; m < NCH; m++) qv[s][m] = qi < a.nq ? qp[16 * m + j] : 0.0f;
  }
  // squared-sum bound of a distance d: any sum whose (float)sqrt((double)sum)
  // is <= d is below (nextafter(d))^2, rounded up once more
  auto sq_bound = [](float d) {
    if (!(d >= 0.0f) || d >= 3.0e38f) return __builtin_huge_valf();  // NaN, inf: no bound
    const double dn = (double)__uint_as_float(__float_as_uint(d) + 1u);  // next float up
    const float s2 = (float)(dn * dn);
    return __uint_as_float(__float_as_uint(s2) + 1u);
  };
  const float rad_s = a.radius < 0.0 || a.radius >= 3.0e38 ? __builtin_huge_valf() : sq_bound((float)a.radius);
  for (uint32_t i = tid; i < (uint32_t)kScanQB; i += 256) {
    cnt[i] = 0;
    thr[i] = ~0ull;
    thr_s[i] = rad_s;
  }

  // this thread's share of one stage: 8 rows x DP floats as float4
  constexpr int kF4 = 2 * kScanPairs * DP / 4;
  constexpr int kPer = (kF4 + 255) / 256;
  float4 pre[kPer];
  uint32_t pre_valid = 0;  // threads 0..7: valid flag of row row0 + tid
  auto fetch = [&](uint64_t row0) {
    if (tid < 2 * kScanPairs) {
      const uint64_t id = row0 + tid;
      pre_valid = id < r1 && (a.valid == nullptr || a.valid[id]) ? 1u : 0u;
    }
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const int f = tid + 256 * u;
      pre[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (f < kF4) {
        const int r = f / (DP / 4), c = f - r * (DP / 4);
        const uint64_t id = row0 + r;
        if (id < r1) pre[u] = reinterpret_cast<const float4*>(a.rows + id * a.row_bytes)[c];
      }
    }
  };
  auto store = [&](f2* buf, int bi) {
    if (tid < 2 * kScanPairs) vflag[bi * 8 + tid] = (uint8_t)pre_valid;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const int f = tid + 256 * u;
      if (f < kF4) {
        const int r = f / (DP / 4), c = f - r * (DP / 4);
        const int p = r >> 1, side = r & 1;
        float* nrm = reinterpret_cast<float*>(buf);                  // {a, b}
        float* swp = reinterpret_cast<float*>(buf + kScanPairs * NCH * 16);  // {b, a}
        const float v[4] = {pre[u].x, pre[u].y, pre[u].z, pre[u].w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int d = 4 * c + e, m = d >> 4, jj = d & 15;
          const int at = ((p * NCH + m) * 16 + jj) * 2;
          nrm[at + side] = v[e];
          swp[at + (side ^ 1)] = v[e];
        }
      }
    }
  };

  const bool hi8 = j >= 8;
  fetch(r0);
  int buf = 0;
  for (uint64_t t0 = r0; t0 < r1; t0 += 2 * kScanPairs, buf ^= 1) {
    f2* cur = stage + buf * kStage;
    store(cur, buf);
    __syncthreads();
    if (t0 + 2 * kScanPairs < r1) fetch(t0 + 2 * kScanPairs);
    const f2* src = cur + (hi8 ? kScanPairs * NCH * 16 : 0);
    const uint64_t vf = *reinterpret_cast<const uint64_t*>(vflag + buf * 8);  // byte r = row r valid
    const uint32_t ql = 8 * g + (j & 7);
    const bool up4 = (j & 4) != 0;
#pragma unroll
    for (int p = 0; p < kScanPairs; p += 2) {
      // two row pairs: their FMA chains and folds interleave (independent
      // work between each DPP and its producer)
      f2 acc[2][kScanQ];
#pragma unroll
      for (int h = 0; h < 2; h++)
#pragma unroll
        for (int s = 0; s < kScanQ; s++) acc[h][s] = (f2){0.f, 0.f};
#pragma unroll
      for (int m = 0; m < NCH; m++) {
        const f2 x0 = src[(p * NCH + m) * 16 + j];
        const f2 x1 = src[((p + 1) * NCH + m) * 16 + j];
        // all differences first, then the FMAs: a packed-f32 result read by
        // the very next instruction costs a wait state (s_nop) on gfx950
        f2 d[2][kScanQ];
#pragma unroll
        for (int s = 0; s < kScanQ; s++) {
          d[0][s] = (f2){qv[s][m], qv[s][m]} - x0;
          d[1][s] = (f2){qv[s][m], qv[s][m]} - x1;
        }
#pragma unroll
        for (int s = 0; s < kScanQ; s++) {
          acc[0][s] = __builtin_elementwise_fma(d[0][s], d[0][s], acc[0][s]);
          acc[1][s] = __builtin_elementwise_fma(d[1][s], d[1][s], acc[1][s]);
        }
      }
      const float ts = thr_s[ql];
      // reduce-scatter in the reference's fold order
      float v[2][kScanQ];
#pragma unroll
      for (int s = 0; s < kScanQ; s++)
#pragma unroll
        for (int h = 0; h < 2; h++) v[h][s] = add_xor8(acc[h][s].x, acc[h][s].y);  // 16 -> 8
#pragma unroll
      for (int s = 0; s < 4; s++)
#pragma unroll
        for (int h = 0; h < 2; h++) v[h][s] = add_xor4(v[h][s], v[h][s + 4], up4);  // 8 -> 4
      float sums[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        v[h][0] = add_xor1(v[h][0], v[h][1]);  // x0 + x1
        v[h][2] = add_xor1(v[h][2], v[h][3]);  // x2 + x3
      }
#pragma unroll
      for (int h = 0; h < 2; h++) sums[h] = add_xor2(v[h][0], v[h][2]);
#pragma unroll
      for (int h = 0; h < 2; h++) {
      const float sum = sums[h];
      // lane j: query qb + 8g + (j & 7), row t0 + 2(p + h) + (j >= 8)
      const int rl = 2 * (p + h) + (hi8 ? 1 : 0);
      const uint64_t id = t0 + rl;
      uint64_t key = ~0ull;
      if (((vf >> (8 * rl)) & 1u) && sum <= ts) {
        // rare: the exact distance (compareL2's double sqrt) and key
        const float dist = (float)sqrt((double)sum);
        if (a.radius < 0.0 || (double)dist <= a.radius) key = make_key(dist, (uint32_t)id);
        if (key >= thr[ql]) key = ~0ull;
      }
      uint64_t cand = ballot64(key != ~0ull);
      while (cand) {
        const int l = __ffsll((long long)cand) - 1;
        cand &= cand - 1;
        const uint32_t q = (uint32_t)__shfl((int)ql, l, 64);
        const uint64_t kk = ((uint64_t)(uint32_t)__shfl((int)(key >> 32), l, 64) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)key, l, 64);
        uint32_t n = cnt[q];
        res_insert(lists + (size_t)q * k, n, k, kk);
        if (lane == 0) {
          cnt[q] = n;
          if (n >= k) {
            const uint64_t kth = lists[(size_t)q * k + k - 1];
            thr[q] = kth;
            thr_s[q] = fminf(rad_s, sq_bound(key_dist(kth)));
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      }
    }
  }
  __syncthreads();
  // this part's k best of each query
  for (uint32_t i = tid; i < (uint32_t)kScanQB * k; i += 256) {
    const uint32_t ql = i / k, r = i - ql * k;
    const uint32_t qi = qb + ql;
    if (qi < a.nq) a.partial[((uint64_t)qi * gridDim.y + part) * k + r] = r < cnt[ql] ? lists[i] : ~0ull;
  }
}

size_t linear_scan_lds_bytes(uint32_t k, int dp) {
  const int nch = dp / 16;
  return (size_t)kScanQB * k * 8 + kScanQB * 8 + kScanQB * 4 + kScanQB * 4 + 16 * 4 +
         (size_t)2 * 2 * kScanPairs * nch * 16 * 8;
}

hipError_t launch_linear_scan(const LinearArgs& a, int metric, int otype, uint32_t nparts, uint32_t rows_per_part,
                              hipStream_t s) {
  if (metric != kL2 || otype != kFloat || a.k > 32 || a.dp > 256 || (a.dp & 15)) return hipErrorNotSupported;
  const size_t lds = linear_scan_lds_bytes(a.k, a.dp);
  const dim3 grid((a.nq + kScanQB - 1) / kScanQB, nparts);
#define L_SCAN(N)                                                                                  \
  case N:                                                                                          \
    hipLaunchKernelGGL((ngt_linear_scan_l2f_kernel<N>), grid, dim3(256), lds, s, a, rows_per_part); \
    break;
  switch (a.dp / 16) {
    L_SCAN(1) L_SCAN(2) L_SCAN(3) L_SCAN(4) L_SCAN(5) L_SCAN(6) L_SCAN(7) L_SCAN(8)
    L_SCAN(9) L_SCAN(10) L_SCAN(11) L_SCAN(12) L_SCAN(13) L_SCAN(14) L_SCAN(15) L_SCAN(16)
    default: return hipErrorNotSupported;
  }
#undef L_SCAN
  return hipGetLastError();
}

}  // namespace ngt_amd
