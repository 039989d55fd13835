// filter_kernels.hip -- the 1-byte filter copy of an L2 float repository.
//
// A graph-search expansion evaluates every fresh neighbour, and in
// NeighborhoodGraph::searchReadOnlyGraph (lib/NGT/Graph.cpp:469-483) a
// neighbour farther than the exploration radius is only discarded.  The
// search kernel therefore first computes, from a 1-byte-per-element copy of
// the rows, a lower bound of each neighbour's distance, and fetches the f32
// row (and computes the comparator's exact distance) only for neighbours the
// bound cannot prove to be outside the radius.  Results, distances and
// distance counts stay identical to the reference; a rejected neighbour costs
// Dp bytes instead of 4*Dp.
//
// Copy: x~_i = a + b * c_i with one global (a, b) over all elements and
// c_i = clamp(rint((x_i - a) / b), 0, 255); per repository the largest
// reconstruction error E = max_x ||x - x~|| and the largest norm X = max ||x~||,
// both evaluated in double and rounded up.  Bound (search_common.h,
// filter_l2u8): ||q - x|| >= ||q - x~|| - E, and the float evaluation of
// ||q - x~|| is within 2^-16 (||q|| + X + sqrt(Dp)|a| + 1) of the real one.
// Rows with non-finite values disable the filter for the index.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ngt_device.h"
#include "ngt_kernels.h"

namespace ngt_amd {

// st[0] = ord(min), st[1] = ord(max), st[2] = non-finite flag,
// st[3] = E bits (float, >= 0), st[4] = X bits
__global__ void __launch_bounds__(256) ngt_filter_range_kernel(const uint8_t* rows, uint64_t row_bytes,
                                                               uint64_t nrows, uint32_t dp, uint32_t* st) {
  uint32_t lo = 0xffffffffu, hi = 0u, bad = 0u;
  const uint64_t total = (nrows - 1) * dp;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = 1 + t / dp, i = t % dp;
    const float x = reinterpret_cast<const float*>(rows + r * row_bytes)[i];
    if (!isfinite(x)) {
      bad = 1u;
      continue;
    }
    const uint32_t o = ord_of(x);
    lo = o < lo ? o : lo;
    hi = o > hi ? o : hi;
  }
  if (lo != 0xffffffffu) atomicMin(&st[0], lo);
  if (hi != 0u) atomicMax(&st[1], hi);
  if (bad) atomicOr(&st[2], 1u);
}

__device__ __forceinline__ void filter_ab(const uint32_t* st, float& a, float& b) {
  a = float_of_ord(st[0]);
  const float mx = float_of_ord(st[1]);
  if (st[0] == 0xffffffffu) {  // no finite element (empty repository)
    a = 0.0f;
    b = 0.0f;
    return;
  }
  b = (mx - a) / 255.0f;
}

// one thread per row: codes, reconstruction error, norm of the reconstruction
__global__ void __launch_bounds__(256) ngt_filter_encode_kernel(const uint8_t* rows, uint64_t row_bytes,
                                                                uint64_t nrows, uint32_t dp, uint64_t stride,
                                                                uint8_t* codes, uint32_t* st) {
  float a, b;
  filter_ab(st, a, b);
  float emax = 0.0f, xmax = 0.0f;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (uint64_t)gridDim.x * blockDim.x) {
    const float* x = reinterpret_cast<const float*>(rows + r * row_bytes);
    uint32_t* out = reinterpret_cast<uint32_t*>(codes + r * stride);
    double e2 = 0.0, n2 = 0.0;
    for (uint32_t i0 = 0; i0 < dp; i0 += 4) {
      uint32_t w = 0;
      for (uint32_t j = 0; j < 4; j++) {
        const float v = x[i0 + j];
        float c = 0.0f;
        if (b > 0.0f && r > 0) {
          c = rintf((v - a) / b);
          c = c < 0.0f ? 0.0f : (c > 255.0f ? 255.0f : c);
        }
        w |= (uint32_t)c << (8 * j);
        const double rec = (double)a + (double)b * (double)c;
        const double d = (double)v - rec;
        e2 += d * d;
        n2 += rec * rec;
      }
      out[i0 >> 2] = w;
    }
    if (r == 0) continue;  // the dummy slot is never a neighbour
    // round up: the float of a double is within 2^-24 relative
    const float e = (float)(sqrt(e2) * (1.0 + 1e-6)) * 1.0000002f;
    const float n = (float)(sqrt(n2) * (1.0 + 1e-6)) * 1.0000002f;
    emax = e > emax ? e : emax;
    xmax = n > xmax ? n : xmax;
  }
  if (emax > 0.0f) atomicMax(&st[3], __float_as_uint(emax));
  if (xmax > 0.0f) atomicMax(&st[4], __float_as_uint(xmax));
}

// params: {a, b, E, X, valid}
__global__ void ngt_filter_finalize_kernel(const uint32_t* st, float* params) {
  if (threadIdx.x != 0) return;
  float a, b;
  filter_ab(st, a, b);
  params[0] = a;
  params[1] = b;
  params[2] = __uint_as_float(st[3]);
  params[3] = __uint_as_float(st[4]);
  params[4] = st[2] ? 0.0f : 1.0f;
}

hipError_t launch_filter_build(const uint8_t* rows, uint64_t row_bytes, uint64_t nrows, uint32_t dp, uint64_t stride,
                               uint8_t* codes, uint32_t* st, float* params, hipStream_t s) {
  hipError_t e = hipMemsetAsync(st, 0xff, sizeof(uint32_t), s);
  if (e == hipSuccess) e = hipMemsetAsync(st + 1, 0, 4 * sizeof(uint32_t), s);
  if (e != hipSuccess) return e;
  if (nrows > 1) {
    hipLaunchKernelGGL(ngt_filter_range_kernel, dim3(4096), dim3(256), 0, s, rows, row_bytes, nrows, dp, st);
    uint64_t blocks = (nrows + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(ngt_filter_encode_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, rows, row_bytes, nrows, dp,
                       stride, codes, st);
  }
  hipLaunchKernelGGL(ngt_filter_finalize_kernel, dim3(1), dim3(64), 0, s, st, params);
  return hipGetLastError();
}

}  // namespace ngt_amd
