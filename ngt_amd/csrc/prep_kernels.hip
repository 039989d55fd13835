// prep_kernels.hip -- Index::allocateObject on the device: convert the caller's
// query to the object type, zero-pad to the padded dimension
// (ObjectRepository::allocateObject, lib/NGT/ObjectRepository.h:222-253) and
// normalize for the normalized metrics (ObjectSpace::normalize,
// lib/NGT/ObjectSpace.h:251-266).
//
// The squared norm is accumulated like the reference's AVX-512 build (16
// FMA lanes over the unpadded dimension, sequential FMA tail); the reference
// then finishes with `vrsqrtss` + one Newton step, whose bits depend on the
// host CPU model, so this kernel uses the source's sqrt + divide instead and
// normalized-metric queries are matched within tolerance, not bit for bit.
#include <hip/hip_runtime.h>

#include "ngt_device.h"
#include "prep_kernels.h"

namespace ngt_amd {

__global__ void __launch_bounds__(64) prep_kernel(const float* __restrict__ in, uint32_t dim, uint32_t nq,
                                                  uint32_t dp, int otype, int normalize, uint8_t* out,
                                                  int* error) {
  const int lane = threadIdx.x;
  for (uint32_t q = blockIdx.x; q < nq; q += gridDim.x) {
    const float* src = in + (uint64_t)q * dim;
    float scale = 1.0f;
    bool div = false;
    if (normalize && otype == kFloat) {
      // lanes 0..15 hold the 16 AVX-512 accumulators
      float acc = 0.f;
      const uint32_t main = dim & ~15u;
      if (lane < 16)
        for (uint32_t i = lane; i < main; i += 16) acc = __builtin_fmaf(src[i], src[i], acc);
      // 16 -> 8 -> 4 -> (x0+x2)+(x1+x3)
      float o = __shfl_xor(acc, 8, 64);
      acc = o + acc;
      o = __shfl_xor(acc, 4, 64);
      acc = o + acc;
      o = __shfl_xor(acc, 2, 64);
      acc = o + acc;
      o = __shfl_xor(acc, 1, 64);
      float sum = o + acc;
      sum = __shfl(sum, 0, 64);
      for (uint32_t i = main; i < dim; i++) sum = __builtin_fmaf(src[i], src[i], sum);
      if (sum == 0.0f) {
        if (lane == 0) atomicOr(error, 2);
      } else {
        scale = sqrtf(sum);
        div = true;
      }
    }
    if (otype == kFloat) {
      float* dst = reinterpret_cast<float*>(out) + (uint64_t)q * dp;
      for (uint32_t i = lane; i < dp; i += 64) dst[i] = i < dim ? (div ? src[i] / scale : src[i]) : 0.f;
    } else {
      uint8_t* dst = out + (uint64_t)q * dp;
      for (uint32_t i = lane; i < dp; i += 64) {
        // static_cast<uint8_t>(value): truncate to int, keep the low byte
        uint8_t v = 0;
        if (i < dim) {
          float x = src[i];
          int iv = (x != x || x >= 2147483648.0f || x < -2147483648.0f) ? (int)0x80000000 : (int)x;
          v = (uint8_t)iv;
        }
        dst[i] = v;
      }
    }
  }
}

hipError_t launch_prepare_queries(const float* d_in, uint32_t dim, uint32_t nq, uint32_t dp, int otype,
                                  bool normalize, void* d_out, int* error, hipStream_t s) {
  uint32_t blocks = nq < 65535 ? nq : 65535;
  hipLaunchKernelGGL(prep_kernel, dim3(blocks), dim3(64), 0, s, d_in, dim, nq, dp, otype, normalize ? 1 : 0,
                     static_cast<uint8_t*>(d_out), error);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) pad_adjacency_kernel(const uint64_t* off, const uint32_t* edges,
                                                            uint64_t nrows, uint64_t stride, uint32_t* adj) {
  const uint64_t total = nrows * stride;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t v = i / stride, e = i - v * stride;
    const uint64_t b = off[v], n = off[v + 1] - b;
    adj[i] = e < n ? edges[b + e] : 0u;
  }
}

hipError_t launch_pad_adjacency(const uint64_t* off, const uint32_t* edges, uint64_t nrows, uint64_t stride,
                                uint32_t* adj, hipStream_t s) {
  hipLaunchKernelGGL(pad_adjacency_kernel, dim3(8192), dim3(256), 0, s, off, edges, nrows, stride, adj);
  return hipGetLastError();
}

}  // namespace ngt_amd
