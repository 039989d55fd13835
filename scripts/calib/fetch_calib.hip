// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE against known byte
// counts for the access patterns of the search kernels (MI355X_MICROARCH.md:
// FETCH_SIZE is exact only for 16-B/lane streaming reads; other widths are
// uncalibrated).  Each kernel reads R distinct random rows of a 2 GiB table
// (beyond the 256 MiB Infinity Cache) exactly once, in the search kernels'
// own load shapes:
//   filter : 128-B code rows, a quad of lanes per row, 4 x 8-B loads per lane
//            (search_common.h filter_l2u8)
//   exact  : 512-B f32 rows, a quad per row, 8 x 16-B loads per lane
//            (ngt_device.h eval_l2f_fast / l2_fold_rows)
//   probe  : one 4-B load per random id (the visited-epoch probe)
//   adj    : 192-B padded adjacency rows, 48 lanes x 4 B (load_adj_row)
//   stream : contiguous 16 B per lane (the guide's calibrated case)
// Prints the bytes each kernel reads; the rocprofv3 pass gives FETCH_SIZE.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void k_filter(const uint8_t* t, const uint32_t* ids, uint32_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, g = lane & 3;
  uint32_t acc = 0;
  for (uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> 2; r < n; r += (gridDim.x * blockDim.x) >> 2) {
    const uint2* p = reinterpret_cast<const uint2*>(t + (uint64_t)ids[r] * 128) + g * 4;
#pragma unroll
    for (int w = 0; w < 4; w++) {
      const uint2 v = p[w];
      acc += v.x ^ v.y;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_exact(const uint8_t* t, const uint32_t* ids, uint32_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, g = lane & 3;
  float acc = 0.f;
  for (uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> 2; r < n; r += (gridDim.x * blockDim.x) >> 2) {
    const float4* p = reinterpret_cast<const float4*>(t + (uint64_t)ids[r] * 512) + g;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const float4 v = p[4 * i];
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 1234.5f) out[0] = 1;
}

__global__ void k_probe(const uint8_t* t, const uint32_t* ids, uint32_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x)
    acc += *reinterpret_cast<const uint32_t*>(t + (uint64_t)ids[r] * 128);
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_adj(const uint8_t* t, const uint32_t* ids, uint32_t n, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += (gridDim.x * blockDim.x) >> 6)
    if (lane < 48) acc += reinterpret_cast<const uint32_t*>(t + (uint64_t)ids[r] * 192)[lane];
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_stream(const uint8_t* t, uint64_t bytes, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) * 16; i < bytes; i += (uint64_t)gridDim.x * blockDim.x * 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(t + i);
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t table = 2ull << 30;
  uint8_t* t;
  uint32_t *ids, *out;
  CHECK(hipMalloc(&t, table));
  CHECK(hipMemset(t, 1, table));
  CHECK(hipMalloc(&out, 4));
  const uint32_t R = 1u << 20;  // rows read by each gather kernel
  CHECK(hipMalloc(&ids, 4ull * R));
  auto upload_perm = [&](uint64_t rows) {
    // R distinct random rows of `rows` (a strided permutation)
    std::vector<uint32_t> h(R);
    const uint64_t step = 2654435761ull % rows;
    for (uint32_t i = 0; i < R; i++) h[i] = (uint32_t)(((uint64_t)i * step + 12345) % rows);
    CHECK(hipMemcpy(ids, h.data(), 4ull * R, hipMemcpyHostToDevice));
  };
  const dim3 grid(1024), block(256);
  upload_perm(table / 128);
  hipLaunchKernelGGL(k_filter, grid, block, 0, 0, t, ids, R, out);
  CHECK(hipDeviceSynchronize());
  printf("k_filter reads %llu bytes of rows (+%llu of ids)\n", (unsigned long long)R * 128, 4ull * R);
  upload_perm(table / 512);
  hipLaunchKernelGGL(k_exact, grid, block, 0, 0, t, ids, R, out);
  CHECK(hipDeviceSynchronize());
  printf("k_exact reads %llu bytes of rows (+%llu of ids)\n", (unsigned long long)R * 512, 4ull * R);
  upload_perm(table / 128);
  hipLaunchKernelGGL(k_probe, grid, block, 0, 0, t, ids, R, out);
  CHECK(hipDeviceSynchronize());
  printf("k_probe reads %llu bytes used (+%llu of ids), one line each\n", 4ull * R, 4ull * R);
  upload_perm(table / 192);
  hipLaunchKernelGGL(k_adj, grid, block, 0, 0, t, ids, R, out);
  CHECK(hipDeviceSynchronize());
  printf("k_adj reads %llu bytes of rows (+%llu of ids)\n", 192ull * R, 4ull * R);
  hipLaunchKernelGGL(k_stream, grid, block, 0, 0, t, table / 4, out);
  CHECK(hipDeviceSynchronize());
  printf("k_stream reads %llu bytes\n", (unsigned long long)(table / 4));
  return 0;
}
