// prep_kernels.h -- query preparation (Index::allocateObject semantics).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ngt_amd {
// d_in: [nq][dim] float; d_out: [nq][dp] elements of the object type (float or
// uint8), zero padded; normalize: ObjectSpace::normalize for the normalized
// metrics.  Sets *error = 2 if a normalized query is the zero vector.
hipError_t launch_prepare_queries(const float* d_in, uint32_t dim, uint32_t nq, uint32_t dp, int otype,
                                  bool normalize, void* d_out, int* error, hipStream_t s);
// adj[v][0..stride) = edges[off[v]..off[v+1]) followed by zeros
hipError_t launch_pad_adjacency(const uint64_t* off, const uint32_t* edges, uint64_t nrows, uint64_t stride,
                                uint32_t* adj, hipStream_t s);
}  // namespace ngt_amd
