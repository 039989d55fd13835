// shard_api.cpp -- the object repository sharded over the GPUs of a node
// (BASELINE configs C4/C5) as C entry points, for C/C++
// callers that run one process (or thread) per GPU without torch.distributed.
//
// Rank r holds shard r as its own ngt_amd_index (objects with global ids
// id_offsets[r] + 1 .. ); every rank searches the whole batch on its shard
// (the exact search of NeighborhoodGraph::searchReadOnlyGraph, Graph.cpp:398-495,
// or NGTQG::Index::search, QuantizedGraph.h:354-372), packs each result list
// into k words (distance bits << 32 | local id, the NGT::ObjectDistance order
// of Common.h:1937-1992), exchanges them with ONE RCCL all-gather over xGMI
// (nq * k * 8 B per rank) and merges the gathered lists on its device: every
// rank ends with the k best by (distance, global id).  The communicator is
// RCCL's; one call at a time per communicator (like an ncclComm_t).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include "index_internal.h"
#include "ngt_kernels.h"

using namespace ngt_amd;

struct ngt_amd_shard_comm {
  ncclComm_t comm = nullptr;
  int device = 0, rank = 0, world = 1;
  DevBuf<uint32_t> ids, n, off;
  DevBuf<float> dists;
  DevBuf<uint64_t> packed, gathered;
  DevBuf<int> err;         // OR of every shard's device error flag since the last synchronize
  bool have_offsets = false;
};

#define NCCL_OK(expr)                                                                       \
  do {                                                                                      \
    ncclResult_t r_ = (expr);                                                               \
    if (r_ != ncclSuccess) return fail("%s failed: %s", #expr, ncclGetErrorString(r_));    \
  } while (0)

extern "C" int ngt_amd_shard_unique_id(uint8_t* id, uint64_t id_bytes) {
  if (!id || id_bytes < sizeof(ncclUniqueId)) return fail("ngt_amd_shard_unique_id: need %zu bytes", sizeof(ncclUniqueId));
  ncclUniqueId u;
  NCCL_OK(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof(u));
  return 0;
}

extern "C" int ngt_amd_shard_comm_create(ngt_amd_shard_comm** out, int device, int rank, int world,
                                         const uint8_t* id, uint64_t id_bytes) {
  if (!out || !id || id_bytes < sizeof(ncclUniqueId) || world < 1 || rank < 0 || rank >= world)
    return fail("ngt_amd_shard_comm_create: bad arguments");
  HIP_OK(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  auto* c = new ngt_amd_shard_comm();
  c->device = device;
  c->rank = rank;
  c->world = world;
  // the error word is zeroed on a stream of its own and only that stream is
  // waited for: a device-wide synchronize would also wait for a resident
  // serving grid (serve.cpp), which leaves only after its idle time
  hipStream_t zs = nullptr;
  bool ok = c->err.alloc(1) == hipSuccess && hipStreamCreateWithFlags(&zs, hipStreamNonBlocking) == hipSuccess &&
            hipMemsetAsync(c->err.p, 0, sizeof(int), zs) == hipSuccess && hipStreamSynchronize(zs) == hipSuccess;
  if (zs) (void)hipStreamDestroy(zs);
  if (!ok) {
    delete c;
    return fail("ngt_amd_shard_comm_create: allocation failed");
  }
  ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail("ncclCommInitRank failed: %s", ncclGetErrorString(r));
  }
  *out = c;
  return 0;
}

extern "C" int ngt_amd_shard_comm_destroy(ngt_amd_shard_comm* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
  return 0;
}

// pack -> all-gather -> merge of this rank's [nq][k] lists (already searched
// on stream s with launch context `ctx`).  Every rank's message carries one
// trailer word after its nq*k result words: that shard's device error flag
// (unchecked-set spill overflow), taken from its launch context and cleared
// there, so a truncated shard list is reported on EVERY rank -- the merge ORs
// the trailers into c->err.  With id_offsets == NULL (offsets stored by
// ngt_amd_shard_comm_set_offsets) nothing here waits for the device: the
// all-gather of one batch overlaps the next batch's search, and
// ngt_amd_shard_comm_synchronize reports the flags.  With a host id_offsets
// array (the original form) the call copies it, synchronizes and reports.
static int exchange_and_merge(ngt_amd_shard_comm* c, ngt_amd_index* ix, uint32_t nq, uint32_t k,
                              const uint32_t* id_offsets, uint32_t* d_out_ids, float* d_out_dists,
                              uint32_t* d_out_n, hipStream_t s) {
  if ((uint64_t)c->world * k * sizeof(uint64_t) > 64 * 1024)
    return fail("sharded search: %d shards x k=%u exceed one workgroup's LDS in the merge", c->world, k);
  if (!id_offsets && !c->have_offsets)
    return fail("sharded search: no id offsets (pass them, or set them once with ngt_amd_shard_comm_set_offsets)");
  SearchCtx* ctx = ctx_for(ix, s);
  if (!ctx) return -1;
  const uint64_t words = (uint64_t)nq * k, stride = words + 1;
  HIP_OK(c->packed.alloc(stride));
  HIP_OK(c->gathered.alloc(stride * c->world));
  HIP_OK(launch_pack_results(c->ids.p, c->dists.p, c->n.p, nq, k, c->packed.p, s));
  HIP_OK(hipMemsetAsync(c->packed.p + words, 0, sizeof(uint64_t), s));
  HIP_OK(hipMemcpyAsync(c->packed.p + words, ctx->err.p, sizeof(int), hipMemcpyDeviceToDevice, s));
  HIP_OK(hipMemsetAsync(ctx->err.p, 0, sizeof(int), s));
  NCCL_OK(ncclAllGather(c->packed.p, c->gathered.p, stride, ncclUint64, c->comm, s));
  if (id_offsets) {
    HIP_OK(c->off.alloc(c->world));
    HIP_OK(hipMemcpyAsync(c->off.p, id_offsets, c->world * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    c->have_offsets = false;  // the caller's array, not a stored set
  }
  MergeArgs a{};
  a.id_offsets = c->off.p;
  a.nparts = (uint32_t)c->world;
  a.nq = nq;
  a.k = k;
  a.out_ids = d_out_ids;
  a.out_dists = d_out_dists;
  a.out_n = d_out_n;
  a.part_stride = stride;
  a.err_out = c->err.p;
  HIP_OK(launch_merge_packed(a, c->gathered.p, s));
  if (!id_offsets) return 0;
  // the offsets came from the caller's host array: done before return
  return ngt_amd_shard_comm_synchronize(c, s);
}

extern "C" int ngt_amd_shard_comm_set_offsets(ngt_amd_shard_comm* c, const uint32_t* id_offsets) {
  if (!c || !id_offsets) return fail("ngt_amd_shard_comm_set_offsets: bad arguments");
  HIP_OK(hipSetDevice(c->device));
  HIP_OK(c->off.upload(id_offsets, (size_t)c->world));
  c->have_offsets = true;
  return 0;
}

extern "C" int ngt_amd_shard_comm_synchronize(ngt_amd_shard_comm* c, void* stream) {
  if (!c) return fail("ngt_amd_shard_comm_synchronize: null communicator");
  HIP_OK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  int flag = 0;
  HIP_OK(hipMemcpyAsync(&flag, c->err.p, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  if (flag) {
    HIP_OK(hipMemsetAsync(c->err.p, 0, sizeof(int), s));
    HIP_OK(hipStreamSynchronize(s));
    return fail("sharded search: a shard's search flagged device error %d (%s)", flag,
                device_error_text(flag).c_str());
  }
  return 0;
}

extern "C" int ngt_amd_sharded_search_device(ngt_amd_shard_comm* c, ngt_amd_index* ix,
                                             const ngt_amd_search_params* prm, const void* d_queries,
                                             uint64_t query_bytes, uint32_t nq, const uint32_t* d_seeds,
                                             const uint64_t* d_seed_off, const uint32_t* id_offsets,
                                             uint32_t* d_out_ids, float* d_out_dists, uint32_t* d_out_n,
                                             void* stream) {
  if (!c || !ix || !prm || !d_out_ids || !d_out_dists || !d_out_n || prm->k == 0)
    return fail("ngt_amd_sharded_search_device: bad arguments");
  HIP_OK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  HIP_OK(c->ids.alloc((uint64_t)nq * prm->k));
  HIP_OK(c->dists.alloc((uint64_t)nq * prm->k));
  HIP_OK(c->n.alloc(nq ? nq : 1));
  if (ngt_amd_search_device(ix, prm, d_queries, query_bytes, nq, d_seeds, d_seed_off, c->ids.p, c->dists.p, c->n.p,
                            nullptr, stream))
    return -1;
  return exchange_and_merge(c, ix, nq, prm->k, id_offsets, d_out_ids, d_out_dists, d_out_n, s);
}

extern "C" int ngt_amd_sharded_qg_search_device(ngt_amd_shard_comm* c, ngt_amd_index* ix,
                                                const ngt_amd_qg_search_params* prm, const void* d_queries,
                                                uint64_t query_bytes, uint32_t nq, const uint32_t* d_seeds,
                                                const uint64_t* d_seed_off, const uint32_t* id_offsets,
                                                uint32_t* d_out_ids, float* d_out_dists, uint32_t* d_out_n,
                                                void* stream) {
  if (!c || !ix || !prm || !d_out_ids || !d_out_dists || !d_out_n || prm->k == 0)
    return fail("ngt_amd_sharded_qg_search_device: bad arguments");
  HIP_OK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  HIP_OK(c->ids.alloc((uint64_t)nq * prm->k));
  HIP_OK(c->dists.alloc((uint64_t)nq * prm->k));
  HIP_OK(c->n.alloc(nq ? nq : 1));
  if (ngt_amd_qg_search_device(ix, prm, d_queries, query_bytes, nq, d_seeds, d_seed_off, c->ids.p, c->dists.p,
                               c->n.p, nullptr, stream))
    return -1;
  return exchange_and_merge(c, ix, nq, prm->k, id_offsets, d_out_ids, d_out_dists, d_out_n, s);
}
