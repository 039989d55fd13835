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

// pack -> all-gather -> merge of this rank's [nq][k] lists (already searched)
static int exchange_and_merge(ngt_amd_shard_comm* c, uint32_t nq, uint32_t k, const uint32_t* id_offsets,
                              uint32_t* d_out_ids, float* d_out_dists, uint32_t* d_out_n, hipStream_t s) {
  if ((uint64_t)c->world * k * sizeof(uint64_t) > 64 * 1024)
    return fail("sharded search: %d shards x k=%u exceed one workgroup's LDS in the merge", c->world, k);
  const uint64_t words = (uint64_t)nq * k;
  HIP_OK(c->packed.alloc(words));
  HIP_OK(c->gathered.alloc(words * c->world));
  HIP_OK(c->off.alloc(c->world));
  HIP_OK(launch_pack_results(c->ids.p, c->dists.p, c->n.p, nq, k, c->packed.p, s));
  NCCL_OK(ncclAllGather(c->packed.p, c->gathered.p, words, ncclUint64, c->comm, s));
  HIP_OK(hipMemcpyAsync(c->off.p, id_offsets, c->world * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  MergeArgs a{};
  a.id_offsets = c->off.p;
  a.nparts = (uint32_t)c->world;
  a.nq = nq;
  a.k = k;
  a.out_ids = d_out_ids;
  a.out_dists = d_out_dists;
  a.out_n = d_out_n;
  HIP_OK(launch_merge_packed(a, c->gathered.p, s));
  // the offsets were copied from the caller's host array: done before return
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int ngt_amd_sharded_search_device(ngt_amd_shard_comm* c, ngt_amd_index* ix,
                                             const ngt_amd_search_params* prm, const void* d_queries,
                                             uint64_t query_bytes, uint32_t nq, const uint32_t* d_seeds,
                                             const uint64_t* d_seed_off, const uint32_t* id_offsets,
                                             uint32_t* d_out_ids, float* d_out_dists, uint32_t* d_out_n,
                                             void* stream) {
  if (!c || !ix || !prm || !id_offsets || !d_out_ids || !d_out_dists || !d_out_n || prm->k == 0)
    return fail("ngt_amd_sharded_search_device: bad arguments");
  HIP_OK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  HIP_OK(c->ids.alloc((uint64_t)nq * prm->k));
  HIP_OK(c->dists.alloc((uint64_t)nq * prm->k));
  HIP_OK(c->n.alloc(nq ? nq : 1));
  if (ngt_amd_search_device(ix, prm, d_queries, query_bytes, nq, d_seeds, d_seed_off, c->ids.p, c->dists.p, c->n.p,
                            nullptr, stream))
    return -1;
  return exchange_and_merge(c, nq, prm->k, id_offsets, d_out_ids, d_out_dists, d_out_n, s);
}

extern "C" int ngt_amd_sharded_qg_search_device(ngt_amd_shard_comm* c, ngt_amd_index* ix,
                                                const ngt_amd_qg_search_params* prm, const void* d_queries,
                                                uint64_t query_bytes, uint32_t nq, const uint32_t* d_seeds,
                                                const uint64_t* d_seed_off, const uint32_t* id_offsets,
                                                uint32_t* d_out_ids, float* d_out_dists, uint32_t* d_out_n,
                                                void* stream) {
  if (!c || !ix || !prm || !id_offsets || !d_out_ids || !d_out_dists || !d_out_n || prm->k == 0)
    return fail("ngt_amd_sharded_qg_search_device: bad arguments");
  HIP_OK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  HIP_OK(c->ids.alloc((uint64_t)nq * prm->k));
  HIP_OK(c->dists.alloc((uint64_t)nq * prm->k));
  HIP_OK(c->n.alloc(nq ? nq : 1));
  if (ngt_amd_qg_search_device(ix, prm, d_queries, query_bytes, nq, d_seeds, d_seed_off, c->ids.p, c->dists.p,
                               c->n.p, nullptr, stream))
    return -1;
  return exchange_and_merge(c, nq, prm->k, id_offsets, d_out_ids, d_out_dists, d_out_n, s);
}
