// qg_api.cpp -- host side of the NGTQG entry points of include/ngt_amd.h.
//
// The quantized graph of an index lives in HBM as two fixed-stride slabs:
//   qids   [nrows][id_stride]   neighbour ids, 0-terminated (id_stride =
//                               max degree rounded up to 16)
//   qcodes [nrows][code_stride] packed 4-bit codes, (id_stride/16) blocks of
//                               8*Me bytes in the reference stream layout
//                               (Quantizer.h:1295-1327)
// so an expansion addresses both from the node id alone.  Every ADC and
// every search runs on the device (qg_kernels.hip); there is no CPU path.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cfloat>
#include <vector>

#include "../../include/ngt_amd.h"
#include "index_internal.h"
#include "ngt_kernels.h"

using namespace ngt_amd;

static const uint32_t kMaxMe = 512;  // packed u16 sums exact up to Me = 514

extern "C" int ngt_amd_qg_set_quantizer(ngt_amd_index* ix, const float* global, const float* local, uint32_t M,
                                        uint32_t dsub) {
  if (!ix || !global || !local || M == 0 || dsub == 0) return fail("ngt_amd_qg_set_quantizer: bad arguments");
  if (ix->metric != NGT_AMD_DISTANCE_L2 || ix->otype != NGT_AMD_OBJECT_FLOAT)
    return fail("ngt_amd_qg_set_quantizer: NGTQG needs an L2 float index");
  if ((uint64_t)M * dsub != ix->dim)
    return fail("ngt_amd_qg_set_quantizer: M (%u) x dsub (%u) != dimension (%u)", M, dsub, ix->dim);
  const uint32_t Me = (M + 1) / 2 * 2;
  if (Me > kMaxMe) return fail("ngt_amd_qg_set_quantizer: %u subspaces exceed the supported %u", M, kMaxMe);
  HIP_OK(hipSetDevice(ix->device));
  QgState& q = ix->qg;
  HIP_OK(q.global.upload(global, ix->dim));
  HIP_OK(q.local.upload(local, (size_t)M * 16 * dsub));
  if (q.M != M) {
    q.qids.release();
    q.qcodes.release();
    q.recs.release();
    q.qkw.release();
    q.packed = false;
    q.has_graph = false;
  }
  q.M = M;
  q.dsub = dsub;
  q.Me = Me;
  q.ready = true;
  q.has_codes = false;
  return 0;
}

extern "C" int ngt_amd_qg_encode(ngt_amd_index* ix, uint8_t* codes_out) {
  if (!ix) return fail("ngt_amd_qg_encode: bad arguments");
  if (!ix->qg.ready) return fail("ngt_amd_qg_encode: set or train the quantizer first");
  if (ix->nrows < 2) return fail("ngt_amd_qg_encode: the index has no objects");
  QgState& q = ix->qg;
  if (q.dsub > 16) return fail("ngt_amd_qg_encode: subvector dimension %u > 16 is not supported", q.dsub);
  HIP_OK(hipSetDevice(ix->device));
  HIP_OK(q.codes.alloc((size_t)ix->nrows * q.M));
  HIP_OK(hipMemsetAsync(q.codes.p, 0, (size_t)q.M, ix->stream));
  QgEncodeArgs a{};
  a.rows = ix->rows.p;
  a.row_bytes = ix->row_bytes;
  a.row0 = 1;
  a.nrows = ix->nrows - 1;
  a.global = q.global.p;
  a.local = q.local.p;
  a.M = q.M;
  a.dsub = q.dsub;
  a.codes = q.codes.p;
  HIP_OK(launch_qg_encode(a, ix->stream));
  HIP_OK(hipStreamSynchronize(ix->stream));
  q.has_codes = true;
  if (codes_out) HIP_OK(hipMemcpy(codes_out, q.codes.p, (size_t)ix->nrows * q.M, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int ngt_amd_qg_train(ngt_amd_index* ix, uint32_t M, uint32_t nsample, uint32_t max_iter,
                                float* local_out, uint32_t* iters_out) {
  if (!ix || M == 0) return fail("ngt_amd_qg_train: bad arguments");
  if (ix->dim % M) return fail("ngt_amd_qg_train: dimension %u is not a multiple of M = %u", ix->dim, M);
  const uint32_t dsub = ix->dim / M;
  if (dsub > 16) return fail("ngt_amd_qg_train: subvector dimension %u > 16 is not supported", dsub);
  if (nsample < 16 || nsample > 4096) return fail("ngt_amd_qg_train: nsample %u not in [16, 4096]", nsample);
  if (ix->nrows < (uint64_t)nsample + 1) return fail("ngt_amd_qg_train: %u samples need %u objects", nsample, nsample);
  if ((size_t)nsample * dsub + 16 * dsub + nsample + nsample / 4 + 1 > 16384)
    return fail("ngt_amd_qg_train: nsample x dsub too large for one workgroup's LDS");
  HIP_OK(hipSetDevice(ix->device));
  std::vector<float> zero(ix->dim, 0.0f);
  DevBuf<float> g, local;
  DevBuf<uint32_t> iters;
  HIP_OK(g.upload(zero.data(), zero.size()));
  HIP_OK(local.alloc((size_t)M * 16 * dsub));
  HIP_OK(iters.alloc(M));
  QgTrainArgs a{};
  a.rows = ix->rows.p;
  a.row_bytes = ix->row_bytes;
  a.nsample = nsample;
  a.global = g.p;
  a.M = M;
  a.dsub = dsub;
  a.max_iter = max_iter == 0 ? 20 : max_iter;
  a.local = local.p;
  a.iters = iters.p;
  HIP_OK(launch_qg_train(a, ix->stream));
  HIP_OK(hipStreamSynchronize(ix->stream));
  std::vector<float> h((size_t)M * 16 * dsub);
  HIP_OK(hipMemcpy(h.data(), local.p, h.size() * sizeof(float), hipMemcpyDeviceToHost));
  if (iters_out) HIP_OK(hipMemcpy(iters_out, iters.p, (size_t)M * sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (local_out) std::copy(h.begin(), h.end(), local_out);
  return ngt_amd_qg_set_quantizer(ix, zero.data(), h.data(), M, dsub);
}

// The packed search layout (qg_kernels.hip): blocks per node on the device,
// record units and key words on the host (a prefix sum in id order), then the
// records.  Used when the search kernel variant holds a whole node's blocks
// (<= 8 with one LUT pair per lane, <= 4 with two) and 2^29 record units of
// at most 4 KiB cover the graph; otherwise searches read the fixed slabs.
static int qg_pack(ngt_amd_index* ix) {
  QgState& q = ix->qg;
  q.packed = false;
  q.recs.release();
  q.qkw.release();
  q.rec_bytes = 0;
  const uint32_t pairs = q.Me / 2;
  const uint32_t nbmax = pairs <= 64 ? 8u : (pairs <= 128 ? 4u : 0u);
  if (q.id_stride / 16 > nbmax) return 0;
  if (const char* v = ngt_amd::knob("NGT_AMD_QG_PACKED"))
    if (atoi(v) == 0) return 0;
  const uint64_t n = ix->nrows;
  DevBuf<uint8_t> dnb;
  HIP_OK(dnb.alloc(n));
  HIP_OK(launch_qg_blocks(q.qids.p, q.id_stride, (uint32_t)n, dnb.p, ix->stream));
  std::vector<uint8_t> nb(n);
  HIP_OK(hipMemcpyAsync(nb.data(), dnb.p, n, hipMemcpyDeviceToHost, ix->stream));
  HIP_OK(hipStreamSynchronize(ix->stream));
  const uint64_t rec_per_block = (uint64_t)8 * q.Me + 128;  // codes + 16 entries of 8 bytes
  uint32_t shift = 7;
  uint64_t units = 0;
  for (; shift <= 12; shift++) {
    units = 0;
    for (uint64_t v = 1; v < n; v++) units += (nb[v] * rec_per_block + (1ull << shift) - 1) >> shift;
    if (units < (1ull << 29)) break;
  }
  if (shift > 12) return 0;
  const uint64_t bytes = units << shift;
  size_t fr = 0, tot = 0;
  HIP_OK(hipMemGetInfo(&fr, &tot));
  if (bytes > fr / 10 * 7) return 0;  // leave room for the search scratch
  std::vector<uint32_t> kw(n, 0u);
  uint64_t u = 0;
  for (uint64_t v = 1; v < n; v++) {
    kw[v] = (uint32_t)(u << 3) | (uint32_t)(nb[v] - 1);
    u += (nb[v] * rec_per_block + (1ull << shift) - 1) >> shift;
  }
  HIP_OK(q.qkw.upload(kw.data(), n));
  HIP_OK(q.recs.alloc(bytes));
  HIP_OK(launch_qg_pack(q.qids.p, q.id_stride, q.qcodes.p, q.code_stride, q.Me, (uint32_t)n, q.qkw.p, shift, q.recs.p,
                        ix->stream));
  HIP_OK(hipStreamSynchronize(ix->stream));
  q.rec_shift = shift;
  q.rec_bytes = bytes;
  q.packed = true;
  return 0;
}

// The packed records are an optional speedup over the fixed slabs the graph
// build leaves in place: a pack that fails (allocation, upload, kernel) leaves
// the index unpacked, and searches read the slabs.
static int qg_pack_or_slabs(ngt_amd_index* ix) {
  if (qg_pack(ix) == 0) return 0;
  QgState& q = ix->qg;
  q.packed = false;
  q.recs.release();
  q.qkw.release();
  q.rec_bytes = 0;
  (void)hipGetLastError();  // the failed call's sticky error
  return 0;
}

extern "C" uint64_t ngt_amd_qg_record_bytes(const ngt_amd_index* ix) {
  return ix && ix->qg.has_graph && ix->qg.packed ? ix->qg.rec_bytes : 0;
}

static int alloc_qg_graph(ngt_amd_index* ix, uint64_t maxdeg) {
  QgState& q = ix->qg;
  const uint32_t stride = (uint32_t)std::max<uint64_t>(16, (maxdeg + 15) & ~15ull);
  if (stride > 256) return fail("qg graph: %llu neighbours per node exceed the supported 256",
                                (unsigned long long)maxdeg);
  q.id_stride = stride;
  q.code_stride = (uint64_t)(stride / 16) * 8 * q.Me;
  HIP_OK(q.qids.alloc((size_t)ix->nrows * q.id_stride));
  HIP_OK(q.qcodes.alloc((size_t)ix->nrows * q.code_stride));
  return 0;
}

extern "C" int ngt_amd_qg_build_graph(ngt_amd_index* ix, const uint8_t* local_codes, uint32_t max_edges) {
  if (!ix || max_edges == 0) return fail("ngt_amd_qg_build_graph: bad arguments");
  if (!local_codes && !ix->qg.has_codes) return fail("ngt_amd_qg_build_graph: no codes given and none encoded");
  if (!ix->qg.ready) return fail("ngt_amd_qg_build_graph: set the quantizer first");
  if (!ix->has_graph) return fail("ngt_amd_qg_build_graph: the index has no graph");
  HIP_OK(hipSetDevice(ix->device));
  QgState& q = ix->qg;
  if (alloc_qg_graph(ix, std::min<uint64_t>(ix->max_degree, max_edges))) return -1;
  DevBuf<uint8_t> codes;
  if (local_codes) HIP_OK(codes.upload(local_codes, (size_t)ix->nrows * q.M));
  QgBuildArgs a{};
  a.edge_off = ix->edge_off.p;
  a.edges = ix->edges.p;
  a.nrows = (uint32_t)ix->nrows;
  a.max_edges = max_edges;
  a.local_codes = local_codes ? codes.p : q.codes.p;
  a.M = q.M;
  a.Me = q.Me;
  a.qids = q.qids.p;
  a.id_stride = q.id_stride;
  a.qcodes = q.qcodes.p;
  a.code_stride = q.code_stride;
  HIP_OK(launch_qg_build(a, ix->stream));
  HIP_OK(hipStreamSynchronize(ix->stream));
  q.has_graph = true;
  return qg_pack_or_slabs(ix);
}

extern "C" int ngt_amd_qg_set_graph(ngt_amd_index* ix, const uint64_t* qoff, const uint32_t* qids,
                                    const uint64_t* code_off, const uint8_t* codes) {
  if (!ix || !qoff || !code_off) return fail("ngt_amd_qg_set_graph: bad arguments");
  if (!ix->qg.ready) return fail("ngt_amd_qg_set_graph: set the quantizer first");
  if (ix->nrows == 0) return fail("ngt_amd_qg_set_graph: set the objects first");
  HIP_OK(hipSetDevice(ix->device));
  QgState& q = ix->qg;
  const uint64_t n = ix->nrows;
  uint64_t maxdeg = 0;
  for (uint64_t v = 0; v < n; v++) {
    const uint64_t deg = qoff[v + 1] - qoff[v];
    const uint64_t nb = deg == 0 ? 0 : (deg - 1) / 16 + 1;
    if (code_off[v + 1] - code_off[v] != nb * 8 * q.Me)
      return fail("ngt_amd_qg_set_graph: node %llu has %llu code bytes, expected %llu", (unsigned long long)v,
                  (unsigned long long)(code_off[v + 1] - code_off[v]), (unsigned long long)(nb * 8 * q.Me));
    for (uint64_t i = qoff[v]; i < qoff[v + 1]; i++)
      if (qids[i] == 0 || qids[i] >= n) return fail("ngt_amd_qg_set_graph: neighbour id %u out of range", qids[i]);
    maxdeg = std::max(maxdeg, deg);
  }
  if (alloc_qg_graph(ix, maxdeg)) return -1;
  std::vector<uint32_t> hid((size_t)n * q.id_stride, 0u);
  std::vector<uint8_t> hcode((size_t)n * q.code_stride, 0u);
  for (uint64_t v = 0; v < n; v++) {
    std::copy(qids + qoff[v], qids + qoff[v + 1], hid.begin() + v * q.id_stride);
    std::copy(codes + code_off[v], codes + code_off[v + 1], hcode.begin() + v * q.code_stride);
  }
  HIP_OK(hipMemcpy(q.qids.p, hid.data(), hid.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(q.qcodes.p, hcode.data(), hcode.size(), hipMemcpyHostToDevice));
  q.has_graph = true;
  return qg_pack_or_slabs(ix);
}

extern "C" uint32_t ngt_amd_qg_max_degree(const ngt_amd_index* ix) {
  return ix && ix->qg.has_graph ? ix->qg.id_stride : 0;
}

extern "C" uint64_t ngt_amd_qg_code_stride(const ngt_amd_index* ix) {
  return ix && ix->qg.has_graph ? ix->qg.code_stride : 0;
}

extern "C" int ngt_amd_qg_get_graph(const ngt_amd_index* ix, uint32_t* ids, uint8_t* codes) {
  if (!ix || !ids || !codes) return fail("ngt_amd_qg_get_graph: bad arguments");
  if (!ix->qg.has_graph) return fail("ngt_amd_qg_get_graph: the index has no quantized graph");
  HIP_OK(hipSetDevice(ix->device));
  const QgState& q = ix->qg;
  HIP_OK(hipMemcpy(ids, q.qids.p, (size_t)ix->nrows * q.id_stride * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(codes, q.qcodes.p, (size_t)ix->nrows * q.code_stride, hipMemcpyDeviceToHost));
  return 0;
}

// LUTs of nq prepared device queries into c->lut/scale/toff.
static int run_lut(ngt_amd_index* ix, SearchCtx* c, const void* d_queries, uint64_t query_bytes, uint32_t nq,
                   hipStream_t s) {
  QgState& q = ix->qg;
  HIP_OK(c->lut.alloc((size_t)nq * q.Me * 16));
  HIP_OK(c->scale.alloc(nq));
  HIP_OK(c->toff.alloc(nq));
  QgLutArgs a{};
  a.queries = static_cast<const uint8_t*>(d_queries);
  a.query_bytes = query_bytes;
  a.nq = nq;
  a.global = q.global.p;
  a.local = q.local.p;
  a.M = q.M;
  a.dsub = q.dsub;
  a.Me = q.Me;
  a.lut = c->lut.p;
  a.lut_stride = (uint64_t)q.Me * 16;
  a.scale = c->scale.p;
  a.toff = c->toff.p;
  HIP_OK(launch_qg_lut(a, s));
  return 0;
}

extern "C" int ngt_amd_qg_lut(ngt_amd_index* ix, const float* queries, uint32_t nq, uint8_t* lut, float* scale,
                              float* total_offset) {
  if (!ix || (!queries && nq) || !lut || !scale || !total_offset) return fail("ngt_amd_qg_lut: bad arguments");
  if (!ix->qg.ready) return fail("ngt_amd_qg_lut: the index has no quantizer");
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(ix->device));
  CallGuard g(ix);
  if (!g.c) return -1;
  hipStream_t s = g.c->stream;
  if (upload_queries(ix, queries, nq, g.c->raw, g.c->prep, s)) return -1;
  SearchCtx* c = ctx_for(ix, s);
  if (!c) return -1;
  if (run_lut(ix, c, g.c->prep.p, ix->row_bytes, nq, s)) return -1;
  const QgState& q = ix->qg;
  HIP_OK(hipMemcpyAsync(lut, c->lut.p, (size_t)nq * q.Me * 16, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(scale, c->scale.p, nq * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(total_offset, c->toff.p, nq * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int ngt_amd_qg_adc(ngt_amd_index* ix, const uint8_t* lut, const float* scale, const float* total_offset,
                              uint32_t nq, const uint32_t* qidx, const uint32_t* node, uint64_t npairs, float* out,
                              uint32_t* out_n) {
  if (!ix || !lut || !scale || !total_offset || !qidx || !node || !out || !out_n)
    return fail("ngt_amd_qg_adc: bad arguments");
  if (!ix->qg.has_graph) return fail("ngt_amd_qg_adc: the index has no quantized graph");
  if (npairs == 0) return 0;
  for (uint64_t i = 0; i < npairs; i++) {
    if (qidx[i] >= nq) return fail("ngt_amd_qg_adc: query index %u out of range", qidx[i]);
    if (node[i] >= ix->nrows) return fail("ngt_amd_qg_adc: node %u out of range", node[i]);
  }
  HIP_OK(hipSetDevice(ix->device));
  CallGuard g(ix);
  if (!g.c) return -1;
  hipStream_t s = g.c->stream;
  const QgState& q = ix->qg;
  DevBuf<uint8_t> dl;
  DevBuf<float> dsc, dto, dout;
  DevBuf<uint32_t> dq, dn, dcnt;
  HIP_OK(dl.upload(lut, (size_t)nq * q.Me * 16));
  HIP_OK(dsc.upload(scale, nq));
  HIP_OK(dto.upload(total_offset, nq));
  HIP_OK(dq.upload(qidx, npairs));
  HIP_OK(dn.upload(node, npairs));
  HIP_OK(dout.alloc((size_t)npairs * q.id_stride));
  HIP_OK(dcnt.alloc(npairs));
  QgAdcArgs a{};
  a.qids = q.qids.p;
  a.id_stride = q.id_stride;
  a.qcodes = q.qcodes.p;
  a.code_stride = q.code_stride;
  a.Me = q.Me;
  a.lut = dl.p;
  a.lut_stride = (uint64_t)q.Me * 16;
  a.scale = dsc.p;
  a.toff = dto.p;
  a.qidx = dq.p;
  a.node = dn.p;
  a.npairs = npairs;
  a.out = dout.p;
  a.out_stride = q.id_stride;
  a.out_n = dcnt.p;
  HIP_OK(hipMemsetAsync(dout.p, 0, (size_t)npairs * q.id_stride * sizeof(float), s));
  HIP_OK(launch_qg_adc(a, s));
  HIP_OK(hipMemcpyAsync(out, dout.p, (size_t)npairs * q.id_stride * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(out_n, dcnt.p, npairs * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

extern "C" int ngt_amd_qg_search_device(ngt_amd_index* ix, const ngt_amd_qg_search_params* prm,
                                        const void* d_queries, uint64_t query_bytes, uint32_t nq,
                                        const uint32_t* d_seeds, const uint64_t* d_seed_off, uint32_t* d_ids,
                                        float* d_dists, uint32_t* d_n, uint64_t* d_counters, void* stream) {
  if (!ix || !prm || (!d_queries && nq)) return fail("ngt_amd_qg_search_device: bad arguments");
  if (nq && query_bytes < ix->row_bytes)
    return fail("ngt_amd_qg_search_device: query stride %llu < %llu bytes (queries are prepared rows of the padded dimension)",
                (unsigned long long)query_bytes, (unsigned long long)ix->row_bytes);
  if (!ix->qg.has_graph) return fail("ngt_amd_qg_search: the index has no quantized graph");
  if (prm->k == 0) return fail("ngt_amd_qg_search: k must be > 0");
  if (nq == 0) return 0;
  HIP_OK(hipSetDevice(ix->device));
  hipStream_t s = (hipStream_t)stream;
  QgState& q = ix->qg;
  SearchCtx* c = ctx_for(ix, s);
  if (!c) return -1;

  QgSearchArgs a{};
  a.rows = ix->rows.p;
  a.row_bytes = ix->row_bytes;
  a.nrows = (uint32_t)ix->nrows;
  a.dp = (int)ix->dp;
  a.qids = q.qids.p;
  a.id_stride = q.id_stride;
  a.qcodes = q.qcodes.p;
  a.code_stride = q.code_stride;
  a.Me = q.Me;
  a.recs = q.packed ? q.recs.p : nullptr;
  a.qkw = q.qkw.p;
  a.rec_shift = q.rec_shift;
  a.queries = static_cast<const uint8_t*>(d_queries);
  a.query_bytes = query_bytes;
  a.nq = nq;
  a.k = prm->k;
  // sc.size *= resultExpansion: size_t * float -> float -> size_t (QuantizedGraph.h:194-196)
  uint64_t size = prm->k;
  if (prm->result_expansion > 1.0f) size = (uint64_t)((float)size * prm->result_expansion);
  if (size == 0) return fail("ngt_amd_qg_search: empty result size");
  a.size = (uint32_t)size;
  a.rerank = prm->result_expansion >= 1.0f;
  a.coef = coef_of(prm->epsilon);
  a.radius = prm->radius < 0.0f ? FLT_MAX : prm->radius;
  a.ht_log2 = 12;
  a.cq_cap = 1024;
  a.vf_log2 = 0;
  if (prm->visited_hash_log2 < 0) {
    // HBM epochs behind an LDS filter of accepted ids, which lets ids_and_adc
    // probe the possibly-visited neighbours while the ADC runs instead of a
    // round trip in the accept step.  With the register head the LDS tail
    // needs only 256 keys, and their room buys a 32 Kbit filter: fewer false
    // positives, fewer probes (round 5, profiles/r5k / r5l: 2M one-ANNG QG
    // +5.6 %, C2-graph QG +3 %; 64 Kbit costs resident waves and loses).
    a.ht_log2 = 0;
    a.cq_cap = 256;
    a.vf_log2 = 15;
  }
  else if (prm->visited_hash_log2 > 0) a.ht_log2 = (uint32_t)std::max(8, std::min(15, prm->visited_hash_log2));
  if (const char* v = ngt_amd::knob("NGT_AMD_HT_LOG2")) a.ht_log2 = (uint32_t)std::max(8, std::min(15, atoi(v)));
  if (const char* v = ngt_amd::knob("NGT_AMD_CQ_CAP")) a.cq_cap = (uint32_t)std::max(64, std::min(8192, atoi(v)));
  if (const char* v = ngt_amd::knob("NGT_AMD_VFILTER")) {
    const int f = atoi(v);
    a.vf_log2 = f <= 0 ? 0u : (uint32_t)std::max(11, std::min(18, f));
  }
  a.out_ids = d_ids;
  a.out_dists = d_dists;
  a.out_n = d_n;
  a.counters = d_counters;
  a.error = c->err.p;

  if (prm->seed_mode == NGT_AMD_SEED_TREE) {
    // getSeedsFromTree with the caller's k (before the expansion, :362)
    if (run_tree_seeds(ix, c, d_queries, query_bytes, nq, prm->k, 0, s)) return -1;
    a.seeds = c->seeds.p;
    a.seed_stride = kTreeSeedStride;
    a.seed_count = c->seed_count.p;
  } else if (prm->seed_mode == NGT_AMD_SEED_RANDOM) {
    std::vector<uint64_t> off;
    std::vector<uint32_t> seeds = random_seed_lists(ix, nq, off);
    HIP_OK(c->seed_off.upload(off.data(), off.size()));
    HIP_OK(c->seeds.upload(seeds.data(), std::max<size_t>(seeds.size(), 1)));
    a.seeds = c->seeds.p;
    a.seed_off = c->seed_off.p;
  } else {
    if (!d_seeds || !d_seed_off) return fail("ngt_amd_qg_search: seed lists required for this seed mode");
    a.seeds = d_seeds;
    a.seed_off = d_seed_off;
  }
  if (run_lut(ix, c, d_queries, query_bytes, nq, s)) return -1;
  a.lut = c->lut.p;
  a.lut_stride = (uint64_t)q.Me * 16;
  a.scale = c->scale.p;
  a.toff = c->toff.p;

  const size_t lds = qg_search_lds_bytes(a);
  if (lds > 64 * 1024)
    return fail("ngt_amd_qg_search: k=%u x expansion needs %zu bytes of LDS per query (max 65536)", a.k, lds);
  if (ensure_vis_scratch(ix, c, lds, nq, s)) return -1;
  a.vis = c->vis.p;
  a.vis_stride = c->vis_stride;
  a.slot_epoch = c->slot_epoch.p;
  a.spill = c->spill.p;
  a.spill_cap = ix->spill_cap;
  a.work = c->work.p;
  HIP_OK(hipMemsetAsync(c->work.p, 0, sizeof(uint32_t), s));
  const uint32_t slots = std::min<uint32_t>(c->slots, nq);
  c->launch_slots = slots;
  HIP_OK(hipEventRecord(c->ev0, s));
  HIP_OK(launch_qg_search(a, slots, s));
  HIP_OK(hipEventRecord(c->ev1, s));
  return 0;
}

extern "C" int ngt_amd_qg_search(ngt_amd_index* ix, const ngt_amd_qg_search_params* prm, const float* queries,
                                 uint32_t nq, const uint32_t* seeds, const uint64_t* seed_off, uint32_t* ids,
                                 float* dists, uint32_t* n, uint64_t* counters) {
  if (!ix || !prm || (!queries && nq) || !ids || !dists || !n) return fail("ngt_amd_qg_search: bad arguments");
  if (nq == 0) return 0;
  if (prm->seed_mode == NGT_AMD_SEED_GIVEN) {
    if (!seeds || !seed_off) return fail("ngt_amd_qg_search: NGT_AMD_SEED_GIVEN needs seeds and seed_off");
    for (uint64_t i = 0; i < seed_off[nq]; i++)
      if (seeds[i] == 0 || seeds[i] >= ix->nrows) return fail("ngt_amd_qg_search: seed id %u out of range", seeds[i]);
  }
  HIP_OK(hipSetDevice(ix->device));
  CallGuard g(ix);
  CallCtx* cc = g.c;
  if (!cc) return -1;
  hipStream_t s = cc->stream;
  if (clear_device_error(ix, s)) return -1;
  if (upload_queries(ix, queries, nq, cc->raw, cc->prep, s)) return -1;
  HIP_OK(cc->ids.alloc((size_t)nq * prm->k));
  HIP_OK(cc->dists.alloc((size_t)nq * prm->k));
  HIP_OK(cc->n.alloc(nq));
  if (counters) HIP_OK(cc->cnt.alloc((size_t)nq * NGT_AMD_COUNTERS_PER_QUERY));
  const uint32_t* sp = nullptr;
  const uint64_t* so = nullptr;
  if (prm->seed_mode == NGT_AMD_SEED_GIVEN) {
    HIP_OK(cc->seeds.alloc(std::max<uint64_t>(seed_off[nq], 1)));
    HIP_OK(cc->seed_off.alloc((size_t)nq + 1));
    HIP_OK(hipMemcpyAsync(cc->seeds.p, seeds, seed_off[nq] * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(cc->seed_off.p, seed_off, ((size_t)nq + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    sp = cc->seeds.p;
    so = cc->seed_off.p;
  }
  if (ngt_amd_qg_search_device(ix, prm, cc->prep.p, ix->row_bytes, nq, sp, so, cc->ids.p, cc->dists.p, cc->n.p,
                               counters ? cc->cnt.p : nullptr, s))
    return -1;
  HIP_OK(hipMemcpyAsync(ids, cc->ids.p, (size_t)nq * prm->k * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(dists, cc->dists.p, (size_t)nq * prm->k * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(n, cc->n.p, (size_t)nq * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (counters)
    HIP_OK(hipMemcpyAsync(counters, cc->cnt.p, (size_t)nq * NGT_AMD_COUNTERS_PER_QUERY * sizeof(uint64_t),
                          hipMemcpyDeviceToHost, s));
  int herr = 0;
  if (take_device_error(ix, s, &herr)) return -1;
  if (herr) return fail("ngt_amd_qg_search: device error flag %d (%s)", herr, device_error_text(herr).c_str());
  return 0;
}
