// qg_kernels.hip -- gfx950 kernels for the NGTQG quantized-graph path.
//
//  * ngt_qg_lut_kernel   : QuantizedObjectDistance::createDistanceLookup
//                          (lib/NGT/NGTQ/Quantizer.h:709-760) over
//                          createFloatL2DistanceLookup (:683-706) -- the
//                          per-query uint8 table, scale and totalOffset.
//  * ngt_qg_build_kernel : QuantizedGraphRepository::construct
//                          (lib/NGT/NGTQ/QuantizedGraph.h:64-115) with the
//                          stream layout of QuantizedObjectProcessingStream
//                          (Quantizer.h:1268-1327), into fixed-stride rows.
//  * ngt_qg_adc_kernel   : QuantizedObjectDistanceFloat::operator()
//                          (Quantizer.h:957-1062) over whole neighbour lists.
//  * ngt_qg_search_kernel: NGTQG::Index::searchQuantizedGraph
//                          (QuantizedGraph.h:192-320), one wave per query.
//
// 4-bit ADC on CDNA4: the reference shuffles 16-entry byte tables with
// pshufb.  Here lane l owns subspace pair p = l (+64 s): its two 16-byte
// table rows sit in 8 VGPRs and a lookup of four nibbles is two v_perm_b32
// (8-byte tables) plus a byte select on bit 3.  A 16-object block is 8*Me
// bytes: the 16 bytes of pair p are contiguous at 16p, so one wave-wide
// 16-byte load streams a whole 1 KiB block (M = 128).  Per-object sums are
// packed (even subspaces | odd subspaces << 16), exactly the reference's two
// u16 accumulators, and reduce-scattered across the wave in 17 shuffles
// (16 values -> 1 per lane) instead of 16 full wave reductions.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ngt_device.h"
#include "ngt_kernels.h"
#include "search_common.h"

// 1: the previous all-VALU cross-lane sum (v_perm packing + reduce-scatter)
#ifndef NGT_AMD_QG_VALU_REDUCE
#define NGT_AMD_QG_VALU_REDUCE 0
#endif

namespace ngt_amd {

// ---------------------------------------------------------------------------
// LUT: one wave per query.  d[m][c] = sum_j fma((q - g - C[m][c])^2) in float
// (the -Ofast reference contracts the sum into an FMA chain), one global
// min/max, quantised with roundf((d - min) / scale).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) ngt_qg_lut_kernel(QgLutArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float* d = reinterpret_cast<float*>(smem);
  const int lane = lane_id();
  const uint32_t n = a.M * 16;
  for (uint32_t qi = blockIdx.x; qi < a.nq; qi += gridDim.x) {
    const float* q = reinterpret_cast<const float*>(a.queries + (uint64_t)qi * a.query_bytes);
    float mn = __int_as_float(0x7f7fffff), mx = -__int_as_float(0x7f7fffff);  // FLT_MAX, -FLT_MAX
    for (uint32_t i = lane; i < n; i += 64) {
      const uint32_t m = i >> 4, c = i & 15;
      const float* qq = q + (uint64_t)m * a.dsub;
      const float* gg = a.global + (uint64_t)m * a.dsub;
      const float* lc = a.local + ((uint64_t)m * 16 + c) * a.dsub;
      float acc = 0.0f;
      for (uint32_t j = 0; j < a.dsub; j++) {
        const float sub = (qq[j] - gg[j]) - lc[j];
        acc = __builtin_fmaf(sub, sub, acc);
      }
      d[i] = acc;
      mx = acc > mx ? acc : mx;
      mn = acc < mn ? acc : mn;
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
      const float omx = __shfl_xor(mx, s, 64), omn = __shfl_xor(mn, s, 64);
      mx = omx > mx ? omx : mx;
      mn = omn < mn ? omn : mn;
    }
    __syncthreads();
    const float offset = mn;
    const float scale = (float)((double)(mx - mn) / 255.0);  // (Quantizer.h:738)
    uint8_t* out = a.lut + (uint64_t)qi * a.lut_stride;
    for (uint32_t i = lane; i < a.Me * 16; i += 64) {
      uint8_t v = 0;  // the odd-M pad subspace is zero (:751-757)
      if (i < n) {
        const float t = (d[i] - offset) / scale;
        // (int32_t)round(x) then uint8 truncation; a NaN quotient (scale 0)
        // converts to INT_MIN on x86, whose low byte is 0
        v = (t == t) ? (uint8_t)(int32_t)roundf(t) : (uint8_t)0;
      }
      out[i] = v;
    }
    if (lane == 0) {
      float tot = 0.0f;
      for (uint32_t m = 0; m < a.M; m++) tot += offset;  // totalOffset (:749)
      a.scale[qi] = scale;
      a.toff[qi] = tot;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Quantized graph construction: node v keeps its first min(deg, max_edges)
// graph edges in stored order; codes = localID - 1 per subspace, arranged per
// 16-object block as byte (8m + j) = obj(2j) | obj(2j+1) << 4.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) ngt_qg_build_kernel(QgBuildArgs a) {
  const uint32_t warps = (gridDim.x * blockDim.x) >> 6;
  const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const uint64_t blk = (uint64_t)8 * a.Me;
  for (uint32_t v = w0; v < a.nrows; v += warps) {
    const uint64_t eb = a.edge_off[v];
    uint64_t deg = a.edge_off[v + 1] - eb;
    if (deg > a.max_edges) deg = a.max_edges;
    uint32_t* ids = a.qids + (uint64_t)v * a.id_stride;
    for (uint32_t i = lane; i < a.id_stride; i += 64) ids[i] = i < deg ? a.edges[eb + i] : 0u;
    uint8_t* codes = a.qcodes + (uint64_t)v * a.code_stride;
    const uint64_t nb = deg == 0 ? 0 : (deg - 1) / 16 + 1;
    for (uint64_t t = lane; t < a.code_stride; t += 64) {
      uint8_t byte = 0;
      const uint64_t b = t / blk;
      if (b < nb) {
        const uint64_t r = t - b * blk;
        const uint32_t m = (uint32_t)(r >> 3), j = (uint32_t)(r & 7);
        const uint64_t o0 = b * 16 + 2 * j, o1 = o0 + 1;
        if (m < a.M) {
          if (o0 < deg) byte |= (uint8_t)(a.local_codes[(uint64_t)a.edges[eb + o0] * a.M + m] & 15);
          if (o1 < deg) byte |= (uint8_t)((a.local_codes[(uint64_t)a.edges[eb + o1] * a.M + m] & 15) << 4);
        }
      }
      codes[t] = byte;
    }
  }
}

// ---------------------------------------------------------------------------
// Packed search layout.  The fixed-stride slabs give every node id_stride/16
// code blocks, and an expansion loads them all before it knows the degree
// (on a 128-slot ANNG-based graph with ~42 neighbours, 5 of 8 KiB per
// expansion for nothing).  The packed layout keeps the reference's per-node
// ceil(deg/16) blocks (QuantizedGraphRepository, QuantizedGraph.h:74-113):
// node v's record -- its code blocks, then 16 entries {neighbour id,
// neighbour key word} per block -- sits at unit u(v) of a byte array, records
// in id order; kw(v) = u(v) << 3 | (blocks(v) - 1).  The search's unchecked
// keys carry kw in place of the id (u(v) grows strictly with v, so
// (distance, kw) orders exactly as (distance, id)), so a pop knows where the
// record is and how long, and issues exactly its loads in one round trip.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) ngt_qg_blocks_kernel(const uint32_t* qids, uint32_t id_stride,
                                                            uint32_t nrows, uint8_t* nb) {
  const uint32_t warps = (gridDim.x * blockDim.x) >> 6;
  const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  for (uint32_t v = w0; v < nrows; v += warps) {
    const uint32_t* ids = qids + (uint64_t)v * id_stride;
    uint32_t deg = 0;
    for (uint32_t j = 0; j < id_stride; j += 64)
      deg += (uint32_t)__popcll(ballot64(j + lane < id_stride && ids[j + lane] != 0u));
    // a node without edges keeps one empty block: every record is at least
    // one unit, so the key words stay strictly increasing with the id
    if (lane == 0) nb[v] = (uint8_t)(deg == 0 ? 1u : (deg - 1) / 16 + 1);
  }
}

__global__ void __launch_bounds__(256) ngt_qg_pack_kernel(const uint32_t* qids, uint32_t id_stride,
                                                          const uint8_t* qcodes, uint64_t code_stride, uint32_t Me,
                                                          uint32_t nrows, const uint32_t* qkw, uint32_t rec_shift,
                                                          uint8_t* recs) {
  const uint32_t warps = (gridDim.x * blockDim.x) >> 6;
  const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const uint64_t blk = (uint64_t)8 * Me;
  for (uint32_t v = 1 + w0; v < nrows; v += warps) {
    const uint32_t kw = qkw[v];
    const uint32_t nb = (kw & 7u) + 1u;
    uint8_t* rec = recs + ((uint64_t)(kw >> 3) << rec_shift);
    const uint4* src = reinterpret_cast<const uint4*>(qcodes + (uint64_t)v * code_stride);
    uint4* dst = reinterpret_cast<uint4*>(rec);
    const uint64_t n16 = nb * blk / 16;
    const uint64_t have = code_stride / 16;
    for (uint64_t t = lane; t < n16; t += 64) dst[t] = t < have ? src[t] : make_uint4(0, 0, 0, 0);
    uint2* ent = reinterpret_cast<uint2*>(rec + nb * blk);
    const uint32_t* ids = qids + (uint64_t)v * id_stride;
    for (uint32_t i = lane; i < 16 * nb; i += 64) {
      const uint32_t id = i < id_stride ? ids[i] : 0u;
      ent[i] = make_uint2(id, id ? qkw[id] : 0u);
    }
  }
}

// ---------------------------------------------------------------------------
// Encoder (the local half of Quantizer::insert, lib/NGT/NGTQ/Quantizer.h:
// 1895-1959): residual subvector r = object - global centroid, computed in
// double and stored as float (GenerateResidualObjectFloat, :1407-1435), coded
// as the local centroid nearest to r.  The reference finds it with an NGT
// insertion search of the 16-object local codebook index (createIndex with
// range FLT_MAX, :1678-1719, Index.cpp:1260-1345), whose distances are
// PrimitiveComparator::compareL2 over the zero-padded subvector and whose
// results are ordered by (distance, id): the scalar restatement below keeps
// the 16 AVX-512 lanes, their 16->8->4 fold and the double sqrt, and ties go
// to the lower local id.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float l2_sub(const float* r, const float* c, uint32_t n) {
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; j++) acc[j] = 0.0f;
  for (uint32_t i = 0; i < n; i += 16) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const float v = i + j < n ? r[i + j] - c[i + j] : 0.0f;
      acc[j] = __builtin_fmaf(v, v, acc[j]);
    }
  }
  float t4[4];
#pragma unroll
  for (int j = 0; j < 4; j++) t4[j] = (acc[j + 12] + acc[j + 4]) + (acc[j + 8] + acc[j]);
  return (float)sqrt((double)((t4[0] + t4[1]) + (t4[2] + t4[3])));
}

__global__ void __launch_bounds__(256) ngt_qg_encode_kernel(QgEncodeArgs a) {
  const uint64_t total = a.nrows * a.M;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const uint64_t o = a.row0 + t / a.M;
    const uint32_t m = (uint32_t)(t % a.M);
    const float* x = reinterpret_cast<const float*>(a.rows + o * a.row_bytes) + (uint64_t)m * a.dsub;
    const float* g = a.global + (uint64_t)m * a.dsub;
    float r[16];
    uint32_t best = 0;
    float bd = 0.0f;
    if (a.dsub <= 16) {
#pragma unroll
      for (int d = 0; d < 16; d++) r[d] = (uint32_t)d < a.dsub ? (float)((double)x[d] - (double)g[d]) : 0.0f;
      for (uint32_t c = 0; c < 16; c++) {
        const float dc = l2_sub(r, a.local + ((uint64_t)m * 16 + c) * a.dsub, a.dsub);
        if (c == 0 || dc < bd) { bd = dc; best = c; }
      }
    }
    a.codes[o * a.M + m] = (uint8_t)best;
  }
}

// Local codebook training, one 256-thread workgroup per subspace: the sample
// is the residual subvectors of objects 1..nsample (the reference's dynamic
// k-means collects the first localCentroidLimit * localClusteringSampleCoefficient
// = 16 * 100 objects, Quantizer.h:1803-1844), the initial centroids are its
// first 16 (Clustering::InitializationModeHead, Clustering.h:835-843), then
// Lloyd iterations with exact nearest-centroid assignment (l2_sub, ties to the
// lower id) and centroids as float means summed in sample order, until no
// centroid changes or max_iter.  An empty cluster takes the sample farthest
// from its centroid among clusters with >= 2 members (the intent of
// moveFartherObjectsToEmptyClusters, :405-437).  NOT the reference's
// kmeansWithNGT: its assignment is an approximate NGT range search per
// centroid (assignWithNGT, :440-577), so codebooks differ; encoding, LUT,
// ADC and search given a codebook are the pinned parts.
__global__ void __launch_bounds__(256) ngt_qg_train_kernel(QgTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t m = blockIdx.x;
  const uint32_t ds = a.dsub, n = a.nsample;
  float* s = reinterpret_cast<float*>(smem);         // [n][ds]
  float* cen = s + (uint64_t)n * ds;                  // [16][ds]
  float* sd = cen + 16 * ds;                          // [n] distance to own centroid
  uint8_t* asg = reinterpret_cast<uint8_t*>(sd + n);  // [n]
  __shared__ uint32_t cnt[16];
  __shared__ int changed;
  for (uint32_t i = threadIdx.x; i < n * ds; i += blockDim.x) {
    const uint32_t o = i / ds + 1, d = i % ds;
    const float* x = reinterpret_cast<const float*>(a.rows + (uint64_t)o * a.row_bytes);
    s[i] = (float)((double)x[m * ds + d] - (double)a.global[m * ds + d]);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 16 * ds; i += blockDim.x) cen[i] = s[i];
  __syncthreads();
  uint32_t it = 0;
  for (; it < a.max_iter; it++) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      float r[16];
      for (uint32_t d = 0; d < 16; d++) r[d] = d < ds ? s[i * ds + d] : 0.0f;
      uint32_t best = 0;
      float bd = 0.0f;
      for (uint32_t c = 0; c < 16; c++) {
        const float dc = l2_sub(r, cen + c * ds, ds);
        if (c == 0 || dc < bd) { bd = dc; best = c; }
      }
      asg[i] = (uint8_t)best;
      sd[i] = bd;
    }
    if (threadIdx.x < 16) cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) changed = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (uint32_t i = 0; i < n; i++) cnt[asg[i]]++;
      for (uint32_t c = 0; c < 16; c++) {
        if (cnt[c] != 0) continue;
        // farthest member of any cluster with >= 2 members moves to c
        float mx = -1.0f;
        uint32_t mi = 0xffffffffu;
        for (uint32_t i = 0; i < n; i++)
          if (cnt[asg[i]] >= 2 && sd[i] > mx) { mx = sd[i]; mi = i; }
        if (mi == 0xffffffffu) break;
        cnt[asg[mi]]--;
        asg[mi] = (uint8_t)c;
        sd[mi] = 0.0f;
        cnt[c] = 1;
      }
    }
    __syncthreads();
    // new centroids: float sums in sample order, then / count
    if (threadIdx.x < 16 * ds) {
      const uint32_t c = threadIdx.x / ds, d = threadIdx.x % ds;
      float sum = 0.0f;
      for (uint32_t i = 0; i < n; i++)
        if (asg[i] == c) sum += s[i * ds + d];
      const float v = cnt[c] ? sum / (float)cnt[c] : cen[c * ds + d];
      if (__float_as_uint(v) != __float_as_uint(cen[c * ds + d])) atomicOr(&changed, 1);
      cen[c * ds + d] = v;
    }
    __syncthreads();
    if (!changed) { it++; break; }
  }
  for (uint32_t i = threadIdx.x; i < 16 * ds; i += blockDim.x) a.local[(uint64_t)m * 16 * ds + i] = cen[i];
  if (threadIdx.x == 0) a.iters[m] = it;
}

// ---------------------------------------------------------------------------
// Four table lookups into the 16-byte table t0..t3 (little-endian dwords):
// byte b of the result = table[nibble of byte b of `w` at bit `sh`] for
// sh = 0 (low nibbles) or 4 (high nibbles).  Two v_perm_b32 look the 3 low
// index bits up in the lower and upper 8 table bytes; a third picks, per
// byte, lower or upper by index bit 3 (selector b or 4 + b).
// The pick selector is one v_and_or_b32 (mask from an SGPR, base 0x03020100
// from a VGPR: VOP3 on gfx9 takes no literal and one scalar operand), which
// the compiler otherwise emits as v_and + v_or.
__device__ __forceinline__ uint32_t and_or_b32(uint32_t x, uint32_t mask, uint32_t base) {
  uint32_t r;
  asm volatile("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(mask), "v"(base));
  return r;
}

template <int SH>
__device__ __forceinline__ uint32_t lut16(uint32_t w, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3,
                                          uint32_t base) {
  const uint32_t sel = (w >> SH) & 0x07070707u;
  const uint32_t lo = __builtin_amdgcn_perm(t1, t0, sel);
  const uint32_t hi = __builtin_amdgcn_perm(t3, t2, sel);
  const uint32_t pick = and_or_b32(w >> (SH + 1), 0x04040404u, base);
  return __builtin_amdgcn_perm(hi, lo, pick);
}

template <int SH>
__device__ __forceinline__ uint32_t lut16(uint32_t w, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3) {
  const uint32_t sel = (w >> SH) & 0x07070707u;
  const uint32_t lo = __builtin_amdgcn_perm(t1, t0, sel);
  const uint32_t hi = __builtin_amdgcn_perm(t3, t2, sel);
  const uint32_t pick = ((w >> (SH + 1)) & 0x04040404u) | 0x03020100u;
  return __builtin_amdgcn_perm(hi, lo, pick);
}

// Lane table of PPL subspace pairs: tab[s][0..3] even subspace 2p, [4..7] odd 2p+1.
template <int PPL>
struct LaneLut {
  uint32_t t[PPL][8];
};

template <int PPL>
__device__ __forceinline__ void load_lane_lut(LaneLut<PPL>& L, const uint8_t* lut, uint32_t npairs) {
  const int lane = lane_id();
#pragma unroll
  for (int s = 0; s < PPL; s++) {
    const uint32_t p = (uint32_t)lane + 64u * s;
    uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
    if (p < npairs) {
      const uint4* src = reinterpret_cast<const uint4*>(lut + (uint64_t)p * 32);
      a = src[0];
      b = src[1];
    }
#if !NGT_AMD_QG_VALU_REDUCE
    // table bytes as signed v - 128 for the i8 MFMA sum (adc_sum_mfma);
    // padding lanes stay 0 and contribute nothing
    if (p < npairs) {
      a.x ^= 0x80808080u; a.y ^= 0x80808080u; a.z ^= 0x80808080u; a.w ^= 0x80808080u;
      b.x ^= 0x80808080u; b.y ^= 0x80808080u; b.z ^= 0x80808080u; b.w ^= 0x80808080u;
    }
#endif
    L.t[s][0] = a.x; L.t[s][1] = a.y; L.t[s][2] = a.z; L.t[s][3] = a.w;
    L.t[s][4] = b.x; L.t[s][5] = b.y; L.t[s][6] = b.z; L.t[s][7] = b.w;
  }
}

// ---------------------------------------------------------------------------
// The cross-lane sum on the matrix cores.  A block's looked-up bytes sit
// lane = subspace pair, byte = object; the sum over subspaces is a sum over
// lanes.  One v_mfma_i32_16x16x64_i8 per subspace (even: e0..e3, odd:
// o0..o3) takes a lane's 16 looked-up bytes as its A fragment (row = lane &
// 15, k = the lane's 16 bytes within lane group lane >> 4) against a constant
// one-hot B whose byte t in column j is 1 iff byte t holds object j, so
// C[i][j] = sum over the four lanes {i, 16+i, 32+i, 48+i} of object j's
// bytes; A and B share the k map, so that map's details do not matter.  The
// 16 rows of C (4 registers x 4 lane groups) are then folded: three adds and
// two lane swaps.  The table bytes are stored as v ^ 0x80 = v - 128 (signed
// i8), so the exact int32 sum is S - 128 * Me; adc_epilogue_total adds it
// back.  Replaces the 16 packing v_perm and ~35 reduce-scatter ops per block.
typedef int qg_i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ qg_i32x4 qg_onehot_b() {
  const uint32_t j = (uint32_t)lane_id() & 15u;
  qg_i32x4 b;
#pragma unroll
  for (int d = 0; d < 4; d++) {
    uint32_t w = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      // dword d of (e0, e1, e2, e3): objects 2t, 2t + 1, 8 + 2t, 9 + 2t
      const uint32_t obj = (uint32_t)((d >> 1) * 8 + 2 * t + (d & 1));
      if (obj == j) w |= 1u << (8 * t);
    }
    b[d] = (int)w;
  }
  return b;
}

// The MFMA part for one block: returns this lane's sum of the four C
// registers (rows 4g..4g+3 of column lane & 15, g = lane >> 4).
template <int PPL>
__device__ __forceinline__ uint32_t adc_part_mfma(const LaneLut<PPL>& L, const uint4 (&c)[PPL], qg_i32x4 onehot,
                                                  uint32_t base) {
  qg_i32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < PPL; s++) {
    const uint32_t* t = L.t[s];
    qg_i32x4 ev, od;
    ev[0] = (int)lut16<0>(c[s].x, t[0], t[1], t[2], t[3], base);  // objects 0,2,4,6
    ev[1] = (int)lut16<4>(c[s].x, t[0], t[1], t[2], t[3], base);  // 1,3,5,7
    ev[2] = (int)lut16<0>(c[s].y, t[0], t[1], t[2], t[3], base);  // 8,...,14
    ev[3] = (int)lut16<4>(c[s].y, t[0], t[1], t[2], t[3], base);  // 9,...,15
    od[0] = (int)lut16<0>(c[s].z, t[4], t[5], t[6], t[7], base);
    od[1] = (int)lut16<4>(c[s].z, t[4], t[5], t[6], t[7], base);
    od[2] = (int)lut16<0>(c[s].w, t[4], t[5], t[6], t[7], base);
    od[3] = (int)lut16<4>(c[s].w, t[4], t[5], t[6], t[7], base);
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(ev, onehot, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(od, onehot, acc, 0, 0, 0);
  }
  return (uint32_t)(acc[0] + acc[1]) + (uint32_t)(acc[2] + acc[3]);
}

// Fold of four blocks' parts: lane group g (lane >> 4) ends with the signed
// sum of block g's object lane & 15 -- one epilogue serves four blocks.
__device__ __forceinline__ uint32_t fold4(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3) {
  const auto x = __builtin_amdgcn_permlane32_swap(p0, p2, false, false);  // lanes < 32 keep p0, else p2
  const auto y = __builtin_amdgcn_permlane32_swap(p1, p3, false, false);
  const uint32_t a = x[0] + x[1], b = y[0] + y[1];
  const auto z = __builtin_amdgcn_permlane16_swap(a, b, false, false);  // even rows keep a, odd rows b
  return z[0] + z[1];
}

// Single block: every lane ends with its object lane & 15.
template <int PPL>
__device__ __forceinline__ uint32_t adc_sum_mfma(const LaneLut<PPL>& L, const uint4 (&c)[PPL], qg_i32x4 onehot,
                                                 uint32_t base) {
  uint32_t r = adc_part_mfma<PPL>(L, c, onehot, base);
  {
    const auto x = __builtin_amdgcn_permlane32_swap(r, r, false, false);  // lane ^ 32
    r = x[0] + x[1];
  }
  {
    const auto x = __builtin_amdgcn_permlane16_swap(r, r, false, false);  // lane ^ 16
    r = x[0] + x[1];
  }
  return r;  // every lane: signed sum of object lane & 15
}

// sqrtf(fmaf(E + O, scale, totalOffset)) from the signed MFMA sum.
__device__ __forceinline__ float adc_epilogue_total(uint32_t ssum, uint32_t Me, float scale, float toff) {
  return sqrtf(__builtin_fmaf((float)(ssum + 128u * Me), scale, toff));
}

// Packed per-object partial sums of one lane for one block: v[o] =
// E(o) | O(o) << 16 over this lane's pairs.  c[s]: the 16 code bytes of pair s.
template <int PPL>
__device__ __forceinline__ void block_partials(const LaneLut<PPL>& L, const uint4 (&c)[PPL], uint32_t (&v)[16]) {
#pragma unroll
  for (int o = 0; o < 16; o++) v[o] = 0;
#pragma unroll
  for (int s = 0; s < PPL; s++) {
    const uint32_t* t = L.t[s];
    // even subspace: c.x = objects 0..7, c.y = 8..15 (low nibble = even object)
    const uint32_t e0 = lut16<0>(c[s].x, t[0], t[1], t[2], t[3]);  // objects 0,2,4,6
    const uint32_t e1 = lut16<4>(c[s].x, t[0], t[1], t[2], t[3]);  // 1,3,5,7
    const uint32_t e2 = lut16<0>(c[s].y, t[0], t[1], t[2], t[3]);  // 8,...,14
    const uint32_t e3 = lut16<4>(c[s].y, t[0], t[1], t[2], t[3]);  // 9,...,15
    const uint32_t o0 = lut16<0>(c[s].z, t[4], t[5], t[6], t[7]);
    const uint32_t o1 = lut16<4>(c[s].z, t[4], t[5], t[6], t[7]);
    const uint32_t o2 = lut16<0>(c[s].w, t[4], t[5], t[6], t[7]);
    const uint32_t o3 = lut16<4>(c[s].w, t[4], t[5], t[6], t[7]);
    // byte b of (e_k, o_k) -> (E | O << 16): selector {b, zero, 4 + b, zero}
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t sel = (uint32_t)b | (12u << 8) | ((4u + b) << 16) | (12u << 24);
      v[2 * b] += __builtin_amdgcn_perm(o0, e0, sel);
      v[2 * b + 1] += __builtin_amdgcn_perm(o1, e1, sel);
      v[8 + 2 * b] += __builtin_amdgcn_perm(o2, e2, sel);
      v[8 + 2 * b + 1] += __builtin_amdgcn_perm(o3, e3, sel);
    }
  }
}

// Reduce-scatter 16 per-lane values over the wave: on return every lane holds
// the full sum of object qg_obj_of_lane(lane).  No LDS traffic: the two
// cross-row stages are gfx950 v_permlane32_swap / v_permlane16_swap (lanes
// 32-63 of the first operand trade with lanes 0-31 of the second, resp. odd
// with even rows), so after one swap of (v[j], v[j+h]) both halves hold
// (own, partner) of the half they keep and a single add reduces it; the
// in-row stages are DPP (row_ror:8 = lane ^ 8, row_shl/shr:4 = lane ^ 4,
// quad_perm = lane ^ 2, lane ^ 1).
__device__ __forceinline__ uint32_t dpp_xor4(uint32_t x, bool up) {
  const uint32_t fwd = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x104, 0xf, 0xf, false);  // row_shl:4 (lane + 4)
  const uint32_t bwd = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xf, 0xf, false);  // row_shr:4 (lane - 4)
  return up ? bwd : fwd;
}

__device__ __forceinline__ uint32_t reduce_scatter16(uint32_t (&v)[16]) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < 8; j++) {  // lane bit 5: keep objects j (low half) or j + 8
    const auto r = __builtin_amdgcn_permlane32_swap(v[j], v[j + 8], false, false);
    v[j] = r[0] + r[1];
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {  // lane bit 4: keep j or j + 4
    const auto r = __builtin_amdgcn_permlane16_swap(v[j], v[j + 4], false, false);
    v[j] = r[0] + r[1];
  }
  {
    const bool hi = lane & 8;  // row_ror:8 pairs lane with lane ^ 8
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t send = hi ? v[j] : v[j + 2];
      const uint32_t keep = hi ? v[j + 2] : v[j];
      v[j] = keep + (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0x128, 0xf, 0xf, false);
    }
  }
  {
    const bool hi = lane & 4;
    const uint32_t send = hi ? v[0] : v[1];
    const uint32_t keep = hi ? v[1] : v[0];
    v[0] = keep + dpp_xor4(send, hi);
  }
  uint32_t r = v[0];
  r += (uint32_t)__builtin_amdgcn_mov_dpp((int)r, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  r += (uint32_t)__builtin_amdgcn_mov_dpp((int)r, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  return r;
}

__device__ __forceinline__ uint32_t qg_obj_of_lane(int lane) {
  return (((uint32_t)lane >> 5) & 1) << 3 | (((uint32_t)lane >> 4) & 1) << 2 |
         (((uint32_t)lane >> 3) & 1) << 1 | (((uint32_t)lane >> 2) & 1);
}

// sqrtf(fmaf(E + O, scale, totalOffset)) (Quantizer.h:1020-1031).  E and O
// are the saturating u16 sums; packed partials stay exact while
// Me/2 * 255 <= 65535 (Me <= 514), which the host enforces.
__device__ __forceinline__ float adc_epilogue(uint32_t packed, float scale, float toff) {
  const uint32_t e = packed & 0xffffu, o = packed >> 16;
  return sqrtf(__builtin_fmaf((float)(e + o), scale, toff));
}

// ADC of one node's neighbour list: nb blocks at `codes` (8*Me bytes each),
// distances of objects [0, n) into dists.  The loads of NBF blocks are issued
// before the first lookup.
template <int PPL>
__device__ __forceinline__ void adc_node(const LaneLut<PPL>& L, const uint8_t* codes, uint32_t Me, uint32_t n,
                                         float scale, float toff, float* dists) {
  const int lane = lane_id();
  const uint32_t npairs = Me >> 1;
  const uint32_t nb = n == 0 ? 0 : (n - 1) / 16 + 1;
  const uint64_t blk = (uint64_t)8 * Me;
  const qg_i32x4 onehot = qg_onehot_b();
  const uint32_t base = 0x03020100u;
  (void)onehot; (void)base;
  // blocks whose loads are in flight together (bounded by VGPRs)
  constexpr int NBF = PPL >= 4 ? 1 : (PPL == 2 ? 2 : 4);
  for (uint32_t b0 = 0; b0 < nb; b0 += NBF) {
    uint4 c[NBF][PPL];
#pragma unroll
    for (int j = 0; j < NBF; j++) {
#pragma unroll
      for (int s = 0; s < PPL; s++) {
        const uint32_t p = (uint32_t)lane + 64u * s;
        c[j][s] = make_uint4(0, 0, 0, 0);
        if (b0 + j < nb && p < npairs)
          c[j][s] = *reinterpret_cast<const uint4*>(codes + (b0 + j) * blk + (uint64_t)p * 16);
      }
    }
#pragma unroll
    for (int j = 0; j < NBF; j++) {
      if (b0 + j < nb) {
#if NGT_AMD_QG_VALU_REDUCE
        uint32_t v[16];
        block_partials<PPL>(L, c[j], v);
        const uint32_t r = reduce_scatter16(v);
        const uint32_t o = (b0 + j) * 16 + qg_obj_of_lane(lane);
        if ((lane & 3) == 0 && o < n) dists[o] = adc_epilogue(r, scale, toff);
#else
        const uint32_t r = adc_sum_mfma<PPL>(L, c[j], onehot, base);
        const uint32_t o = (b0 + j) * 16 + ((uint32_t)lane & 15u);
        if (lane < 16 && o < n) dists[o] = adc_epilogue_total(r, Me, scale, toff);
#endif
      }
    }
  }
}

// One expansion's neighbour ids and code blocks in a single memory round trip:
// the loads of the 0-terminated id row and of all `nbs` = id_stride/16 code
// blocks (<= NB) are issued together, before the degree is known; blocks past
// the degree are then skipped (their bytes were fetched for nothing, ~10 % of
// the code traffic at degree ~115 of 128, for one HBM latency less).
// Returns the degree; ids land in nid[0..id_stride), ADC distances in dists.
// With `probe` (HBM-epoch visited set behind an LDS filter of accepted ids),
// the epoch bytes of every neighbour whose filter bit is set are loaded as
// soon as the ids arrive, under the ADC arithmetic, and seen[c] returns the
// visited mask of id chunk c -- so the accept step needs no round trip of its
// own.  A clear filter bit proves an id unvisited (nothing loaded).
template <int PPL, int NB>
__device__ __forceinline__ uint32_t ids_and_adc(const LaneLut<PPL>& L, const uint32_t* nbr, uint32_t id_stride,
                                                const uint8_t* codes, uint32_t Me, float scale, float toff,
                                                uint32_t* nid, float* dists, bool probe, const SearchState& st,
                                                const uint8_t* vis, uint32_t epoch, uint64_t (&seen)[2]) {
  const int lane = lane_id();
  const uint32_t npairs = Me >> 1;
  const uint64_t blk = (uint64_t)8 * Me;
  const uint32_t nbs = id_stride >> 4;
  const qg_i32x4 onehot = qg_onehot_b();
  (void)onehot;
  uint4 c[NB][PPL];
#pragma unroll
  for (int j = 0; j < NB; j++) {
#pragma unroll
    for (int s = 0; s < PPL; s++) {
      const uint32_t p = (uint32_t)lane + 64u * s;
      c[j][s] = make_uint4(0, 0, 0, 0);
      if ((uint32_t)j < nbs && p < npairs)
        c[j][s] = *reinterpret_cast<const uint4*>(codes + (uint64_t)j * blk + (uint64_t)p * 16);
    }
  }
  static_assert(NB <= 8, "two 64-id chunks at most");
  constexpr int NC = (16 * NB + 63) / 64;
  uint32_t deg = 0;
  uint32_t idr[NC];
#pragma unroll
  for (int cc = 0; cc < NC; cc++) {
    const uint32_t j = 64u * cc;
    const uint32_t id = j + lane < id_stride ? nbr[j + lane] : 0u;
    idr[cc] = id;
    if (j < id_stride) nid[j + lane] = id;
    deg += (uint32_t)__popcll(ballot64(id != 0u));
  }
  bool pre[NC];
  uint32_t word[NC];
#pragma unroll
  for (int cc = 0; cc < NC; cc++) {
    pre[cc] = false;
    word[cc] = 0;
    if (probe && idr[cc] != 0u) {
      const uint32_t b = (idr[cc] * 0x85EBCA77u) >> st.vf_shift;
      pre[cc] = (st.vf[b >> 5] >> (b & 31)) & 1u;
      if (pre[cc])
        word[cc] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(vis + (idr[cc] & ~3u)), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const uint32_t nb = deg == 0 ? 0 : (deg - 1) / 16 + 1;
#if NGT_AMD_QG_VALU_REDUCE
#pragma unroll
  for (int j = 0; j < NB; j++) {
    if ((uint32_t)j < nb) {
      uint32_t v[16];
      block_partials<PPL>(L, c[j], v);
      const uint32_t r = reduce_scatter16(v);
      const uint32_t o = (uint32_t)j * 16 + qg_obj_of_lane(lane);
      if ((lane & 3) == 0 && o < deg) dists[o] = adc_epilogue(r, scale, toff);
    }
  }
#else
  // four blocks per fold and epilogue: lane group g writes block 4q + g
  const uint32_t base = 0x03020100u;
#pragma unroll
  for (int q = 0; q < (NB + 3) / 4; q++) {
    if ((uint32_t)(4 * q) < nb) {
      uint32_t part[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int j = 4 * q + u;
        part[u] = 0;
        if (j < NB && (uint32_t)j < nb) part[u] = adc_part_mfma<PPL>(L, c[j < NB ? j : 0], onehot, base);
      }
      const uint32_t r = fold4(part[0], part[1], part[2], part[3]);
      const uint32_t o = (uint32_t)(4 * q) * 16 + (uint32_t)lane;
      if (o < deg) dists[o] = adc_epilogue_total(r, Me, scale, toff);
    }
  }
#endif
  seen[0] = seen[1] = 0;
#pragma unroll
  for (int cc = 0; cc < NC; cc++)
    seen[cc] = ballot64(pre[cc] && ((word[cc] >> (8 * (idr[cc] & 3))) & 0xffu) == epoch);
  return deg;
}

// ids_and_adc over a packed record (the node's key word gave `rec` and its
// `nb` <= NB blocks): exactly the node's code blocks and 16*nb entries load
// together; nid / nkw receive the neighbour ids and key words.
template <int PPL, int NB>
__device__ __forceinline__ uint32_t ids_and_adc_packed(const LaneLut<PPL>& L, const uint8_t* rec, uint32_t nb,
                                                       uint32_t Me, float scale, float toff, uint32_t* nid,
                                                       uint32_t* nkw, float* dists, bool probe, const SearchState& st,
                                                       const uint8_t* vis, uint32_t epoch, float expr,
                                                       uint64_t (&seen)[2]) {
  const int lane = lane_id();
  const uint32_t npairs = Me >> 1;
  const uint64_t blk = (uint64_t)8 * Me;
  const qg_i32x4 onehot = qg_onehot_b();
  (void)onehot;
  uint4 c[NB][PPL];
#pragma unroll
  for (int j = 0; j < NB; j++) {
#pragma unroll
    for (int s = 0; s < PPL; s++) {
      const uint32_t p = (uint32_t)lane + 64u * s;
      c[j][s] = make_uint4(0, 0, 0, 0);
      if ((uint32_t)j < nb && p < npairs)
        c[j][s] = *reinterpret_cast<const uint4*>(rec + (uint64_t)j * blk + (uint64_t)p * 16);
    }
  }
  static_assert(NB <= 8, "two 64-id chunks at most");
  constexpr int NC = (16 * NB + 63) / 64;
  const uint2* ent = reinterpret_cast<const uint2*>(rec + (uint64_t)nb * blk);
  const uint32_t ne = 16 * nb;
  uint32_t deg = 0;
  uint32_t idr[NC];
#pragma unroll
  for (int cc = 0; cc < NC; cc++) {
    const uint32_t j = 64u * cc;
    const uint2 e = j + lane < ne ? ent[j + lane] : make_uint2(0u, 0u);
    idr[cc] = e.x;
    if (j < ne) {
      nid[j + lane] = e.x;
      nkw[j + lane] = e.y;
    }
    deg += (uint32_t)__popcll(ballot64(e.x != 0u));
  }
  const uint32_t nbd = deg == 0 ? 0 : (deg - 1) / 16 + 1;
  // lane l's entries' ADC distances (entry 64 * cc + l)
  float dv[NC];
#pragma unroll
  for (int cc = 0; cc < NC; cc++) dv[cc] = __int_as_float(0x7f800000);
#if NGT_AMD_QG_VALU_REDUCE
#pragma unroll
  for (int j = 0; j < NB; j++) {
    if ((uint32_t)j < nbd) {
      uint32_t v[16];
      block_partials<PPL>(L, c[j], v);
      const uint32_t r = reduce_scatter16(v);
      const uint32_t o = (uint32_t)j * 16 + qg_obj_of_lane(lane);
      if ((lane & 3) == 0 && o < deg) dists[o] = adc_epilogue(r, scale, toff);
    }
  }
  __syncthreads();
#pragma unroll
  for (int cc = 0; cc < NC; cc++)
    if (64u * cc + lane < deg) dv[cc] = dists[64u * cc + lane];
#else
  const uint32_t base = 0x03020100u;
  static_assert((NB + 3) / 4 == NC, "ADC pass q covers entries 64q..64q+63");
#pragma unroll
  for (int q = 0; q < (NB + 3) / 4; q++) {
    if ((uint32_t)(4 * q) < nbd) {
      uint32_t part[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int j = 4 * q + u;
        part[u] = 0;
        if (j < NB && (uint32_t)j < nbd) part[u] = adc_part_mfma<PPL>(L, c[j < NB ? j : 0], onehot, base);
      }
      const uint32_t r = fold4(part[0], part[1], part[2], part[3]);
      const uint32_t o = (uint32_t)(4 * q) * 16 + (uint32_t)lane;
      if (o < deg) {
        dv[q] = adc_epilogue_total(r, Me, scale, toff);
        dists[o] = dv[q];
      }
    }
  }
#endif
  // the visited probe, after the ADC: only an entry within the exploration
  // radius can be accepted (the accept step tests `d <= expr` with an expr
  // that only shrinks), so only those whose filter bit is set read their
  // epoch word -- the others' seen bits are never looked at
  bool pre[NC];
  uint32_t word[NC];
#pragma unroll
  for (int cc = 0; cc < NC; cc++) {
    pre[cc] = false;
    word[cc] = 0;
    if (probe && idr[cc] != 0u && dv[cc] <= expr) {
      const uint32_t b = (idr[cc] * 0x85EBCA77u) >> st.vf_shift;
      pre[cc] = (st.vf[b >> 5] >> (b & 31)) & 1u;
      if (pre[cc])
        word[cc] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(vis + (idr[cc] & ~3u)), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  seen[0] = seen[1] = 0;
#pragma unroll
  for (int cc = 0; cc < NC; cc++)
    seen[cc] = ballot64(pre[cc] && ((word[cc] >> (8 * (idr[cc] & 3))) & 0xffu) == epoch);
  return deg;
}

// Standalone ADC: wave per (query, node) pair; out[i*out_stride + j] for the
// node's neighbours j (full list, the QG loop's call at QuantizedGraph.h:240).
template <int PPL>
__global__ void __launch_bounds__(64) ngt_qg_adc_kernel(QgAdcArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float* dd = reinterpret_cast<float*>(smem);
  const int lane = lane_id();
  for (uint32_t i = blockIdx.x; i < a.npairs; i += gridDim.x) {
    const uint32_t qi = a.qidx[i], v = a.node[i];
    LaneLut<PPL> L;
    load_lane_lut<PPL>(L, a.lut + (uint64_t)qi * a.lut_stride, a.Me >> 1);
    const uint32_t* ids = a.qids + (uint64_t)v * a.id_stride;
    uint32_t n = 0;
    for (uint32_t j = 0; j < a.id_stride; j += 64)
      n += (uint32_t)__popcll(ballot64(j + lane < a.id_stride && ids[j + lane] != 0u));
    adc_node<PPL>(L, a.qcodes + (uint64_t)v * a.code_stride, a.Me, n, a.scale[qi], a.toff[qi], dd);
    __syncthreads();
    for (uint32_t j = lane; j < n; j += 64) a.out[(uint64_t)i * a.out_stride + j] = dd[j];
    if (lane == 0) a.out_n[i] = n;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Quantized-graph search: one wave per query, persistent over a work counter.
// ---------------------------------------------------------------------------
// Visited test without insertion (the QG loop tests before it marks).
__device__ __forceinline__ bool visited_test(uint32_t ht_log2, const SearchState& st, uint32_t id, bool vis_mode,
                                             const uint8_t* vis, uint32_t epoch) {
  const uint32_t* ht = st.ht;
  if (vis_mode) {
    // a clear filter bit proves the id unvisited (see visit())
    if (st.vf) {
      const uint32_t b = (id * 0x85EBCA77u) >> st.vf_shift;
      if (!((st.vf[b >> 5] >> (b & 31)) & 1u)) return false;
    }
    // the LDS table doubles as a cache of visited ids (see visit())
    if (ht_log2 && ht[ht_hash(id, 32 - ht_log2)] == id) return true;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(vis + (id & ~3u));
    const uint32_t word = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return ((word >> (8 * (id & 3))) & 0xffu) == epoch;
  }
  const uint32_t mask = (1u << ht_log2) - 1;
  uint32_t h = ht_hash(id, 32 - ht_log2);
  for (;;) {
    const uint32_t old = ht[h];
    if (old == 0u) return false;
    if (old == id) return true;
    h = (h + 1) & mask;
  }
}

template <int PPL, int NCH>
__device__ __forceinline__ void qg_exact(const float* qlds, const QgSearchArgs& a, const uint32_t* ids, float* dists,
                                         int m) {
  if constexpr (NCH > 0) {
    eval_l2f_fast<NCH, 1>(qlds, a.rows, a.row_bytes, ids, dists, m);
  } else {
    eval_batch<kL2, float>(qlds, a.rows, a.row_bytes, a.dp, ids, dists, m);
  }
}

// NB > 0: id rows of up to 16*NB entries load together with all their code
// blocks (ids_and_adc); NB = 0: ids, then the codes of the degree read.
#ifndef NGT_AMD_QG_WPE
#define NGT_AMD_QG_WPE 4  // waves per SIMD (a build-time A/B choice)
#endif
template <int PPL, int NCH, int NB>
__global__ void __launch_bounds__(64, NGT_AMD_QG_WPE) ngt_qg_search_kernel(QgSearchArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = lane_id();
  SearchState st;
  uint8_t* p = smem;
  const bool use_hash = a.ht_log2 != 0;
  st.ht = reinterpret_cast<uint32_t*>(p);
  if (use_hash) p += (size_t)4 << a.ht_log2;
  st.vf = a.vf_log2 ? reinterpret_cast<uint32_t*>(p) : nullptr;
  st.vf_shift = 32 - a.vf_log2;
  const uint32_t vf_words = a.vf_log2 ? (1u << a.vf_log2) / 32 : 0u;
  p += (size_t)4 * vf_words;
  st.cq = reinterpret_cast<uint64_t*>(p);
  p += (size_t)8 * a.cq_cap;
  st.res = reinterpret_cast<uint64_t*>(p);
  p += ((size_t)8 * (a.size + 1) + 15) & ~(size_t)15;
  uint64_t* rr = reinterpret_cast<uint64_t*>(p);  // rerank order
  p += ((size_t)8 * (a.size + 1) + 15) & ~(size_t)15;
  const uint32_t nstage = a.id_stride > a.size ? a.id_stride : a.size;
  const uint32_t nstage64 = (nstage + 63) & ~63u;
  st.nid = reinterpret_cast<uint32_t*>(p);
  p += (size_t)4 * nstage64;
  st.nd = reinterpret_cast<float*>(p);
  p += (size_t)4 * nstage64;
  uint32_t* nkw = reinterpret_cast<uint32_t*>(p);  // packed layout: the neighbours' key words
  p += (size_t)4 * nstage64;
  uint32_t* hist = reinterpret_cast<uint32_t*>(p);  // threshold selection: 64 counters, then 64 staged keys
  p += 256 + 512;
  float* qlds = reinterpret_cast<float*>(p);
  const bool packed = a.recs != nullptr;

  const uint32_t slot = blockIdx.x;
  uint8_t* vis = a.vis + (uint64_t)slot * a.vis_stride;
  uint64_t* spill = a.spill + (uint64_t)slot * a.spill_cap;  // the unchecked set's HBM level
  const uint32_t hcap = use_hash ? 1u << a.ht_log2 : 0u;
  const uint32_t hlimit = hcap - (hcap >> 2);
  const uint32_t npairs = a.Me >> 1;

  for (;;) {
    uint32_t qi = 0;
    if (lane == 0) qi = atomicAdd(a.work, 1u);
    qi = __shfl(qi, 0, 64);
    if (qi >= a.nq) break;

    for (uint32_t i = lane; i < hcap; i += 64) st.ht[i] = 0u;
    for (uint32_t i = lane; i < vf_words; i += 64) st.vf[i] = 0u;
    load_query<float>(qlds, a.queries + (uint64_t)qi * a.query_bytes, a.dp);
    LaneLut<PPL> L;
    load_lane_lut<PPL>(L, a.lut + (uint64_t)qi * a.lut_stride, npairs);
    const float scale = a.scale[qi], toff = a.toff[qi];
    uint32_t epoch = a.slot_epoch[slot] + 1;
    if (epoch > 255) {
      uint4* v4 = reinterpret_cast<uint4*>(vis);
      for (uint64_t i = lane; i < a.vis_stride / 16; i += 64) v4[i] = make_uint4(0, 0, 0, 0);
      epoch = 1;
    }
    __syncthreads();
    if (lane == 0) a.slot_epoch[slot] = epoch;

    bool bitmap_mode = !use_hash;
    uint32_t nvisited = 0, nres = 0, maxq = 0;
    uint64_t nadc = 0, nacc = 0, nexp = 0, nexact = 0, nblk = 0;
    uint64_t t_pop = 0, t_ids = 0, t_adc = 0, t_acc = 0, t_last = 0;
    (void)t_pop; (void)t_ids; (void)t_adc; (void)t_acc; (void)t_last;
    const uint32_t size = a.size;
    float radius = a.radius;
    float expr = __fmul_rn(a.coef, radius);

    // ---- the unchecked set: a sorted head of the 64 smallest keys in
    // registers (lane i = i-th smallest, hn keys) < B <= an unsorted LDS tail
    // (st.cq, ntail keys) < T <= an HBM spill (nspill keys) -- the latency
    // kernel's form (search_lat.hip), so a pop is a lane shift and never scans
    // anything: a quantized graph over 12.5M objects keeps ~40k unchecked keys
    // per query, and the chunk-minimum scans of a flat spill were most of its
    // expansions' time.  Exact throughout; keys beyond the exploration radius
    // are dropped when the tail fills (they can never be popped,
    // QuantizedGraph.h:226-229 / Graph.cpp:433-435).
    uint64_t hk = ~0ull, B = ~0ull, T = ~0ull;
    uint32_t hn = 0, ntail = 0, nspill = 0;
    uint64_t* tail = st.cq;
    uint32_t ntrim = 0;  // spill trims (counter 7)
    // a full spill first drops its keys beyond the exploration radius (they
    // can never be popped: expr only shrinks); the capacity error is left for
    // a spill still full of keys within it
    auto spill_trim = [&]() {
      const uint64_t lim = ((uint64_t)ord_of(expr) << 32) | 0xffffffffull;
      uint32_t out = 0;
      for (uint32_t b0 = 0; b0 < nspill; b0 += 64) {
        const uint32_t i = b0 + (uint32_t)lane;
        const uint64_t key = i < nspill ? spill[i] : ~0ull;
        const bool kp = i < nspill && key <= lim;
        const uint64_t km = ballot64(kp);
        __builtin_amdgcn_wave_barrier();
        if (kp) spill[out + mbcnt(km)] = key;
        __builtin_amdgcn_wave_barrier();
        out += (uint32_t)__popcll(km);
      }
      nspill = out;
      ntrim++;
    };
    auto spill_push = [&](uint64_t key) {
      if (nspill >= a.spill_cap) spill_trim();
      if (nspill >= a.spill_cap) {
        if (lane == 0) atomicOr(a.error, 1);
      } else {
        if (lane == 0) spill[nspill] = key;
        nspill++;
      }
    };
    auto tail_room = [&]() {
      uint32_t out = 0;
      for (uint32_t b0 = 0; b0 < ntail; b0 += 64) {
        const uint32_t i = b0 + (uint32_t)lane;
        const uint64_t key = i < ntail ? tail[i] : ~0ull;
        const bool keep = i < ntail && key_dist(key) <= expr;
        const uint64_t km = ballot64(keep);
        __builtin_amdgcn_wave_barrier();
        if (keep) tail[out + mbcnt(km)] = key;
        __builtin_amdgcn_wave_barrier();
        out += (uint32_t)__popcll(km);
      }
      ntail = out;
      const uint32_t keep = a.cq_cap / 2;
      if (ntail <= keep) return;
      const uint64_t l = lat_select(tail, ntail, keep, ~0ull, hist);
      out = 0;
      for (uint32_t b0 = 0; b0 < ntail; b0 += 64) {
        const uint32_t i = b0 + (uint32_t)lane;
        const uint64_t key = i < ntail ? tail[i] : ~0ull;
        const bool mv = i < ntail && key >= l;
        const bool kp = i < ntail && key < l;
        const uint64_t mm = ballot64(mv), km = ballot64(kp);
        const uint32_t nm = (uint32_t)__popcll(mm);
        if (nspill + nm > a.spill_cap) spill_trim();
        if (nspill + nm > a.spill_cap) {
          if (lane == 0) atomicOr(a.error, 1);
        } else if (mv) {
          spill[nspill + mbcnt(mm)] = key;
        }
        if (nspill + nm <= a.spill_cap) nspill += nm;
        __builtin_amdgcn_wave_barrier();
        if (kp) tail[out + mbcnt(km)] = key;
        __builtin_amdgcn_wave_barrier();
        out += (uint32_t)__popcll(km);
      }
      if ((out == 0u || out > keep) && lane == 0) atomicOr(a.error, 32);  // selection check
      ntail = out;
      T = l;
    };
    auto tail_push = [&](uint64_t key) {
      if (key >= T) {
        spill_push(key);
      } else {
        if (ntail >= a.cq_cap) tail_room();
        if (key >= T) {
          spill_push(key);
        } else {
          if (lane == 0) tail[ntail] = key;
          ntail++;
        }
      }
      __builtin_amdgcn_wave_barrier();
    };
    auto insert_key = [&](uint64_t key) {
      if (key < B) {
        const uint32_t pos = (uint32_t)__popcll(ballot64((uint32_t)lane < hn && hk < key));
        if (hn == 64u) {
          // the head is full: its largest key (or this one) moves to the tail
          if (pos == 64u) {
            B = key;
            tail_push(key);
          } else {
            const uint64_t e = readlane_u64(hk, 63);
            const uint64_t uk = wave_up1_u64(hk);
            if ((uint32_t)lane > pos) hk = uk;
            if ((uint32_t)lane == pos) hk = key;
            B = e;
            tail_push(e);
          }
        } else {
          const uint64_t uk = wave_up1_u64(hk);
          if ((uint32_t)lane > pos && (uint32_t)lane <= hn) hk = uk;
          if ((uint32_t)lane == pos) hk = key;
          hn++;
        }
      } else {
        tail_push(key);
      }
      const uint32_t q = hn + ntail + nspill;
      if (q > maxq) maxq = q;
    };
    // an empty tail takes the smallest spill keys within the radius (the ones
    // beyond it are dropped)
    auto refill_tail = [&]() {
      const uint32_t want = a.cq_cap / 2;
      const uint64_t lim = ((uint64_t)ord_of(expr) << 32) | 0xffffffffull;
      const uint64_t l = lat_select(spill, nspill, want, lim, hist);
      if (l == 0ull) {  // nothing within the radius: the search ends
        nspill = 0;
        T = ~0ull;
        return;
      }
      uint32_t out = 0;
      for (uint32_t b0 = 0; b0 < nspill; b0 += 64) {
        const uint32_t i = b0 + (uint32_t)lane;
        const uint64_t key = i < nspill ? spill[i] : ~0ull;
        const bool in = i < nspill && key <= lim;
        const bool mv = in && key < l;
        const bool sy = in && !mv;
        const uint64_t mm = ballot64(mv), sm = ballot64(sy);
        __builtin_amdgcn_wave_barrier();
        if (mv) tail[ntail + mbcnt(mm)] = key;
        if (sy) spill[out + mbcnt(sm)] = key;
        __builtin_amdgcn_wave_barrier();
        ntail += (uint32_t)__popcll(mm);
        out += (uint32_t)__popcll(sm);
      }
      nspill = out;
      T = nspill ? l : ~0ull;
      if ((ntail == 0u || ntail > want) && lane == 0) atomicOr(a.error, 64);  // selection check
    };
    // an empty head takes the (at most 64) smallest tail keys, sorted across
    // the lanes by a bitonic network
    auto refill_head = [&]() {
      if (ntail == 0 && nspill != 0) refill_tail();
      if (ntail == 0) return;
      const uint64_t t = lat_select(tail, ntail, 64u, ~0ull, hist);
      uint64_t* st64 = reinterpret_cast<uint64_t*>(hist + 64);  // 64 staged keys
      uint32_t got = 0, out = 0;
      for (uint32_t b0 = 0; b0 < ntail; b0 += 64) {
        const uint32_t i = b0 + (uint32_t)lane;
        const uint64_t key = i < ntail ? tail[i] : ~0ull;
        const bool mv = i < ntail && key < t;
        const bool kp = i < ntail && !mv;
        const uint64_t mm = ballot64(mv), km = ballot64(kp);
        __builtin_amdgcn_wave_barrier();
        if (mv) st64[got + mbcnt(mm)] = key;
        if (kp) tail[out + mbcnt(km)] = key;
        __builtin_amdgcn_wave_barrier();
        got += (uint32_t)__popcll(mm);
        out += (uint32_t)__popcll(km);
      }
      uint64_t v = (uint32_t)lane < got ? st64[lane] : ~0ull;
      ntail = out;
      if ((got == 0u || got > 64u) && lane == 0) atomicOr(a.error, 128);  // selection check
#pragma unroll
      for (int kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
          const uint64_t o = shfl_xor_u64(v, j);
          const bool up = ((lane & kk) == 0);
          const bool lower = (lane & j) == 0;
          const uint64_t mn = o < v ? o : v, mx = o < v ? v : o;
          v = (lower == up) ? mn : mx;
        }
      }
      hk = v;
      hn = got;
      B = (ntail + nspill) ? readlane_u64(hk, (int)got - 1) + 1 : ~0ull;
      __builtin_amdgcn_wave_barrier();
    };
    auto pop = [&](uint64_t& key) -> bool {
      if (hn == 0) refill_head();
      if (hn == 0) return false;
      key = readlane_u64(hk, 0);
      const uint64_t dk = wave_down1_u64(hk);
      hk = (uint32_t)lane < hn - 1 ? dk : ~0ull;
      hn--;
      return true;
    };

    // ---- setupDistances (exact L2) + setupSeeds (Graph.cpp:293-367) -------
    const uint64_t sb = a.seed_off ? a.seed_off[qi] : (uint64_t)qi * a.seed_stride;
    const uint32_t ns = a.seed_off ? (uint32_t)(a.seed_off[qi + 1] - sb) : a.seed_count[qi];
    for (uint32_t base = 0; base < ns; base += 64) {
      const uint32_t m = ns - base < 64 ? ns - base : 64;
      if ((uint32_t)lane < m) st.nid[lane] = a.seeds[sb + base + lane];
      __syncthreads();
      qg_exact<PPL, NCH>(qlds, a, st.nid, st.nd, (int)m);
      __syncthreads();
      if ((uint32_t)lane < m) visit(a.ht_log2, st, st.nid[lane], bitmap_mode, vis, epoch);
      __syncthreads();
      for (uint32_t j = 0; j < m; j++) {
        const float d = st.nd[j];
        const uint32_t id = st.nid[j];
        insert_key(make_key(d, packed ? a.qkw[id] : id));
        if (d <= a.radius) res_insert(st.res, nres, size, make_key(d, id));
      }
      nexact += m;
      nvisited += m;
      __syncthreads();
      if (!bitmap_mode && nvisited > hlimit) {
        ht_to_vis(a.ht_log2, st, vis, epoch);
        bitmap_mode = true;
        __syncthreads();
      }
    }
    if (nres >= size) radius = key_dist(st.res[size - 1]);
    expr = __fmul_rn(a.coef, radius);

    // ---- best-first loop over ADC distances (QuantizedGraph.h:220-268) ----
#ifdef NGT_AMD_STAMPS
    t_last = stamp();
#endif
    for (;;) {
      uint64_t wbest;
      if (!pop(wbest)) break;
      if (key_dist(wbest) > expr) break;
      nexp++;
      NGT_MARK(t_pop);

      // neighbour ids (0-terminated fixed-stride row) and their ADC distances
      const uint32_t target = key_id(wbest);  // the node id, or its key word in the packed layout
      const uint32_t* nbr = a.qids + (uint64_t)target * a.id_stride;
      uint32_t deg = 0;
      uint64_t seen_pre[2] = {0, 0};
      const bool early = NB > 0 && a.id_stride <= 16u * NB;
      const bool probe = early && !use_hash && st.vf != nullptr;
      if (packed) {
        // the key word names the record and its block count (qg_api.cpp qg_pack)
        const uint8_t* rec = a.recs + ((uint64_t)(target >> 3) << a.rec_shift);
        deg = ids_and_adc_packed<PPL, (NB > 0 ? NB : 1)>(L, rec, (target & 7u) + 1u, a.Me, scale, toff, st.nid, nkw,
                                                         st.nd, !use_hash && st.vf != nullptr, st, vis, epoch,
                                                         expr, seen_pre);
        NGT_MARK(t_ids);
      } else if (early) {
        deg = ids_and_adc<PPL, (NB > 0 ? NB : 1)>(L, nbr, a.id_stride, a.qcodes + (uint64_t)target * a.code_stride,
                                                  a.Me, scale, toff, st.nid, st.nd, probe, st, vis, epoch, seen_pre);
        NGT_MARK(t_ids);
      } else {
        for (uint32_t j = 0; j < a.id_stride; j += 64) {
          const uint32_t id = j + lane < a.id_stride ? nbr[j + lane] : 0u;
          st.nid[j + lane] = id;
          deg += (uint32_t)__popcll(ballot64(id != 0u));
        }
        NGT_MARK(t_ids);
        adc_node<PPL>(L, a.qcodes + (uint64_t)target * a.code_stride, a.Me, deg, scale, toff, st.nd);
      }
      __syncthreads();
      NGT_MARK(t_adc);
      nadc += deg;
      nblk += deg == 0 ? 0 : (deg - 1) / 16 + 1;

      // accept in neighbour order (QuantizedGraph.h:241-266): ids of one list
      // are distinct, so the visited test of a chunk runs in parallel and only
      // the radius bookkeeping is sequential.
      for (uint32_t base = 0; base < deg; base += 64) {
        const uint32_t i = base + lane;
        const bool in = i < deg && st.nd[i] <= expr;
        const bool pre_probed = packed ? (!use_hash && st.vf != nullptr) : probe;
        const bool seen = in && (pre_probed ? ((((base == 0) ? seen_pre[0] : seen_pre[1]) >> lane) & 1ull) != 0
                                            : visited_test(a.ht_log2, st, st.nid[i], bitmap_mode, vis, epoch));
        uint64_t cand = ballot64(in && !seen);
        uint64_t acc = 0;
        while (cand) {
          const int j = __ffsll((long long)cand) - 1;
          cand &= cand - 1;
          const float d = st.nd[base + j];
          if (!(d <= expr)) continue;
          acc |= 1ull << j;
          // results by (distance, id); the unchecked set by (distance, key
          // word) in the packed layout -- the same order
          const uint64_t rkey = make_key(d, st.nid[base + j]);
          insert_key(packed ? make_key(d, nkw[base + j]) : rkey);
          if (d <= radius) {
            res_insert(st.res, nres, size, rkey);
            if (nres >= size) {
              radius = key_dist(st.res[size - 1]);
              expr = __fmul_rn(a.coef, radius);
            }
          }
          __builtin_amdgcn_wave_barrier();
        }
        // mark the accepted ids
        if ((acc >> lane) & 1ull) visit(a.ht_log2, st, st.nid[i], bitmap_mode, vis, epoch);
        const uint32_t na = (uint32_t)__popcll(acc);
        nacc += na;
        nvisited += na;
        __syncthreads();
        if (!bitmap_mode && nvisited > hlimit) {
          ht_to_vis(a.ht_log2, st, vis, epoch);
          bitmap_mode = true;
          __syncthreads();
        }
      }
      NGT_MARK(t_acc);
    }

    // ---- results (QuantizedGraph.h:270-299) ------------------------------
    uint32_t nout = nres;
    if (a.rerank) {
      // exact distances of the expanded result set, sorted by (distance, id),
      // resized to k (padding {0, 0} when short)
      for (uint32_t base = 0; base < nres; base += 64) {
        const uint32_t m = nres - base < 64 ? nres - base : 64;
        if ((uint32_t)lane < m) st.nid[lane] = key_id(st.res[base + lane]);
        __syncthreads();
        qg_exact<PPL, NCH>(qlds, a, st.nid, st.nd, (int)m);
        __syncthreads();
        if ((uint32_t)lane < m) rr[base + lane] = make_key(st.nd[lane], st.nid[lane]);
        __syncthreads();
      }
      nexact += nres;
      // rank sort: position of each key = number of smaller keys (distinct ids)
      for (uint32_t i = lane; i < nres; i += 64) {
        const uint64_t key = rr[i];
        uint32_t pos = 0;
        for (uint32_t j = 0; j < nres; j++) pos += rr[j] < key ? 1u : 0u;
        st.res[pos] = key;
      }
      __syncthreads();
      for (uint32_t i = lane; i < a.k; i += 64) {
        a.out_ids[(uint64_t)qi * a.k + i] = i < nres ? key_id(st.res[i]) : 0u;
        a.out_dists[(uint64_t)qi * a.k + i] = i < nres ? key_dist(st.res[i]) : 0.0f;
      }
      nout = a.k;
    } else {
      for (uint32_t i = lane; i < nres; i += 64) {
        a.out_ids[(uint64_t)qi * a.k + i] = key_id(st.res[i]);
        a.out_dists[(uint64_t)qi * a.k + i] = key_dist(st.res[i]);
      }
    }
    if (lane == 0) {
      a.out_n[qi] = nout;
      if (a.counters) {
        uint64_t* c = a.counters + (uint64_t)qi * 8;
        c[0] = nadc;
        c[1] = nacc;
        c[2] = nexp;
        c[3] = nexact;
        c[4] = nblk;
        c[5] = maxq;
        c[6] = (bitmap_mode && use_hash) ? 1 : 0;
        c[7] = ntrim;
#ifdef NGT_AMD_STAMPS
        c[4] = t_pop;
        c[5] = t_ids;
        c[6] = t_adc;
        c[7] = t_acc;
#endif
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Launchers.
// ---------------------------------------------------------------------------
static int ppl_of(uint32_t Me) {
  const uint32_t pairs = Me / 2;
  if (pairs <= 64) return 1;
  if (pairs <= 128) return 2;
  if (pairs <= 256) return 4;  // Me <= 512 keeps the packed u16 sums exact
  return 0;
}

hipError_t launch_qg_lut(const QgLutArgs& a, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const size_t lds = (size_t)a.M * 16 * sizeof(float);
  const uint32_t blocks = a.nq < 16384 ? a.nq : 16384;
  hipLaunchKernelGGL(ngt_qg_lut_kernel, dim3(blocks), dim3(64), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_qg_build(const QgBuildArgs& a, hipStream_t s) {
  if (a.nrows == 0) return hipSuccess;
  uint64_t blocks = ((uint64_t)a.nrows + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(ngt_qg_build_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_qg_encode(const QgEncodeArgs& a, hipStream_t s) {
  if (a.nrows == 0) return hipSuccess;
  if (a.dsub == 0 || a.dsub > 16) return hipErrorInvalidValue;
  uint64_t blocks = (a.nrows * a.M + 255) / 256;
  if (blocks > 262144) blocks = 262144;
  hipLaunchKernelGGL(ngt_qg_encode_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_qg_train(const QgTrainArgs& a, hipStream_t s) {
  if (a.dsub == 0 || a.dsub > 16 || a.nsample < 16) return hipErrorInvalidValue;
  const size_t lds = ((size_t)a.nsample * a.dsub + 16 * a.dsub + a.nsample) * sizeof(float) + a.nsample;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ngt_qg_train_kernel, dim3(a.M), dim3(256), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_qg_adc(const QgAdcArgs& a, hipStream_t s) {
  if (a.npairs == 0) return hipSuccess;
  const size_t lds = (size_t)((a.id_stride + 63) & ~63u) * sizeof(float);
  const uint32_t blocks = a.npairs < 65536 ? (uint32_t)a.npairs : 65536;
  switch (ppl_of(a.Me)) {
    case 1: hipLaunchKernelGGL((ngt_qg_adc_kernel<1>), dim3(blocks), dim3(64), lds, s, a); break;
    case 2: hipLaunchKernelGGL((ngt_qg_adc_kernel<2>), dim3(blocks), dim3(64), lds, s, a); break;
    case 4: hipLaunchKernelGGL((ngt_qg_adc_kernel<4>), dim3(blocks), dim3(64), lds, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

size_t qg_search_lds_bytes(const QgSearchArgs& a) {
  size_t b = (a.ht_log2 ? ((size_t)4 << a.ht_log2) : 0) + (size_t)8 * a.cq_cap;
  b += a.vf_log2 ? ((size_t)1 << a.vf_log2) / 8 : 0;
  b += 2 * (((size_t)8 * (a.size + 1) + 15) & ~(size_t)15);
  const uint32_t nstage = a.id_stride > a.size ? a.id_stride : a.size;
  b += (size_t)12 * ((nstage + 63) & ~63u);
  b += 256 + 512;  // threshold-selection counters and staged keys
  b += (size_t)a.dp * 4;
  return b;
}

hipError_t launch_qg_blocks(const uint32_t* qids, uint32_t id_stride, uint32_t nrows, uint8_t* nb, hipStream_t s) {
  if (nrows == 0) return hipSuccess;
  uint64_t blocks = ((uint64_t)nrows + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(ngt_qg_blocks_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, qids, id_stride, nrows, nb);
  return hipGetLastError();
}

hipError_t launch_qg_pack(const uint32_t* qids, uint32_t id_stride, const uint8_t* qcodes, uint64_t code_stride,
                          uint32_t Me, uint32_t nrows, const uint32_t* qkw, uint32_t rec_shift, uint8_t* recs,
                          hipStream_t s) {
  if (nrows < 2) return hipSuccess;
  uint64_t blocks = ((uint64_t)nrows + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(ngt_qg_pack_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, qids, id_stride, qcodes,
                     code_stride, Me, nrows, qkw, rec_shift, recs);
  return hipGetLastError();
}

hipError_t launch_qg_search(const QgSearchArgs& a, uint32_t slots, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  const size_t lds = qg_search_lds_bytes(a);
#define L_QG(P, N, B) hipLaunchKernelGGL((ngt_qg_search_kernel<P, N, B>), dim3(slots), dim3(64), lds, s, a)
  const int ppl = ppl_of(a.Me);
  if (a.dp == 128) {
    switch (ppl) {
      case 1: L_QG(1, 8, 8); break;
      case 2: L_QG(2, 8, 4); break;
      case 4: L_QG(4, 8, 0); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (ppl) {
      case 1: L_QG(1, 0, 8); break;
      case 2: L_QG(2, 0, 4); break;
      case 4: L_QG(4, 0, 0); break;
      default: return hipErrorInvalidValue;
    }
  }
#undef L_QG
  return hipGetLastError();
}

}  // namespace ngt_amd
