// ngt_kernels.h -- argument blocks and launchers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "knobs.h"

namespace ngt_amd {

struct DistanceArgs {
  const uint8_t* rows;     // padded object rows, row_bytes apart (row 0 = dummy)
  uint64_t row_bytes;
  const uint8_t* queries;  // padded query rows, query_bytes apart
  uint64_t query_bytes;
  const uint32_t* qidx;    // per pair: query index
  const uint32_t* oid;     // per pair: object id
  float* out;
  uint64_t npairs;
  int dp;                  // padded dimension (elements)
};

struct TreeSeedArgs {
  const uint8_t* queries;
  uint64_t query_bytes;
  uint32_t nq;
  int dp;
  uint64_t row_bytes;            // pivot row stride
  const uint8_t* in_pivot;       // [n_internal][row_bytes]
  const uint32_t* in_child;      // [n_internal][children] raw Node::ID
  const float* in_border;        // [n_internal][children-1]
  uint32_t children;
  uint32_t root;                 // raw Node::ID of the root
  const uint64_t* leaf_off;      // [n_leaf+1] (CSR leaves), or
  const uint32_t* leaf_count;    // [n_leaf] with leaf j's ids at leaf_ids + j * leaf_stride
  uint32_t leaf_stride;
  const uint32_t* leaf_ids;
  uint32_t seed_size;            // property.seedSize (0 => k)
  uint32_t k;
  int all_leaf_nodes;            // sc.useAllNodesInLeaf / SeedTypeAllLeafNodes
  uint32_t* seeds;               // [nq][seed_stride]
  uint32_t seed_stride;
  uint32_t* seed_count;          // [nq]
  uint32_t* tree_ndist;          // [nq] or null
  // construction only (all null otherwise): the leaf each query descends to,
  // its object count, and the distance to its pivot when the count is > 0
  uint32_t* out_leaf;            // [nq]
  uint32_t* out_count;           // [nq]
  float* out_pdist;              // [nq]
  const uint8_t* leaf_pivot;     // [n_leaf][row_bytes]
};

struct SearchArgs {
  const uint8_t* rows;
  uint64_t row_bytes;
  uint32_t nrows;
  int dp;
  const uint64_t* edge_off;      // CSR [nrows+1]
  const uint32_t* edges;
  const uint32_t* adj;           // optional padded adjacency [nrows][adj_stride], 0-terminated
  uint64_t adj_stride;
  const uint8_t* queries;
  uint64_t query_bytes;
  uint32_t nq;
  // seeds: either CSR (seed_off != null) or fixed stride + counts
  const uint32_t* seeds;
  const uint64_t* seed_off;
  uint32_t seed_stride;
  const uint32_t* seed_count;
  uint32_t k;
  float coef;                    // explorationCoefficient = epsilon + 1 (float)
  float radius;                  // sc.radius
  uint64_t edge_size;            // resolved getEdgeSize()
  uint32_t ht_log2;              // visited hash capacity (log2); 0 = HBM bitmap only
  uint32_t cq_cap;               // unchecked LDS capacity
  uint32_t vf_log2;              // LDS visited-filter bits (log2) before the HBM epochs; 0 = none
  uint32_t accepted_only;        // epochs/filter hold only ids that entered the unchecked set
  const uint8_t* fcodes;         // 1-byte filter copy [nrows][fstride] (filter_kernels.hip) or null
  uint64_t fstride;              // bytes per code row: dp (L2 rows of 96/128), dp rounded up to 128 B (long rows)
  const float* fparams;          // {a, b, E, X, valid} of the filter copy
  uint32_t* out_ids;             // [nq][k]
  float* out_dists;              // [nq][k]
  uint32_t* out_n;               // [nq]
  uint64_t* counters;            // [nq][8]: distances, visits, expansions, overflow, edges, max queue
  uint32_t* work;                // work counter (zeroed before launch)
  uint8_t* vis;                  // [slots][vis_stride] visited epochs, zero-initialised
  uint64_t vis_stride;           // >= nrows, multiple of 16
  uint32_t* slot_epoch;          // [slots] last epoch used by each slot
  uint64_t* spill;               // [slots][spill_cap]
  uint32_t spill_cap;
  int* error;
  // lookahead kernel (search_la.hip): list capacity (entries of one step's
  // target lists, >= 256) and log2 of the per-step id hash (>= log2(2 lmax))
  uint32_t la_lmax;
  uint32_t la_sh_log2;
  // latency kernel (search_lat.hip): speculation slots and LDS tail keys
  uint32_t lat_slots;
  uint32_t lat_tail;
  uint32_t lat_hop;              // latency kernel: warm L2 for the nearest fresh neighbour of each list part
  uint32_t lat_feed;             // latency kernel: head entries kept speculated (0: 16; capped by lat_slots)
  // launch schedule (ngt_amd_api.cpp run_search, "probe and resume"): the
  // w-th work item a slot claims is query order[w] (null: w), and a launch
  // has *nwork_dev work items (null: nq).  A probe launch (pause_after > 0)
  // pauses every query after pause_after expansions: its state goes to
  // qstate[qi] (PauseLayout), qflag[qi] = 1 and prio[qi] = the unchecked keys
  // within the exploration radius (the predicted rest of its search); a query
  // that ends first writes its results and qflag[qi] = 2.  A later launch
  // resumes the paused queries (qflag 1) from their saved state, longest
  // predicted first.  Results, distance bits and expansion / edge counts are
  // the single launch's in any order and split; the evaluation counters
  // ([0], [1], [6]) may be higher: the resume rebuilds the accepted-only set
  // from the popped ids and the unchecked keys, and accepted ids that a
  // compaction had dropped beyond the radius are evaluated (and rejected)
  // again.  The bench takes U(q) from a full-visited-set run, never scheduled.
  const uint32_t* order;
  const uint32_t* nwork_dev;
  uint32_t pause_after;
  uint8_t* qstate;
  uint64_t qstate_stride;
  uint32_t* qflag;
  float* prio;
  unsigned long long* stat;      // [2]: expansions and queries finished by this launch (device sums) or null
};

// One paused query's saved state (the one-expansion kernel's accepted-only
// filtered path): counters and radius, the results, the unchecked keys (LDS
// and spill) and the ids popped so far.  The accepted-only visited set is
// rebuilt from the popped ids and the unchecked keys: every accepted id is
// one of them, except keys compaction dropped beyond the exploration radius,
// which a re-evaluation rejects again (search_common.h not_accepted).
constexpr uint32_t kPauseSpillMax = 1024;  // a query with more spill keys is not paused
constexpr uint32_t kPauseStepMax = 8;      // popped ids one step may add past pause_after
struct PauseHdr {
  uint32_t ncq, nspill, nres, npop, maxq, pad0;
  float radius, pad1;
  unsigned long long ndist, nvisit, nexp, nedge, nexact, pad2;
};
struct PauseLayout {
  uint64_t off_res, off_cq, off_spill, off_pop, total;
  __host__ __device__ PauseLayout(uint32_t k, uint32_t cq_cap, uint32_t pause_after) {
    off_res = 128;
    off_cq = off_res + 8ull * ((k + 1) & ~1u);
    off_spill = off_cq + 8ull * cq_cap;
    off_pop = off_spill + 8ull * kPauseSpillMax;
    // a lookahead step commits up to kPauseStepMax targets, so a query may
    // pass pause_after by that many before the check at the step's start
    total = (off_pop + 4ull * (pause_after + kPauseStepMax) + 127) & ~127ull;
  }
};

// Serving form of the latency kernel (search_lat.hip, serve.cpp): a resident
// grid takes single queries from a ring in pinned host memory as callers post
// them and answers each one as soon as it finishes -- no launch per call and
// no batch waiting for its slowest query.
//
// A request slot: ServeReqHdr, kServeMaxSeeds seed ids, then the prepared
// query (dp floats) at kServeQueryOff; req_bytes apart.
constexpr uint32_t kServeMaxSeeds = 128;
constexpr uint32_t kServeQueryOff = 32 + 4 * kServeMaxSeeds;
struct ServeReqHdr {
  uint32_t seq;      // ticket + 1 once the slot is posted (host release store)
  uint32_t k;        // SearchContainer::size, <= 64
  uint32_t ns;       // random seeds in the slot (tree mode: descend instead)
  uint32_t flags;
  float coef;        // explorationCoefficient
  float radius;      // sc.radius
  uint32_t pad[2];
};
struct ServeResp {
  uint32_t seq;      // ticket + 1 once answered (device system-scope release)
  uint32_t n;
  uint32_t err;      // the batch kernel's error bits for this query
  uint32_t pad;
  uint64_t counters[8];
  uint32_t ids[64];
  float dists[64];
};
struct ServeDevCtl {
  uint32_t avail;    // tickets below this are posted (dispatcher)
  uint32_t claimed;  // tickets below this are taken by a worker
  uint32_t closing;  // the dispatcher has stopped: drain and leave
  uint32_t pad;      // why it stopped: 1 asked, 2 idle, 3 lifetime
  uint32_t done;     // tickets answered (counted from the launch's first)
};
struct ServeArgs {
  const uint8_t* ring;     // [nring][req_bytes] pinned host memory
  uint64_t req_bytes;
  ServeResp* resp;         // [nring] pinned host memory
  uint32_t nring;
  uint32_t workers;        // worker workgroups; block `workers` dispatches
  ServeDevCtl* dctl;       // device memory
  const uint32_t* stop;    // pinned host words: [0] stop dispatching, [1] tickets handed out
  uint32_t start;          // first ticket of this launch
  uint32_t use_tree;       // seeds from the tree (else the request's)
  uint64_t idle_ticks;     // dispatcher leaves after this long with nothing posted or in flight (100 MHz clock)
  uint64_t life_ticks;     // ... or this long in all; workers' own bound is longer
  TreeSeedArgs tree;
};

// lookahead targets per step of search_la.hip: mode 0 (throughput, one wave
// per query), mode 1 (latency, eight waves per query)
inline uint32_t la_targets(int mode) {
  if (mode != 0) return 8u;
  // 2: ANNG 88.4k QPS vs 72.5k at 3 and 57.8k at 4 targets per step
  // (profiles/r3/anng_p)
  return 2u;
}
// resident waves per SIMD of the throughput form: 4 (128 VGPRs, 4 filter
// groups in flight, 256 LDS keys, 16 Kbit filter: <= 10 KB of LDS so 16
// workgroups fit a CU; ANNG 72.0k QPS) or 3 (168 VGPRs, 6 groups, 512 keys,
// 32 Kbit; 64.7k QPS): 4
inline int la_wpe() { return 4; }
// latency kernel: hop prefetch of each list part's nearest fresh neighbour
// (search_lat.hip); NGT_AMD_LAT_HOP=0 turns it off (A/B)
// (read per launch, so a test process can compare both forms)
inline uint32_t lat_hop_default() {
  const char* e = ngt_amd::knob("NGT_AMD_LAT_HOP");
  return e ? (atoi(e) != 0 ? 1u : 0u) : 1u;
}
// latency kernel: head entries kept speculated; NGT_AMD_LAT_FEED=n (A/B)
inline uint32_t lat_feed_default() {
  const char* e = ngt_amd::knob("NGT_AMD_LAT_FEED");
  return e ? (uint32_t)std::max(1, std::min(64, atoi(e))) : 0u;
}
uint32_t search_la_lds_bytes(const SearchArgs& a, int P);
uint32_t search_lat_lds_bytes(const SearchArgs& a);
hipError_t launch_graph_search_lat(const SearchArgs& a, uint32_t slots, hipStream_t s);
hipError_t launch_graph_serve_lat(const SearchArgs& a, const ServeArgs& sv, hipStream_t s);
hipError_t launch_graph_search_la(const SearchArgs& a, int mode, bool full, uint32_t slots, hipStream_t s);

struct LinearArgs {
  const uint8_t* rows;
  uint64_t row_bytes;
  uint64_t nrows;
  int dp;
  const uint8_t* valid;          // [nrows] or null
  const uint8_t* queries;
  uint64_t query_bytes;
  uint32_t nq;
  uint32_t k;
  double radius;                 // < 0 => unbounded
  uint64_t* partial;             // [nq][nslices][k]
  uint32_t* out_ids;
  float* out_dists;
  uint32_t* out_n;
};

struct MergeArgs {
  const uint32_t* in_ids;        // [nparts][nq][k] shard-local ids
  const float* in_dists;         // [nparts][nq][k]
  const uint32_t* in_n;          // [nparts][nq]
  const uint32_t* id_offsets;    // [nparts] local -> global id offset
  uint32_t nparts, nq, k;
  uint32_t* out_ids;             // [nq][k] global ids
  float* out_dists;
  uint32_t* out_n;               // [nq]
  // packed merge only: words between parts (0: nq * k) and, when non-null,
  // the flag ORed with every part's trailer word (packed[part * stride + nq * k])
  uint64_t part_stride;
  int* err_out;
};

// ---- ANNG construction (build_kernels.hip) ----------------------------------
struct TreeBuildArgs {
  const uint8_t* rows;           // object rows (row_bytes apart)
  uint64_t row_bytes;
  int dp;
  // leaves [leaf_cap_nodes]: parent (raw Node::ID), pivot row, objects (id, distance)
  uint32_t* lf_parent;
  uint8_t* lf_has_pivot;
  uint8_t* lf_pivot;             // [L][row_bytes]
  uint32_t* lf_count;
  uint32_t* lf_ids;              // [L][leaf_cap]
  float* lf_dist;                // [L][leaf_cap]
  uint32_t leaf_cap;             // >= leaf_size + 1
  // internal nodes [in_cap_nodes]
  uint32_t* in_parent;
  uint8_t* in_pivot;             // [I][row_bytes]
  uint32_t* in_child;            // [I][5]
  float* in_border;              // [I][4]
  uint32_t* counts;              // [0] next leaf id, [1] next internal id, [2] root raw id
  uint32_t leaf_cap_nodes, in_cap_nodes;
  uint32_t leaf_size;            // leafObjectsSize (100)
  const uint32_t* ids;           // batch object ids, batch order
  const uint8_t* insert_flag;    // [n] 0 = not inserted into the tree
  // leaf / count / pivot distance of each batch object against the tree at
  // batch start (TreeSeedArgs::out_*), or null to descend from the root
  const uint32_t* pre_leaf;
  const uint32_t* pre_count;
  const float* pre_dist;
  uint32_t n;
  int* error;
};

// insertMultipleSearchResults (Index.cpp:673-727) on the device: the batch's
// pair distances, then per batch object the edgeSizeForCreation best of its
// search results and the earlier batch objects, by (distance, id).
struct BatchPairArgs {
  const uint8_t* rows;           // object rows
  uint64_t row_bytes;
  int dp;
  const uint8_t* batch;          // the batch objects' rows, batch order
  const uint32_t* ids;           // [n] batch ids
  uint32_t n;
  float* out;                    // [n(n-1)/2]: pair (i, j), j < i, at i(i-1)/2 + j
};

struct BatchMergeArgs {
  const uint32_t* res_ids;       // [n][K] insertion search results
  const float* res_dists;
  const uint32_t* res_n;         // [n]
  uint32_t K;                    // edgeSizeForCreation
  const uint32_t* ids;           // [n] batch ids
  const float* pair;             // BatchPairArgs::out
  uint32_t n;
  uint32_t* out_ids;             // [n][K]
  float* out_dists;
  uint32_t* out_n;               // [n]
  uint8_t* flag;                 // [n] DVP-tree insertion flag (Index.cpp:1201-1203)
};

hipError_t launch_batch_pairs(const BatchPairArgs& a, int metric, int otype, hipStream_t s);
hipError_t launch_batch_merge(const BatchMergeArgs& a, hipStream_t s);
hipError_t launch_tree_insert(const TreeBuildArgs& a, int metric, int otype, hipStream_t s);
hipError_t launch_adj_scatter(uint32_t* adj, uint64_t stride, const uint32_t* nodes, const uint32_t* vals,
                              uint32_t n, hipStream_t s);
hipError_t launch_gather_rows(uint8_t* dst, const uint8_t* rows, uint64_t row_bytes, const uint32_t* ids,
                              uint32_t n, hipStream_t s);

hipError_t launch_distances(const DistanceArgs& a, int metric, int otype, hipStream_t s);
hipError_t launch_merge_results(const MergeArgs& a, hipStream_t s);
hipError_t launch_pack_results(const uint32_t* ids, const float* dists, const uint32_t* n, uint32_t nq, uint32_t k,
                               uint64_t* out, hipStream_t s);
hipError_t launch_merge_packed(const MergeArgs& a, const uint64_t* packed, hipStream_t s);
hipError_t launch_tree_seeds(const TreeSeedArgs& a, int metric, int otype, hipStream_t s);
size_t search_lds_bytes(const SearchArgs& a, int otype);
// the resume launch's order: paused queries (qflag 1) by descending prio
hipError_t launch_schedule(const uint32_t* qflag, const float* prio, uint32_t nq, uint32_t* order, uint32_t* n_out,
                           hipStream_t s);
hipError_t launch_graph_search(const SearchArgs& a, int metric, int otype, uint32_t slots,
                               hipStream_t s);
hipError_t launch_linear_search(const LinearArgs& a, int metric, int otype, uint32_t nslices,
                                hipStream_t s);
hipError_t launch_linear_merge(const LinearArgs& a, uint32_t nslices, hipStream_t s);
// query-tiled exact scan (scan_kernels.hip): float L2, Dp <= 256, k <= 32;
// hipErrorNotSupported otherwise.  Writes a.partial [nq][nparts][k].
hipError_t launch_linear_scan(const LinearArgs& a, int metric, int otype, uint32_t nparts, uint32_t rows_per_part,
                              hipStream_t s);
size_t linear_scan_lds_bytes(uint32_t k, int dp);

// Matrix-core filtered exact scan (scan_mfma.hip).  Operands in fragment order:
// [32-object tile][k-step][64 lanes][8 bf16], k-steps = dp/16 + 1 (the last one
// carries the filter's norm column).
struct ScanPrepArgs {
  const uint8_t* src;            // float rows / prepared queries
  uint64_t stride;               // bytes between objects
  uint64_t n;                    // objects
  uint64_t n_pad;                // queries: entries of hb to write
  const uint8_t* valid;          // rows: [n] or null
  int dp;
  uint32_t ks;
  uint64_t ntiles32;
  uint16_t* out_h;
  uint16_t* out_l;
  float one_minus_kappa, kappa, slack, kappa_boot;
  uint32_t* xmax_bits;           // rows: atomicMax target; queries: read
  float* hb;                     // queries: [n_pad] filter base
  float* hm;                     // queries: [n_pad] bootstrap margin
};
struct MfmaScanArgs {
  const uint16_t* rh;
  const uint16_t* rl;
  const uint16_t* qh;
  const uint16_t* ql;
  const float* hb;
  const float* hm;
  const uint8_t* rows;
  uint64_t row_bytes;
  const uint8_t* queries;
  uint64_t query_bytes;
  uint32_t nq, k, ks;
  int dp;
  uint32_t mb0, mblocks, ntiles, tiles_per_part, nparts;  // this launch: query blocks mb0 .. + mblocks
  uint32_t xcd;                  // parts a multiple of 8, part p on XCD p % 8
  double radius;
  float scale, t_init;
  uint32_t dbg;                  // profiling knobs (NGT_AMD_SCAN_DBG): 1 no filter, 2 no processing
  unsigned long long* stats;     // or null: [0] candidates, [1] processing rounds, [2] tiles with candidates
  unsigned long long* gthr;      // [nq] smallest k-th key over the parts (all ones at launch)
  uint64_t* partial;             // [nq][nparts][k]
};
hipError_t launch_scan_prep(const ScanPrepArgs& a, bool cosine, bool query, hipStream_t s);
hipError_t launch_scan_mfma(const MfmaScanArgs& a, int metric, int passes, hipStream_t s);
size_t scan_mfma_lds_bytes(uint32_t k);

// ---- NGTQG (qg_kernels.hip) ------------------------------------------------
struct QgLutArgs {
  const uint8_t* queries;        // prepared float query rows (padded dp)
  uint64_t query_bytes;
  uint32_t nq;
  const float* global;           // [D] global centroid
  const float* local;            // [M][16][dsub] local centroids (ids 1..16)
  uint32_t M, dsub, Me;          // Me = M rounded up to even
  uint8_t* lut;                  // [nq][lut_stride], lut_stride >= Me*16
  uint64_t lut_stride;
  float* scale;                  // [nq]
  float* toff;                   // [nq] totalOffset
};

struct QgBuildArgs {
  const uint64_t* edge_off;      // graph CSR [nrows+1]
  const uint32_t* edges;
  uint32_t nrows;
  uint32_t max_edges;
  const uint8_t* local_codes;    // [nrows][M] localID - 1 (0..15)
  uint32_t M, Me;
  uint32_t* qids;                // [nrows][id_stride], 0-terminated
  uint32_t id_stride;
  uint8_t* qcodes;               // [nrows][code_stride]
  uint64_t code_stride;          // (id_stride / 16) * 8 * Me
};

// NGTQG encoder: per object and subspace, the nearest local centroid of the
// residual (object - global centroid), ties to the lower local id.
struct QgEncodeArgs {
  const uint8_t* rows;           // padded float rows, row_bytes apart
  uint64_t row_bytes;
  uint64_t row0, nrows;          // encode rows [row0, row0 + nrows)
  const float* global;           // [D]
  const float* local;            // [M][16][dsub]
  uint32_t M, dsub;
  uint8_t* codes;                // [row0 + nrows][M] localID - 1
};

// Local codebook training (one workgroup per subspace): Lloyd iterations
// over the residual subvectors of objects 1..nsample from the first 16.
struct QgTrainArgs {
  const uint8_t* rows;
  uint64_t row_bytes;
  uint32_t nsample;              // objects 1..nsample (<= 4096)
  const float* global;
  uint32_t M, dsub;              // dsub <= 16
  uint32_t max_iter;
  float* local;                  // [M][16][dsub] out
  uint32_t* iters;               // [M] iterations run (out)
};

struct QgAdcArgs {
  const uint32_t* qids;
  uint32_t id_stride;
  const uint8_t* qcodes;
  uint64_t code_stride;
  uint32_t Me;
  const uint8_t* lut;
  uint64_t lut_stride;
  const float* scale;
  const float* toff;
  const uint32_t* qidx;          // per pair: query
  const uint32_t* node;          // per pair: node whose neighbour list is scored
  uint64_t npairs;
  float* out;                    // [npairs][out_stride]
  uint32_t out_stride;
  uint32_t* out_n;               // [npairs] neighbour count
};

struct QgSearchArgs {
  const uint8_t* rows;           // exact rows (seeds, rerank)
  uint64_t row_bytes;
  uint32_t nrows;
  int dp;
  const uint32_t* qids;
  uint32_t id_stride;
  const uint8_t* qcodes;
  uint64_t code_stride;
  uint32_t Me;
  const uint8_t* lut;
  uint64_t lut_stride;
  const float* scale;
  const float* toff;
  const uint8_t* queries;
  uint64_t query_bytes;
  uint32_t nq;
  const uint32_t* seeds;
  const uint64_t* seed_off;
  uint32_t seed_stride;
  const uint32_t* seed_count;
  uint32_t k;                    // sizeBackup
  uint32_t size;                 // sc.size after *= resultExpansion
  int rerank;                    // resultExpansion >= 1
  float coef;
  float radius;
  uint32_t ht_log2;
  uint32_t cq_cap;
  uint32_t vf_log2;              // LDS visited-filter bits (log2); 0 = none
  const uint8_t* recs;           // packed records (QgState::recs), or null: the fixed-stride slabs
  const uint32_t* qkw;           // [nrows] key words of the packed layout
  uint32_t rec_shift;            // record unit = 1 << rec_shift bytes
  uint32_t* out_ids;             // [nq][k]
  float* out_dists;
  uint32_t* out_n;
  uint64_t* counters;            // [nq][8]: ADC, accepted, expansions, exact, code blocks, max queue, spilled
  uint32_t* work;
  uint8_t* vis;
  uint64_t vis_stride;
  uint32_t* slot_epoch;
  uint64_t* spill;
  uint32_t spill_cap;
  int* error;
};

hipError_t launch_qg_lut(const QgLutArgs& a, hipStream_t s);
hipError_t launch_qg_build(const QgBuildArgs& a, hipStream_t s);
// packed search layout: blocks per node (>= 1) from the fixed id rows, then
// every node's record and key word (QgState::recs / qkw)
hipError_t launch_qg_blocks(const uint32_t* qids, uint32_t id_stride, uint32_t nrows, uint8_t* nb, hipStream_t s);
hipError_t launch_qg_pack(const uint32_t* qids, uint32_t id_stride, const uint8_t* qcodes, uint64_t code_stride,
                          uint32_t Me, uint32_t nrows, const uint32_t* qkw, uint32_t rec_shift, uint8_t* recs,
                          hipStream_t s);
hipError_t launch_qg_adc(const QgAdcArgs& a, hipStream_t s);
hipError_t launch_qg_encode(const QgEncodeArgs& a, hipStream_t s);
hipError_t launch_qg_train(const QgTrainArgs& a, hipStream_t s);
size_t qg_search_lds_bytes(const QgSearchArgs& a);
hipError_t launch_qg_search(const QgSearchArgs& a, uint32_t slots, hipStream_t s);

// NGTQ IVF-ADC aggregation (ivf_kernels.hip): NGTQ::AggregationMode values
// the kernel distinguishes.
enum IvfMode : int { kIvfApprox = 0, kIvfCache = 1, kIvfLut = 2, kIvfExact = 3, kIvfRefine = 4 };

struct IvfSearchArgs {
  const uint8_t* queries;        // prepared padded float rows, query_bytes apart
  uint64_t query_bytes;
  uint32_t nq;
  int dp;
  const uint32_t* cent_ids;      // [nq][cent_stride] global-codebook search results
  const float* cent_d;
  const uint32_t* cent_n;        // [nq]
  uint32_t cent_stride;
  const uint8_t* grows;          // global centroid rows (padded floats)
  uint64_t grow_bytes;
  const float* local;            // [N][17][dsub] local centroids (entry 0 unused)
  uint32_t N, dsub, lid_stride;  // lid_stride: uint16 local ids per entry
  const uint64_t* list_off;      // [nlists + 1] inverted lists by global id
  uint32_t nlists;
  const uint32_t* eids;          // [entries] object ids
  const uint16_t* elids;         // [entries][lid_stride] local ids
  const uint8_t* orows;          // object list rows (padded floats)
  uint64_t orow_bytes;
  uint32_t size;                 // result size
  uint64_t ass;                  // approximateSearchSize
  int mode;                      // IvfMode
  uint32_t* out_ids;             // [nq][size]
  float* out_dists;
  uint32_t* out_n;               // [nq]
};
size_t ivf_search_lds_bytes(const IvfSearchArgs& a);
// 1-byte filter copy of an L2 float repository: codes [nrows][dp], st [5]
// scratch, params [5] = {a, b, E, X, valid}
hipError_t launch_filter_build(const uint8_t* rows, uint64_t row_bytes, uint64_t nrows, uint32_t dp, uint64_t stride,
                               uint8_t* codes,
                               uint32_t* st, float* params, hipStream_t s);
hipError_t launch_ivf_search(const IvfSearchArgs& a, hipStream_t s);

}  // namespace ngt_amd
