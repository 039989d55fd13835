/*
 * ngt_amd.h -- C ABI of the MI355X-native NGT distance hot path.
 *
 * These entry points are the batched device form of the reference's search
 * path.  Each one names the reference interface it replaces:
 *
 *   ngt_amd_search          <- NGT::GraphAndTreeIndex::search(SearchContainer&)
 *                              (lib/NGT/Index.h:1570-1577) and
 *                              NGT::Index::searchUsingOnlyGraph (Index.h:479-484),
 *                              i.e. getSeedsFromTree (Index.h:1524-1567) +
 *                              NeighborhoodGraph::searchReadOnlyGraph
 *                              (lib/NGT/Graph.cpp:398-495), for a batch of queries.
 *   ngt_amd_linear_search   <- NGT::GraphIndex::linearSearch (Index.h:729-749) /
 *                              ObjectSpaceRepository::linearSearch
 *                              (lib/NGT/ObjectSpaceRepository.h:466-502).
 *   ngt_amd_distances       <- PrimitiveComparator::<Metric>::compare
 *                              (lib/NGT/PrimitiveComparator.h:650-752) over a
 *                              batch of (query, object id) pairs.
 *   ngt_amd_index_*         <- the object repository / graph / tree that
 *                              NGT::Index::open loads (lib/NGT/Index.cpp:92-111),
 *                              laid out in HBM (padded row-major slab, CSR
 *                              adjacency, flattened DVP tree).
 *
 * The drop-in `ngt_*` C API (include/NGT/Capi.h, same names and signatures as
 * lib/NGT/Capi.h) is implemented on top of these.
 *
 * Conventions: plain pointers and sizes; functions return 0 on success and a
 * negative value on failure with a message retrievable by
 * ngt_amd_last_error().  `*_device` variants take device pointers and enqueue
 * on the given HIP stream (hipStream_t passed as void*; NULL = the default
 * stream, ordered with every blocking stream); the others take host
 * pointers and are synchronous.  There is no CPU fallback: without a usable
 * gfx950 device every compute call fails with an error.
 */
#ifndef NGT_AMD_H
#define NGT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* NGT::ObjectSpace::DistanceType values (lib/NGT/ObjectSpace.h:166-180). */
#define NGT_AMD_DISTANCE_L1 0
#define NGT_AMD_DISTANCE_L2 1
#define NGT_AMD_DISTANCE_HAMMING 2
#define NGT_AMD_DISTANCE_ANGLE 3
#define NGT_AMD_DISTANCE_COSINE 4
#define NGT_AMD_DISTANCE_NORMALIZED_ANGLE 5
#define NGT_AMD_DISTANCE_NORMALIZED_COSINE 6
#define NGT_AMD_DISTANCE_JACCARD 7
#define NGT_AMD_DISTANCE_SPARSE_JACCARD 8
#define NGT_AMD_DISTANCE_NORMALIZED_L2 9
#define NGT_AMD_DISTANCE_POINCARE 100
#define NGT_AMD_DISTANCE_LORENTZ 101
/* NGT::ObjectSpace::ObjectType (lib/NGT/ObjectSpace.h:182-186). */
#define NGT_AMD_OBJECT_UINT8 1
#define NGT_AMD_OBJECT_FLOAT 2

/* Seed providers (NeighborhoodGraph::SeedType, lib/NGT/Graph.h:279-285). */
#define NGT_AMD_SEED_TREE 0    /* DVP-tree leaf (GraphAndTreeIndex::search)        */
#define NGT_AMD_SEED_GIVEN 1   /* caller-supplied seed lists (search(sc, seeds))    */
#define NGT_AMD_SEED_RANDOM 2  /* getRandomSeeds over the library's rand() stream   */

typedef struct ngt_amd_index ngt_amd_index;

typedef struct {
  uint32_t k;            /* SearchContainer::size                                  */
  float epsilon;         /* SearchContainer::setEpsilon (coef = epsilon + 1)         */
  float radius;          /* SearchContainer::radius; < 0 => FLT_MAX (Capi.cpp:357)   */
  int64_t edge_size;     /* SearchContainer::edgeSize: -1 property, 0 all, -2 dyn.   */
  int32_t seed_mode;     /* NGT_AMD_SEED_*                                          */
  int32_t all_leaf_nodes;/* SearchContainer::useAllNodesInLeaf                      */
  int32_t visited_hash_log2; /* visited set: 0 = default LDS hash (2^12 ids, spills
                                exactly to an HBM bitmap), 8..15 = LDS hash of that
                                size, -1 = HBM bitmap from the start (for searches
                                that visit far more ids than an LDS hash holds),
                                -2 = as -1 but the set holds only ids that entered
                                the unchecked set: identical results, fewer HBM
                                probes; rejected neighbours met again are
                                re-evaluated, so counters[0] counts evaluations,
                                not the reference's distinct distance count    */
  int32_t distance_filter; /* 1-byte filter copy of L2 float rows (96/128 elements):
                                0 = auto (launches of >= 2 queries per CU), 1 = on,
                                -1 = off; identical results either way          */
} ngt_amd_search_params;

/* Per-query counters written by the search (8 x uint64 per query):
 * [0] distance computations (seeds + evaluated neighbours), [1] evaluated
 * neighbours (visitCount), [2] expanded nodes, [3] 1 if the visited set spilled
 * from LDS to the HBM bitmap, [4] adjacency entries read, [5] largest unchecked
 * set, [6] exact distances of neighbours, [7] seed distances. */
#define NGT_AMD_COUNTERS_PER_QUERY 8

const char *ngt_amd_last_error(void);
int ngt_amd_device_count(void);
/* Reseed the rand() stream NGT_AMD_SEED_RANDOM searches draw from.  It is a
 * glibc random(3) TYPE_3 sequence private to the library, seeded 1 at load --
 * what a fresh reference process's rand() returns (GraphIndex::getRandomSeeds,
 * lib/NGT/Index.h:775-801) -- so other rand() users cannot shift it. */
void ngt_amd_srand(unsigned int seed);

/* ---- index ------------------------------------------------------------- */
int ngt_amd_index_create(ngt_amd_index **out, int device, int distance_type,
                         int object_type, uint32_t dimension);
void ngt_amd_index_destroy(ngt_amd_index *index);
/* Padded dimension ((dim-1)/16+1)*16 (ObjectSpace::getPaddedDimension). */
uint32_t ngt_amd_index_padded_dimension(const ngt_amd_index *index);
/* rows: host [nrows][padded_dimension] elements, row 0 the dummy slot;
 * valid: [nrows] (0 = removed slot) or NULL. */
int ngt_amd_index_set_objects(ngt_amd_index *index, const void *rows, uint64_t nrows,
                              const uint8_t *valid);
/* Device rows already in HBM (row-major padded, row_bytes = padded dim *
 * element size); the index keeps the pointer, the caller keeps ownership. */
int ngt_amd_index_set_objects_device(ngt_amd_index *index, const void *d_rows, uint64_t nrows);
/* CSR adjacency: edges of node v are edges[offsets[v] .. offsets[v+1]). */
int ngt_amd_index_set_graph(ngt_amd_index *index, const uint64_t *offsets,
                            const uint32_t *edges, uint64_t nedges);
int ngt_amd_index_set_graph_device(ngt_amd_index *index, const uint64_t *d_offsets,
                                   const uint32_t *d_edges, uint64_t nedges);
/* Flattened DVP tree (lib/NGT/Tree.h, Node.h): internal node i has pivot row
 * in_pivot[i] (padded), children in_child[i*children..], borders
 * in_border[i*(children-1)..]; leaf j holds leaf_ids[leaf_off[j]..leaf_off[j+1]).
 * root is the raw Node::ID (bit 31 = leaf). */
int ngt_amd_index_set_tree(ngt_amd_index *index, const void *in_pivot, uint32_t n_internal,
                           const uint32_t *in_child, const float *in_border, uint32_t children,
                           uint32_t root, const uint64_t *leaf_off, uint32_t n_leaf,
                           const uint32_t *leaf_ids, uint64_t n_leaf_ids);
/* Graph/search properties (NeighborhoodGraph::Property, lib/NGT/Graph.h:383-524). */
int ngt_amd_index_set_search_property(ngt_amd_index *index, int32_t edge_size_for_search,
                                      int32_t dynamic_edge_size_base,
                                      int32_t dynamic_edge_size_rate, int32_t seed_size,
                                      int32_t seed_type);
/* Resolve NeighborhoodGraph::getEdgeSize (lib/NGT/Graph.h:675-692). */
uint64_t ngt_amd_resolve_edge_size(const ngt_amd_index *index, int64_t edge_size, float epsilon);

/* ---- search ------------------------------------------------------------ */
/* Host pointers.  queries: [nq][dimension] floats for every object type; they
 * are converted/normalized on the device exactly like Index::allocateObject.  seeds /
 * seed_off: CSR seed lists for NGT_AMD_SEED_GIVEN (else NULL).  Outputs:
 * ids/dists [nq][k] ascending (distance, id), n [nq], counters [nq][4] or NULL. */
int ngt_amd_search(ngt_amd_index *index, const ngt_amd_search_params *params,
                   const void *queries, uint32_t nq, const uint32_t *seeds,
                   const uint64_t *seed_off, uint32_t *ids, float *dists, uint32_t *n,
                   uint64_t *counters);
/* Device pointers; queries are already padded rows of the object type
 * (query_bytes apart) and already normalized where the metric requires it. */
/* The tree seeds of nq prepared device queries: GraphAndTreeIndex::
 * getSeedsFromTree (lib/NGT/Index.h:1524-1567) -- DVP-tree leaf descent
 * (Tree.cpp:400-563) and the srand(leafID) thinning to min(seedSize, k) --
 * into d_seeds [nq][seed_stride >= 128] and d_count [nq]: the seed lists a
 * NGT_AMD_SEED_TREE search starts from, for callers that keep them. */
int ngt_amd_tree_seeds_device(ngt_amd_index *index, const void *d_queries, uint64_t query_bytes, uint32_t nq,
                              uint32_t k, uint32_t *d_seeds, uint32_t seed_stride, uint32_t *d_count,
                              void *stream);
/* The form of the latest graph-search launch on this index: -1 the
 * one-expansion-per-pop kernel, 0 the lookahead kernel with a wave per query,
 * 1 the lookahead kernel with eight waves per query (search_la.hip). */
int ngt_amd_last_search_lookahead(const ngt_amd_index *index);
/* One query through the resident serving grid: the single-query search of
 * ngt_search_index (lib/NGT/Capi.cpp:377-406 -> NeighborhoodGraph::search)
 * for concurrent callers.  A long-lived launch of the latency kernel takes
 * queries from a ring in pinned host memory as they are posted and answers
 * each one as soon as it finishes (no launch per call, no batch waiting for
 * its slowest member); it leaves by itself when idle.  query: host floats of
 * the index's object dimension (L2 float rows of 96/128 padded elements);
 * params->seed_mode NGT_AMD_SEED_RANDOM or NGT_AMD_SEED_TREE, k <= 64.
 * Results, distances and counters equal ngt_amd_search's.  Thread-safe.
 * Returns 0 when served, 1 when this index or request is not one the grid
 * serves (call ngt_amd_search instead), -1 on error. */
int ngt_amd_search_served(ngt_amd_index *index, const ngt_amd_search_params *params, const float *query,
                          uint32_t *ids, float *dists, uint32_t *n, uint64_t *counters);
/* Stop the serving grid now (it also stops by itself after a short idle time). */
int ngt_amd_serve_stop(ngt_amd_index *index);
/* Queries the serving grid answered and grids launched since the index was created. */
int ngt_amd_serve_stats(ngt_amd_index *index, uint64_t *served, uint64_t *launches);
int ngt_amd_search_device(ngt_amd_index *index, const ngt_amd_search_params *params,
                          const void *d_queries, uint64_t query_bytes, uint32_t nq,
                          const uint32_t *d_seeds, const uint64_t *d_seed_off, uint32_t *d_ids,
                          float *d_dists, uint32_t *d_n, uint64_t *d_counters, void *stream);

int ngt_amd_linear_search(ngt_amd_index *index, const void *queries, uint32_t nq, uint32_t k,
                          double radius, uint32_t *ids, float *dists, uint32_t *n);
int ngt_amd_linear_search_device(ngt_amd_index *index, const void *d_queries,
                                 uint64_t query_bytes, uint32_t nq, uint32_t k, double radius,
                                 uint32_t *d_ids, float *d_dists, uint32_t *d_n, void *stream);

/* Pairwise comparator: out[i] = distance(queries[qidx[i]], object oid[i]).
 * queries are prepared objects ([nq][padded dim] of the object type, as stored). */
int ngt_amd_distances(ngt_amd_index *index, const void *queries, uint32_t nq,
                      const uint32_t *qidx, const uint32_t *oid, uint64_t npairs, float *out);

/* Prepare queries on the device exactly like Index::allocateObject: convert
 * to the object type, zero-pad to the padded dimension, normalize for the
 * normalized metrics (ObjectSpace::normalize, lib/NGT/ObjectSpace.h:251-266). */
int ngt_amd_prepare_queries_device(ngt_amd_index *index, const float *d_in, uint32_t nq,
                                   void *d_out, void *stream);

/* Timing of the last search call's kernels (HIP events on the search stream), ms. */
float ngt_amd_last_search_kernel_ms(const ngt_amd_index *index);
/* 1 if the last graph-search launch read the 1-byte filter copy of the rows
 * (L2 float rows of 96/128 elements, launches of >= 2 queries per CU): its
 * counters [6] are then the exact distances of neighbours the filter bound
 * could not place outside the exploration radius, [7] the seed distances. */
int ngt_amd_last_search_filtered(const ngt_amd_index *index);
/* The device error word of the launch context of `stream` (created on first
 * use, zeroed on that stream and waited for), read on that stream: the word a
 * search on the stream would start from.  Diagnostic; 0 unless a search on
 * the stream left an invariant bit set (device_error_text). */
int ngt_amd_stream_error_word(ngt_amd_index *index, void *stream, int *word);
/* Workgroups (resident one-wave query slots) of the last search launch: per-CU
 * occupancy x CUs for a full batch, bounded by the visited-scratch HBM budget. */
uint32_t ngt_amd_last_search_slots(const ngt_amd_index *index);
/* Launch schedule of the last search call: 0 = one launch in query order;
 * B > 0 = "probe and resume" -- a probe launch paused every query after B
 * expansions (saving its state and the unchecked keys within its exploration
 * radius as the predicted rest of its search) and a resume launch ran the
 * paused ones longest-predicted first, so long searches do not start last
 * (NGT_AMD_SCHED=0 turns it off; results are the same either way). */
uint32_t ngt_amd_last_search_budget(const ngt_amd_index *index);

/* ---- ANNG construction --------------------------------------------------- *
 *   ngt_amd_build_begin / _insert <- GraphAndTreeIndex::createIndex(threadPoolSize)
 *   (lib/NGT/Index.cpp:1158-1257) for graphType ANNG (truncation disabled, the
 *   default): per batch of batch_size_for_creation objects in id order, the
 *   insertion searches (searchForNNGInsertion, Index.h:1457-1479: DVP-tree
 *   seeds with useAllNodesInLeaf, size edgeSizeForCreation, coefficient
 *   epsilon_for_creation + 1), the batch's pairwise distances and merge
 *   (insertMultipleSearchResults, Index.cpp:673-727), insertANNGNode
 *   (Graph.h:611-625) and DVPTree::insert (Tree.cpp:27-265).  The objects must
 *   be set first (ngt_amd_index_set_objects); the index's search graph is
 *   replaced by the construction's padded adjacency until the built graph is
 *   set back with ngt_amd_index_set_graph. */
typedef struct {
  int32_t edge_size_for_creation;   /* EdgeSizeForCreation (10)                      */
  int32_t edge_size_for_search;     /* EdgeSizeForSearch (40), <= 256; 0 = all edges */
  int32_t batch_size_for_creation;  /* BatchSizeForCreation (200)                    */
  int32_t seed_size;                /* SeedSize (10)                                 */
  float epsilon_for_creation;       /* EpsilonForCreation (0.1)                      */
  int32_t reserved;
} ngt_amd_build_params;

int ngt_amd_build_begin(ngt_amd_index *index, const ngt_amd_build_params *params);
/* Insert the valid objects with ids in [first_id, end_id) not yet in the graph. */
int ngt_amd_build_insert(ngt_amd_index *index, uint64_t first_id, uint64_t end_id);
/* GraphRepository size (max inserted id + 1) and total edge count. */
int ngt_amd_build_graph_size(const ngt_amd_index *index, uint64_t *graph_size, uint64_t *nedges);
/* CSR of the built graph: node v's edges ids/dists[offsets[v] .. offsets[v+1]),
 * sorted by (distance, id); offsets [graph_size + 1]. */
int ngt_amd_build_get_graph(const ngt_amd_index *index, uint64_t *offsets, uint32_t *ids, float *dists);
/* Node-slot counts of the built DVP tree (slot 0 of each is the unused dummy)
 * and the total number of leaf entries. */
int ngt_amd_build_tree_size(const ngt_amd_index *index, uint32_t *n_leaf, uint32_t *n_internal,
                            uint64_t *n_leaf_ids);
/* The built DVP tree (Node.h:90-480 fields): per leaf slot parent (raw
 * Node::ID), objects (id, distance) at leaf_off, pivot row; per internal slot
 * parent, pivot row, children[5] (raw ids), borders[4]. */
int ngt_amd_build_get_tree(const ngt_amd_index *index, uint32_t *leaf_parent, uint64_t *leaf_off,
                           uint32_t *leaf_ids, float *leaf_dists, uint8_t *leaf_has_pivot,
                           void *leaf_pivot, uint32_t *in_parent, void *in_pivot, uint32_t *in_child,
                           float *in_border);

/* Incremental construction (createIndex inserts only the objects that have no
 * graph node yet, Index.cpp:618-621, 648-651): after ngt_amd_build_begin, load
 * the index's existing graph and DVP tree -- the inverse of the two getters
 * above -- then ngt_amd_build_insert adds the rest.  A node with no edges is
 * taken as not yet inserted. */
int ngt_amd_build_set_graph(ngt_amd_index *index, const uint64_t *offsets, const uint32_t *ids,
                            const float *dists, uint64_t graph_rows);
int ngt_amd_build_set_tree(ngt_amd_index *index, const uint32_t *leaf_parent, const uint64_t *leaf_off,
                           const uint32_t *leaf_ids, const float *leaf_dists, const uint8_t *leaf_has_pivot,
                           const void *leaf_pivot, uint32_t n_leaf, const uint32_t *in_parent,
                           const void *in_pivot, const uint32_t *in_child, const float *in_border,
                           uint32_t n_internal, uint32_t root);

/* ---- repository sharding (one shard per GPU) ------------ *
 * Merge of per-shard result lists gathered from every rank (RCCL all-gather
 * over xGMI): the k best (distance, global id) per query, the ordering of
 * NGT::ObjectDistance (lib/NGT/Common.h:1946-1959) -- the result a single
 * index over the union would rank.  d_ids/d_dists: [nparts][nq][k] sorted
 * shard-local results, d_n: [nparts][nq] valid entries; id_offsets (host):
 * [nparts] added to shard-local ids.  Outputs [nq][k] and [nq]. */
int ngt_amd_merge_results_device(int device, const uint32_t *d_ids, const float *d_dists,
                                 const uint32_t *d_n, uint32_t nparts, uint32_t nq, uint32_t k,
                                 const uint32_t *id_offsets, uint32_t *d_out_ids, float *d_out_dists,
                                 uint32_t *d_out_n, void *stream);
/* The exchange as ONE message per rank: each result slot packed into a
 * uint64 {float distance bits << 32 | shard-local id} (the ObjectDistance
 * pair, 8 B), 0 = empty slot (slot j >= n[q], or the {0, 0} padding of an
 * NGTQG rerank).  d_packed: [nq][k].  The merge takes the all-gathered
 * [nparts][nq][k] words and ranks by (distance, global id) like
 * ngt_amd_merge_results_device. */
int ngt_amd_pack_results_device(int device, const uint32_t *d_ids, const float *d_dists,
                                const uint32_t *d_n, uint32_t nq, uint32_t k, uint64_t *d_packed,
                                void *stream);
int ngt_amd_merge_packed_device(int device, const uint64_t *d_packed, uint32_t nparts, uint32_t nq,
                                uint32_t k, const uint32_t *id_offsets, uint32_t *d_out_ids,
                                float *d_out_dists, uint32_t *d_out_n, void *stream);

/* ---- sharded repository over the GPUs of a node (shard_api.cpp) --------- *
 * SURVEY.md 8(e), BASELINE C4/C5: rank r holds shard r (global ids
 * id_offsets[r] + 1 ..) as its own index; each call searches the batch on the
 * shard, packs the per-query top-k, exchanges them with ONE RCCL all-gather
 * (nq * k * 8 B per rank) and merges on the device, so every rank returns the
 * k best over the union by (distance, global id) (Common.h:1937-1992).
 * ngt_amd_shard_unique_id fills an RCCL unique id (>= 128 bytes) on one rank;
 * the caller distributes it and every rank creates its communicator with it.
 * id_offsets: host array of every rank's offset -- the call then copies it
 * and synchronizes before returning -- or NULL after
 * ngt_amd_shard_comm_set_offsets stored them on the device: the call then only
 * enqueues (search, pack, all-gather, merge on `stream`), so the exchange of
 * one batch overlaps the search of the next; ngt_amd_shard_comm_synchronize
 * waits and reports.  Each shard's device error flag (unchecked-set spill
 * overflow) travels with its all-gathered message, so every rank fails the
 * batch (at its return or at its synchronize) when any shard's list was
 * truncated.  One call at a time per communicator, and asynchronous calls on
 * one stream.  Replaces nothing in the reference (NGT has no multi-GPU form);
 * the per-shard searches replace NGT::Index::search / NGTQG::Index::search. */
typedef struct ngt_amd_shard_comm ngt_amd_shard_comm;
int ngt_amd_shard_unique_id(uint8_t *id, uint64_t id_bytes);
int ngt_amd_shard_comm_create(ngt_amd_shard_comm **comm, int device, int rank, int world,
                              const uint8_t *id, uint64_t id_bytes);
int ngt_amd_shard_comm_destroy(ngt_amd_shard_comm *comm);
int ngt_amd_shard_comm_set_offsets(ngt_amd_shard_comm *comm, const uint32_t *id_offsets);
int ngt_amd_shard_comm_synchronize(ngt_amd_shard_comm *comm, void *stream);
int ngt_amd_sharded_search_device(ngt_amd_shard_comm *comm, ngt_amd_index *index,
                                  const ngt_amd_search_params *params, const void *d_queries,
                                  uint64_t query_bytes, uint32_t nq, const uint32_t *d_seeds,
                                  const uint64_t *d_seed_off, const uint32_t *id_offsets,
                                  uint32_t *d_out_ids, float *d_out_dists, uint32_t *d_out_n,
                                  void *stream);

/* ---- NGTQG quantized graph (L2, float objects) -------------------------- *
 *   ngt_amd_qg_set_quantizer  <- the NGTQ::Quantizer NGTQG::Index opens from
 *                                <index>/qg (lib/NGT/NGTQ/QuantizedGraph.h:170-185):
 *                                global codebook centroid 1 (QG: the zero
 *                                vector, :397-399) and the M local codebooks.
 *   ngt_amd_qg_build_graph    <- QuantizedGraphRepository::construct (:64-115).
 *   ngt_amd_qg_set_graph      <- QuantizedGraphRepository::deserialize (qg/grp, :130-150).
 *   ngt_amd_qg_lut            <- QuantizedObjectDistance::createDistanceLookup
 *                                (lib/NGT/NGTQ/Quantizer.h:709-760).
 *   ngt_amd_qg_adc            <- QuantizedObjectDistanceFloat::operator()(void*, float*,
 *                                size_t, DistanceLookupTableUint8&) (Quantizer.h:957-1062).
 *   ngt_amd_qg_search[_device]<- NGTQG::Index::search(SearchQuery&) (QuantizedGraph.h:354-372):
 *                                getSeedsFromTree + searchQuantizedGraph (:192-320).
 * M subspaces of dsub dimensions (M * dsub = dimension), 16 centroids each;
 * Me = M rounded up to even, at most 512. */
typedef struct {
  uint32_t k;               /* NGTQGQuery::size                                    */
  float epsilon;            /* NGTQGQuery::epsilon                                 */
  float result_expansion;   /* NGTQGQuery::result_expansion (>= 1: exact rerank)   */
  float radius;             /* NGTQGQuery::radius; < 0 => FLT_MAX                  */
  int32_t seed_mode;        /* NGT_AMD_SEED_TREE / _GIVEN / _RANDOM                */
  int32_t visited_hash_log2;/* as ngt_amd_search_params                            */
} ngt_amd_qg_search_params;

/* global: [dimension] floats; local: [M][16][dsub] floats (local ids 1..16). */
int ngt_amd_qg_set_quantizer(ngt_amd_index *index, const float *global, const float *local,
                             uint32_t M, uint32_t dsub);
/* local_codes: [nrows][M] bytes, localID - 1 (0..15) of every object (qg/ivt),
 * or NULL for the codes of the last ngt_amd_qg_encode (kept in HBM);
 * node v keeps its first min(degree, max_edges) graph edges. */
int ngt_amd_qg_build_graph(ngt_amd_index *index, const uint8_t *local_codes, uint32_t max_edges);
/* Encoder <- the local half of Quantizer::insert (lib/NGT/NGTQ/Quantizer.h:
 * 1895-1959, residuals :1407-1435, nearest centroid by the codebook index's
 * insertion search :1678-1719): every object row 1..nrows-1 coded as its
 * nearest local centroid per subspace (dsub <= 16), ties to the lower id.
 * Codes stay in HBM for ngt_amd_qg_build_graph(NULL); codes_out (nullable):
 * [nrows][M] bytes, localID - 1, row 0 zero. */
int ngt_amd_qg_encode(ngt_amd_index *index, uint8_t *codes_out);
/* Local codebook training for NGTQG (ngtqg quantize, QuantizedGraph.h:423-475):
 * global centroid = the zero vector (:397-399), M subspaces of dim/M (<= 16),
 * 16 centroids each by Lloyd iterations over objects 1..nsample (<= 4096;
 * the reference samples 16 * 100), initialised from the first 16 (Head).
 * The reference clusters with kmeansWithNGT (approximate NGT assignment), so
 * its codebooks are not reproduced bit for bit.  Installs the quantizer like
 * ngt_amd_qg_set_quantizer; local_out (nullable): [M][16][dsub]; iters_out
 * (nullable): [M] iterations run. */
int ngt_amd_qg_train(ngt_amd_index *index, uint32_t M, uint32_t nsample, uint32_t max_iter, float *local_out,
                     uint32_t *iters_out);
/* Node v: neighbour ids qids[qoff[v] .. qoff[v+1]) and packed 4-bit codes
 * codes[code_off[v] .. code_off[v+1]) in the reference stream layout. */
int ngt_amd_qg_set_graph(ngt_amd_index *index, const uint64_t *qoff, const uint32_t *qids,
                         const uint64_t *code_off, const uint8_t *codes);
/* Widest quantized neighbour list (row stride of ngt_amd_qg_adc's output). */
uint32_t ngt_amd_qg_max_degree(const ngt_amd_index *index);
/* Bytes of one node's code row (max degree / 16 blocks of 8 * Me bytes). */
uint64_t ngt_amd_qg_code_stride(const ngt_amd_index *index);
/* Bytes of the packed search layout of the quantized graph (per node its
 * ceil(degree/16) code blocks and their {id, key word} entries, the reference's
 * per-node layout of QuantizedGraphRepository, QuantizedGraph.h:74-113), or 0
 * when searches read the fixed-stride slabs. */
uint64_t ngt_amd_qg_record_bytes(const ngt_amd_index *index);
/* Copy the quantized graph back to the host (what QuantizedGraphRepository::
 * serialize writes, QuantizedGraph.h:117-128): ids [nrows][max_degree]
 * (0-terminated) and codes [nrows][code_stride] in the reference stream layout. */
int ngt_amd_qg_get_graph(const ngt_amd_index *index, uint32_t *ids, uint8_t *codes);
/* Per query: lut [nq][Me*16] bytes, scale [nq], total_offset [nq]. */
int ngt_amd_qg_lut(ngt_amd_index *index, const float *queries, uint32_t nq, uint8_t *lut,
                   float *scale, float *total_offset);
/* ADC distances of node[i]'s whole neighbour list under query qidx[i]'s table:
 * out [npairs][ngt_amd_qg_max_degree], out_n [npairs]. */
int ngt_amd_qg_adc(ngt_amd_index *index, const uint8_t *lut, const float *scale,
                   const float *total_offset, uint32_t nq, const uint32_t *qidx,
                   const uint32_t *node, uint64_t npairs, float *out, uint32_t *out_n);
/* Host pointers; ids/dists [nq][k], n [nq] (k when result_expansion >= 1, padded
 * with {0, 0} as the reference's resize does), counters [nq][8] or NULL:
 * [0] ADC distances, [1] accepted, [2] expansions, [3] exact distances,
 * [4] 16-object code blocks read, [5] max unchecked, [6] visited spill. */
int ngt_amd_qg_search(ngt_amd_index *index, const ngt_amd_qg_search_params *params,
                      const float *queries, uint32_t nq, const uint32_t *seeds,
                      const uint64_t *seed_off, uint32_t *ids, float *dists, uint32_t *n,
                      uint64_t *counters);
/* Device pointers; queries are prepared padded float rows, query_bytes apart. */
int ngt_amd_qg_search_device(ngt_amd_index *index, const ngt_amd_qg_search_params *params,
                             const void *d_queries, uint64_t query_bytes, uint32_t nq,
                             const uint32_t *d_seeds, const uint64_t *d_seed_off, uint32_t *d_ids,
                             float *d_dists, uint32_t *d_n, uint64_t *d_counters, void *stream);

/* NGTQG form of the sharded search (BASELINE C5): as ngt_amd_sharded_search_device. */
int ngt_amd_sharded_qg_search_device(ngt_amd_shard_comm *comm, ngt_amd_index *index,
                                     const ngt_amd_qg_search_params *params, const void *d_queries,
                                     uint64_t query_bytes, uint32_t nq, const uint32_t *d_seeds,
                                     const uint64_t *d_seed_off, const uint32_t *id_offsets,
                                     uint32_t *d_out_ids, float *d_out_dists, uint32_t *d_out_n,
                                     void *stream);

/* The local codebooks ngtqg_quantize trains: the kmeansWithNGT restatement
 * (lib/NGT/Clustering.h:648-760, as NGTQ drives it, NGTQ/Quantizer.h:1802-1858)
 * over the first 1,600 objects of rows [nrows][dim] (row 0 the dummy slot);
 * local_out [dim/dsub][16][dsub]. */
int ngt_amd_qg_train_local_ngt(const float *rows, uint64_t nrows, uint32_t dim, uint32_t dsub, float *local_out);

/* ---- NGTQ IVF-ADC ------------------------------------------------------- *
 *   ngt_amd_ngtq_open          <- NGTQ::Index(path) (lib/NGT/NGTQ/Quantizer.h:2832-2836,
 *                                 QuantizerInstance::open :1520-1570): prf, global/
 *                                 (the global codebook, an NGT index), local-<i>/obj,
 *                                 ivt and the object list obj, loaded into HBM.
 *   ngt_amd_ngtq_set           <- the same state from host arrays; the index is
 *                                 the global codebook (rows/graph/tree set).
 *   ngt_amd_ngtq_search[_device] <- NGTQ::Index::search(object, objs, size,
 *                                 expansion, aggregationMode, epsilon) (:2877-2883)
 *                                 = QuantizerInstance::search (:2471-2549):
 *                                 searchGlobalCodebook (:2248-2262, linear when
 *                                 epsilon < 0 or >= FLT_MAX, the CLI's "-e -"),
 *                                 aggregateObjects* (:2266-2441) with the float-LUT
 *                                 ADC (:942-953), residual distances (:579-608,
 *                                 :1102-1153) or exact distances, refineDistance.
 * Float L2 indexes with 2-byte local ids; the cache and refine modes need a
 * subvector dimension that is a multiple of 8 (the reference reads whole
 * 8-float blocks). */
#define NGT_AMD_NGTQ_APPROXIMATE 0   /* AggregationModeApproximateDistance                */
#define NGT_AMD_NGTQ_LOOKUP_TABLE 1  /* AggregationModeApproximateDistanceWithLookupTable */
#define NGT_AMD_NGTQ_CACHE 2         /* AggregationModeApproximateDistanceWithCache       */
#define NGT_AMD_NGTQ_REFINE 3        /* AggregationModeExactDistanceThroughApproximateDistance */
#define NGT_AMD_NGTQ_EXACT 4         /* AggregationModeExactDistance                      */
typedef struct {
  uint32_t size;         /* results per query                                      */
  float expansion;       /* approximateSearchSize = size * expansion                */
  float epsilon;         /* global-codebook search; < 0 => linear search (FLT_MAX)  */
  int32_t mode;          /* NGT_AMD_NGTQ_*                                          */
} ngt_amd_ngtq_search_params;

int ngt_amd_ngtq_open(const char *path, int device, ngt_amd_index **out);
/* local: [N][16][dsub] local centroids (ids 1..16); list_off [nlists+1] CSR of
 * the inverted lists by global centroid id; eids [entries] object ids;
 * elids [entries][N] uint16 local ids (0 = the object is its centroid);
 * objects [object_records][dimension] floats (the object list, record 0 unused). */
int ngt_amd_ngtq_set(ngt_amd_index *index, const float *local, uint32_t N, uint32_t dsub,
                     const uint64_t *list_off, uint64_t nlists, const uint32_t *eids,
                     const uint16_t *elids, uint64_t nentries, const float *objects,
                     uint64_t object_records);
/* Host pointers; ids/dists [nq][size] ascending (distance, id), n [nq]. */
int ngt_amd_ngtq_search(ngt_amd_index *index, const ngt_amd_ngtq_search_params *params,
                        const float *queries, uint32_t nq, uint32_t *ids, float *dists, uint32_t *n);
/* Device pointers; queries are prepared padded float rows, query_bytes apart. */
int ngt_amd_ngtq_search_device(ngt_amd_index *index, const ngt_amd_ngtq_search_params *params,
                               const void *d_queries, uint64_t query_bytes, uint32_t nq,
                               uint32_t *d_ids, float *d_dists, uint32_t *d_n, void *stream);

#ifdef __cplusplus
}
#endif
#endif
