/*
 * ngt_oracle.h -- CPU restatement of NGT 1.13.8's distance / search hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the *checker* for the HIP
 * product path in ngt_amd/.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product never links it and
 * never falls back to it.
 *
 * Every function restates the reference algorithm and cites the reference
 * file:line it follows (paths relative to the reference repository root).
 * The float reduction orders were read off the AVX-512 build of the
 * reference (`-Ofast -march=native`, objdump of
 * ObjectSpaceRepository<float,double>::Comparator*::operator()) and are pinned
 * bit-exactly by tests/golden (edge distances stored in reference-built
 * `grp` files).
 */
#ifndef NGT_ORACLE_H
#define NGT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* NGT::ObjectSpace::DistanceType (lib/NGT/ObjectSpace.h:166-180) */
enum {
  NGTO_L1 = 0, NGTO_L2 = 1, NGTO_HAMMING = 2, NGTO_ANGLE = 3, NGTO_COSINE = 4,
  NGTO_NORMALIZED_ANGLE = 5, NGTO_NORMALIZED_COSINE = 6, NGTO_JACCARD = 7,
  NGTO_SPARSE_JACCARD = 8, NGTO_NORMALIZED_L2 = 9, NGTO_POINCARE = 100,
  NGTO_LORENTZ = 101
};
/* NGT::ObjectSpace::ObjectType (lib/NGT/ObjectSpace.h:182-186) */
enum { NGTO_UINT8 = 1, NGTO_FLOAT = 2 };

/* One comparator call, returned as the float the callers store
 * (Distance = float, lib/NGT/Common.h:47).  a, b point at padded rows of
 * `dp` elements (zero padded, lib/NGT/ObjectSpace.h:392-397). */
float ngto_distance(int metric, int otype, const void *a, const void *b, size_t dp);

/* Batched form: out[i] = distance(query, rows + ids[i]*row_bytes). */
void ngto_distances(int metric, int otype, const void *query, const void *rows,
                    size_t row_bytes, const uint32_t *ids, size_t n, size_t dp,
                    float *out);

/* NGT::ObjectSpace::normalize (lib/NGT/ObjectSpace.h:251-266) on a float row. */
int ngto_normalize_f32(float *v, size_t dim);

/* NeighborhoodGraph::searchReadOnlyGraph<COMPARATOR, CHECK_LIST>
 * (lib/NGT/Graph.cpp:398-495) with setupDistances (:293-338) and setupSeeds
 * (:341-367).  Graph is CSR: edges of node v are edge_ids[edge_off[v] ..
 * edge_off[v+1]).  `edge_size` is the already-resolved getEdgeSize()
 * (lib/NGT/Graph.h:675-692; 0 or INT_MAX = unlimited).
 * Returns the number of results (<= k) written to out_ids/out_dists in
 * ascending (distance, id) order; counters[0] = distance computations,
 * counters[1] = visited edges, counters[2] = expansions. */
int ngto_search(int metric, int otype, const void *rows, size_t row_bytes,
                size_t nrows, size_t dp, const uint64_t *edge_off,
                const uint32_t *edge_ids, const void *query,
                const uint32_t *seeds, size_t nseeds, size_t k, float epsilon,
                float radius, size_t edge_size, uint32_t *out_ids,
                float *out_dists, uint64_t *counters);

/* ObjectSpaceRepository::linearSearch (lib/NGT/ObjectSpaceRepository.h:466-502):
 * all rows 1..nrows-1 whose valid[i] != 0 (valid may be NULL). */
int ngto_linear_search(int metric, int otype, const void *rows, size_t row_bytes,
                       size_t nrows, size_t dp, const uint8_t *valid,
                       const void *query, size_t k, double radius,
                       uint32_t *out_ids, float *out_dists);

/* glibc random(3) TYPE_3 restatement, used by getSeedsFromTree's
 * srand(leafID) thinning (lib/NGT/Index.h:1555-1561) and getRandomSeeds
 * (lib/NGT/Index.h:775-801). */
typedef struct { uint32_t s[31]; int f, r; } ngto_rand_t;
void ngto_srand(ngto_rand_t *g, unsigned seed);
int ngto_rand(ngto_rand_t *g);

/* GraphAndTreeIndex::getSeedsFromTree seed thinning (lib/NGT/Index.h:1548-1566):
 * seeds (leaf object ids, in leaf order) are thinned in place to
 * min(seed_size==0?k:seed_size, k) using srand(leaf_id).  Returns new count. */
size_t ngto_thin_seeds(uint32_t *seeds, size_t n, unsigned leaf_id,
                       size_t seed_size, size_t k);

/* DVPTree::search in SearchLeaf mode with radius 0 (lib/NGT/Tree.cpp:400-480,
 * 531-563).  Tree arrays: internal node i: pivot row `in_pivot + i*row_bytes`,
 * children in_child[i*5..], borders in_border[i*4..]; node ids follow
 * Node::ID (bit 31 = leaf).  root = raw ID of the root.  Returns the leaf's
 * raw node ID; *ndist gets the number of distance computations. */
uint32_t ngto_tree_leaf(int metric, int otype, const void *query, size_t dp,
                        uint32_t root, const void *in_pivot, size_t row_bytes,
                        const uint32_t *in_child, const float *in_border,
                        size_t children, uint64_t *ndist);

/* ---- NGTQG (quantized graph) -------------------------------------------- */
/* QuantizedObjectDistance::createDistanceLookup(Object&, id,
 * DistanceLookupTableUint8&) (lib/NGT/NGTQ/Quantizer.h:709-760) over
 * createFloatL2DistanceLookup (:683-706).  query/global: D floats; local:
 * [M][17][dsub] centroids (slot 0 unused, NGT object ids 1..16).  Writes
 * lut[Me*16] (Me = M rounded up to even; the pad subspace is zero), the one
 * scale and totalOffset used by the ADC. */
void ngto_qg_lut(const float *query, const float *global, const float *local, size_t M,
                 size_t dsub, uint8_t *lut, float *scale, float *total_offset);

/* QuantizedObjectDistanceFloat::operator()(void*, float*, size_t,
 * DistanceLookupTableUint8&) (Quantizer.h:957-1062, AVX-512 build): packed
 * 4-bit codes of n objects (ceil(n/16) blocks of 8*Me bytes) -> out[n]. */
void ngto_qg_adc(const uint8_t *codes, size_t n, const uint8_t *lut, size_t M, float scale,
                 float total_offset, float *out);

/* NGTQG::Index::searchQuantizedGraph (lib/NGT/NGTQ/QuantizedGraph.h:192-320)
 * for one query, given its seeds (getSeedsFromTree / getSeedsFromGraph
 * output, unsorted).  Quantized graph: node v has neighbours
 * qids[qoff[v]..qoff[v+1]) and codes at codes + code_off[v].  rows: exact f32
 * rows (padded dp) for seed distances and the rerank.  Returns the number of
 * entries written (k when expansion >= 1: the reference's resize pads with
 * {id 0, distance 0}); counters: [0] ADC distances, [1] accepted (visitCount
 * semantics of this loop), [2] expansions, [3] exact distances. */
int ngto_qg_search(const float *rows, size_t dp, size_t nrows, const uint64_t *qoff,
                   const uint32_t *qids, const uint64_t *code_off, const uint8_t *codes, size_t M,
                   const uint8_t *lut, float scale, float total_offset, const float *query,
                   const uint32_t *seeds, size_t nseeds, size_t k, float epsilon,
                   float result_expansion, float radius, uint32_t *out_ids, float *out_dists,
                   uint64_t *counters);

/* ---- query batches, one query per thread (OpenMP builds; bench.py's
 * cpu_baseline and parity sample).  Per query exactly the single-query
 * function above: ngto_search (ids/dists [nq][k], n [nq], counters [nq][3]),
 * ngto_linear_search, ngto_qg_search (outputs [nq][out_stride], counters
 * [nq][4]; luts [nq][lut_stride]).  Queries are padded rows query_bytes
 * apart (QG: dp floats apart); seeds CSR: seeds[seed_off[q] .. seed_off[q+1]). */
void ngto_search_batch(int metric, int otype, const void *rows, size_t row_bytes, size_t nrows, size_t dp,
                       const uint64_t *edge_off, const uint32_t *edge_ids, const void *queries,
                       size_t query_bytes, size_t nq, const uint32_t *seeds, const uint64_t *seed_off, size_t k,
                       float epsilon, float radius, size_t edge_size, uint32_t *out_ids, float *out_dists,
                       uint32_t *out_n, uint64_t *counters, int nthreads);
void ngto_linear_search_batch(int metric, int otype, const void *rows, size_t row_bytes, size_t nrows, size_t dp,
                              const void *queries, size_t query_bytes, size_t nq, size_t k, double radius,
                              uint32_t *out_ids, float *out_dists, uint32_t *out_n, int nthreads);
void ngto_qg_search_batch(const float *rows, size_t dp, size_t nrows, const uint64_t *qoff, const uint32_t *qids,
                          const uint64_t *code_off, const uint8_t *codes, size_t M, const uint8_t *luts,
                          size_t lut_stride, const float *scales, const float *offsets, const float *queries,
                          size_t nq, const uint32_t *seeds, const uint64_t *seed_off, size_t k, float epsilon,
                          float result_expansion, float radius, size_t out_stride, uint32_t *out_ids,
                          float *out_dists, uint32_t *out_n, uint64_t *counters, int nthreads);

/* NGTQ IVF-ADC: the aggregation of QuantizerInstance::search
 * (lib/NGT/NGTQ/Quantizer.h:2499-2549) for one query, given the
 * global-codebook search result (cent_ids/cent_d, ncent entries in order).
 * mode = NGTQ::AggregationMode: 0 approximate (getL2DistanceFloat :579-608),
 * 1 lookup table (createFloatL2DistanceLookup :683-706 + :942-953), 2 cache
 * (:1102-1153), 3 cache + refineDistance (:2450-2460), 4 exact.  grows /
 * orows: padded global-centroid / object-list rows (dp floats); local
 * [N][17][dsub] (slot 0 unused); inverted lists CSR by global id with N
 * uint16 local ids per entry.  Returns min(#aggregated, size) results in
 * ascending (distance, id). */
size_t ngto_ngtq_aggregate(int mode, const float *query, size_t dp, const uint32_t *cent_ids,
                           const float *cent_d, size_t ncent, const float *grows, const float *local, size_t N,
                           size_t dsub, const uint64_t *list_off, size_t nlists, const uint32_t *eids,
                           const uint16_t *elids, const float *orows, size_t size, uint64_t ass,
                           uint32_t *out_ids, float *out_d);
/* One residual term of mode 0/1/2 (float LUT entry as double for mode 1). */
double ngto_ngtq_term(int mode, const float *o, const float *g, const float *l, size_t dsub);

#ifdef __cplusplus
}
#endif
#endif
