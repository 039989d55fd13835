/*
 * NGT/Capi.h -- the `ngt_*` C API of NGT 1.13.8 (lib/NGT/Capi.h:27-212),
 * served by the MI355X-native implementation in ngt_amd/csrc/capi.cpp.
 *
 * Names, argument order and types, handle ownership and the error convention
 * (false / NULL / 0 plus "Capi : <func>() : Error: <what>" in the NGTError
 * string, lib/NGT/Capi.cpp:25-38) are those of the reference, so a program or
 * binding written against libngt links against libngt_amd.so unchanged for
 * the paths this build implements (open / create / append / ANNG construction
 * / search / linear search / object access / save / properties / results /
 * errors).  Graph-maintenance entry points (remove, optimizer, refine) are
 * declared for link compatibility and report an error (out of scope).
 *
 * Threading: any number of threads may search one handle concurrently, as with
 * the reference (Capi.cpp:377-406).  Concurrent single-query calls with equal
 * parameters are coalesced into one device launch (ngt_amd/csrc/coalesce.h;
 * NGT_AMD_COALESCE=0 turns it off).  Appends, inserts and ngt_create_index on a
 * handle are serialized against its searches (a reader/writer lock: a write
 * waits for the searches in flight, later searches wait for the write and see
 * its objects); the reference itself leaves writes concurrent with searches
 * undefined.
 *
 * Extensions (not in the reference): ngt_batch_search_index*,
 * ngt_get_last_search_counters, ngt_get_coalesce_stats, ngt_get_device_index.
 */
#ifndef NGT_AMD_CAPI_H
#define NGT_AMD_CAPI_H

#ifdef __cplusplus
extern "C" {
#endif

#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int ObjectID;
typedef void *NGTIndex;
typedef void *NGTProperty;
typedef void *NGTObjectSpace;
typedef void *NGTObjectDistances;
typedef void *NGTError;
typedef void *NGTOptimizer;

typedef struct {
  ObjectID id;
  float distance;
} NGTObjectDistance;

typedef struct {
  float *query;
  size_t size;      /* number of results */
  float epsilon;
  float accuracy;   /* expected accuracy (unused by ngt_search_index_with_query, as in the reference) */
  float radius;
  size_t edge_size; /* edges explored per node */
} NGTQuery;

typedef struct {
  size_t no_of_queries;
  size_t no_of_results;
  size_t no_of_threads;
  float target_accuracy;
  size_t target_no_of_objects;
  size_t no_of_sample_objects;
  size_t max_of_no_of_edges;
  bool log;
} NGTAnngEdgeOptimizationParameter;

NGTIndex ngt_open_index(const char *, NGTError);
NGTIndex ngt_create_graph_and_tree(const char *, NGTProperty, NGTError);
NGTIndex ngt_create_graph_and_tree_in_memory(NGTProperty, NGTError);
NGTProperty ngt_create_property(NGTError);
bool ngt_save_index(const NGTIndex, const char *, NGTError);
bool ngt_get_property(const NGTIndex, NGTProperty, NGTError);
int32_t ngt_get_property_dimension(NGTProperty, NGTError);
bool ngt_set_property_dimension(NGTProperty, int32_t, NGTError);
bool ngt_set_property_edge_size_for_creation(NGTProperty, int16_t, NGTError);
bool ngt_set_property_edge_size_for_search(NGTProperty, int16_t, NGTError);
int32_t ngt_get_property_object_type(NGTProperty, NGTError);
bool ngt_is_property_object_type_float(int32_t);
bool ngt_is_property_object_type_integer(int32_t);
bool ngt_set_property_object_type_float(NGTProperty, NGTError);
bool ngt_set_property_object_type_integer(NGTProperty, NGTError);
bool ngt_set_property_distance_type_l1(NGTProperty, NGTError);
bool ngt_set_property_distance_type_l2(NGTProperty, NGTError);
bool ngt_set_property_distance_type_angle(NGTProperty, NGTError);
bool ngt_set_property_distance_type_hamming(NGTProperty, NGTError);
bool ngt_set_property_distance_type_jaccard(NGTProperty, NGTError);
bool ngt_set_property_distance_type_cosine(NGTProperty, NGTError);
bool ngt_set_property_distance_type_normalized_angle(NGTProperty, NGTError);
bool ngt_set_property_distance_type_normalized_cosine(NGTProperty, NGTError);
NGTObjectDistances ngt_create_empty_results(NGTError);
bool ngt_search_index(NGTIndex, double *, int32_t, size_t, float, float, NGTObjectDistances, NGTError);
bool ngt_search_index_as_float(NGTIndex, float *, int32_t, size_t, float, float, NGTObjectDistances, NGTError);
bool ngt_search_index_with_query(NGTIndex, NGTQuery, NGTObjectDistances, NGTError);
bool ngt_linear_search_index(NGTIndex, double *, int32_t, size_t, NGTObjectDistances, NGTError);
bool ngt_linear_search_index_as_float(NGTIndex, float *, int32_t, size_t, NGTObjectDistances, NGTError);
bool ngt_linear_search_index_with_query(NGTIndex, NGTQuery, NGTObjectDistances, NGTError);
int32_t ngt_get_size(NGTObjectDistances, NGTError); /* deprecated */
uint32_t ngt_get_result_size(NGTObjectDistances, NGTError);
NGTObjectDistance ngt_get_result(const NGTObjectDistances, const uint32_t, NGTError);
ObjectID ngt_insert_index(NGTIndex, double *, uint32_t, NGTError);
ObjectID ngt_append_index(NGTIndex, double *, uint32_t, NGTError);
ObjectID ngt_insert_index_as_float(NGTIndex, float *, uint32_t, NGTError);
ObjectID ngt_append_index_as_float(NGTIndex, float *, uint32_t, NGTError);
bool ngt_batch_append_index(NGTIndex, float *, uint32_t, NGTError);
bool ngt_batch_insert_index(NGTIndex, float *, uint32_t, uint32_t *, NGTError);
bool ngt_create_index(NGTIndex, uint32_t, NGTError);
bool ngt_remove_index(NGTIndex, ObjectID, NGTError);
NGTObjectSpace ngt_get_object_space(NGTIndex, NGTError);
float *ngt_get_object_as_float(NGTObjectSpace, ObjectID, NGTError);
uint8_t *ngt_get_object_as_integer(NGTObjectSpace, ObjectID, NGTError);
void ngt_destroy_results(NGTObjectDistances);
void ngt_destroy_property(NGTProperty);
void ngt_close_index(NGTIndex);
int16_t ngt_get_property_edge_size_for_creation(NGTProperty, NGTError);
int16_t ngt_get_property_edge_size_for_search(NGTProperty, NGTError);
int32_t ngt_get_property_distance_type(NGTProperty, NGTError);
NGTError ngt_create_error_object(void);
const char *ngt_get_error_string(const NGTError);
void ngt_clear_error_string(NGTError);
void ngt_destroy_error_object(NGTError);
NGTOptimizer ngt_create_optimizer(bool logDisabled, NGTError);
bool ngt_optimizer_adjust_search_coefficients(NGTOptimizer, const char *, NGTError);
bool ngt_optimizer_execute(NGTOptimizer, const char *, const char *, NGTError);
bool ngt_optimizer_set(NGTOptimizer optimizer, int outgoing, int incoming, int nofqs,
                       float baseAccuracyFrom, float baseAccuracyTo, float rateAccuracyFrom,
                       float rateAccuracyTo, double gte, double m, NGTError error);
bool ngt_optimizer_set_minimum(NGTOptimizer optimizer, int outgoing, int incoming, int nofqs,
                               int nofrs, NGTError error);
bool ngt_optimizer_set_extension(NGTOptimizer optimizer, float baseAccuracyFrom,
                                 float baseAccuracyTo, float rateAccuracyFrom, float rateAccuracyTo,
                                 double gte, double m, NGTError error);
bool ngt_optimizer_set_processing_modes(NGTOptimizer optimizer, bool searchParameter,
                                        bool prefetchParameter, bool accuracyTable, NGTError error);
void ngt_destroy_optimizer(NGTOptimizer);
bool ngt_refine_anng(NGTIndex index, float epsilon, float expectedAccuracy, int noOfEdges,
                     int edgeSize, size_t batchSize, NGTError error);
bool ngt_get_edges(NGTIndex index, ObjectID id, NGTObjectDistances edges, NGTError error);
uint32_t ngt_get_object_repository_size(NGTIndex index, NGTError error);
NGTAnngEdgeOptimizationParameter ngt_get_anng_edge_optimization_parameter(void);
bool ngt_optimize_number_of_edges(const char *indexPath, NGTAnngEdgeOptimizationParameter parameter,
                                  NGTError error);

/* ---- extensions: distance types the reference sets only through the C++
 * NGT::Property (ngtpy.cpp:79-94 "Normalized L2"; SparseJaccard, Index.cpp:488-490) */
bool ngt_set_property_distance_type_normalized_l2(NGTProperty, NGTError);
bool ngt_set_property_distance_type_sparse_jaccard(NGTProperty, NGTError);

/* ---- extensions: any NGT::Property field by its prf key (PropertySet,
 * Common.h:573-666; keys of Index.h:105-261 and Graph.h:423-489), the way the
 * C++ facade (include/NGT/Index.h) reads and writes NGT::Property ------- */
bool ngt_set_property_value(NGTProperty, const char *key, const char *value, NGTError);
/* value into buf (truncated to len - 1 chars); returns its full length, -1 if absent */
int32_t ngt_get_property_value(NGTProperty, const char *key, char *buf, size_t len, NGTError);

/* ---- extensions: batched device search ---------------------------------- */
/* queries: [nq][dim] floats.  ids/dists: [nq][size], n: [nq] (results per query). */
bool ngt_batch_search_index(NGTIndex, const float *queries, uint32_t nq, int32_t dim, size_t size,
                            float epsilon, float radius, int64_t edge_size, uint32_t *ids,
                            float *dists, uint32_t *n, NGTError);
/* seeds from the process-wide rand() stream instead of the tree (searchUsingOnlyGraph) */
bool ngt_batch_search_index_using_only_graph(NGTIndex, const float *queries, uint32_t nq,
                                             int32_t dim, size_t size, float epsilon, float radius,
                                             int64_t edge_size, uint32_t *ids, float *dists,
                                             uint32_t *n, NGTError);
bool ngt_batch_linear_search_index(NGTIndex, const float *queries, uint32_t nq, int32_t dim,
                                   size_t size, uint32_t *ids, float *dists, uint32_t *n, NGTError);
/* as above with SearchContainer::radius (< 0: unbounded), the form ngtpy's
 * linear_search uses (ngtpy.cpp:236-242) */
bool ngt_batch_linear_search_index_with_radius(NGTIndex, const float *queries, uint32_t nq,
                                               int32_t dim, size_t size, float radius, uint32_t *ids,
                                               float *dists, uint32_t *n, NGTError);
/* counters of this thread's last search on this handle, summed over its
 * queries, with the reference's read-write SearchContainer semantics
 * (Graph.cpp:588-604): [0] distanceComputationCount (neighbour distances; the
 * seeds' are not counted), [1] visitCount (edges scanned), [2] expansions */
bool ngt_get_last_search_counters(NGTIndex, uint64_t *counters3, NGTError);
/* single-query calls served so far: device launches issued and queries served
 * by them (served / batches = mean coalesced batch size) */
bool ngt_get_coalesce_stats(NGTIndex, uint64_t *batches, uint64_t *served, NGTError);
/* the device-resident index (an ngt_amd_index *, include/ngt_amd.h) serving
 * this handle, built or refreshed from the host mirror on the call: for
 * batched device-pointer searches on an index opened or built through this
 * API.  Owned by the handle; valid until the next write to it or its close. */
void *ngt_get_device_index(NGTIndex, NGTError);

#ifdef __cplusplus
}
#endif
#endif
