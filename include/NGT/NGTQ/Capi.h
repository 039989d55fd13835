/*
 * NGT/NGTQ/Capi.h -- the `ngtqg_*` C API of NGT 1.13.8 (lib/NGT/NGTQ/Capi.h:100-140,
 * lib/NGT/NGTQ/Capi.cpp:40-131), served by ngt_amd/csrc/qg_capi.cpp on the
 * MI355X path: the quantized graph, its uint8 lookup tables and the 4-bit ADC
 * run as HIP kernels (ngt_amd/csrc/qg_kernels.hip).
 *
 * Same names, argument types, defaults (ngtqg_initialize_query: size 20,
 * epsilon 0.03, result_expansion 3.0, radius FLT_MAX) and error convention
 * ("Capi : <func>() : Error: <what>" / "... parametor error: ...") as the
 * reference.  ngtqg_quantize (NGTQ/Capi.cpp:120-131 -> NGTQG::Index::quantize,
 * QuantizedGraph.h:456-475) trains the local codebooks, encodes every object
 * and builds the quantized graph on the device, and writes <index>/qg in the
 * reference's formats (qg/prf and the codebook prf files byte-identical to
 * the reference's; codebook indexes built by this library's ANNG
 * construction).  Its k-means is Lloyd's with exact assignment, not the
 * reference's kmeansWithNGT, so codebooks differ from the reference's own;
 * given a codebook, codes and quantized graph are the reference's.
 *
 * Extension (not in the reference): ngtqg_batch_search_index.
 */
#ifndef NGT_AMD_NGTQ_CAPI_H
#define NGT_AMD_NGTQ_CAPI_H

#ifdef __cplusplus
extern "C" {
#endif

#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>

#include "../Capi.h"

typedef void *NGTQGIndex;
typedef NGTError NGTQGError;

typedef struct {
  float *query;
  size_t size;             /* # of returned objects */
  float epsilon;
  float result_expansion;
  float radius;
} NGTQGQuery;

typedef struct {
  float dimension_of_subvector;
  size_t max_number_of_edges;
} NGTQGQuantizationParameters;

NGTQGIndex ngtqg_open_index(const char *, NGTError);
/* extension: NGTQG::Index(path, maxNoOfEdges) (QuantizedGraph.h:170-185) --
 * the quantized graph built at open keeps at most max_edges neighbours/node */
NGTQGIndex ngtqg_open_index_with_max_edges(const char *, uint32_t max_edges, NGTError);

void ngtqg_close_index(NGTQGIndex);

void ngtqg_initialize_quantization_parameters(NGTQGQuantizationParameters *);

bool ngtqg_quantize(const char *, NGTQGQuantizationParameters, NGTError);

void ngtqg_initialize_query(NGTQGQuery *);

bool ngtqg_search_index(NGTQGIndex, NGTQGQuery, NGTObjectDistances, NGTError);

/* Extension: nq queries ([nq][dim] floats) in one device batch, same
 * semantics as nq calls of ngtqg_search_index.  ids/dists: [nq][size],
 * n: [nq] entries written per query. */
bool ngtqg_batch_search_index(NGTQGIndex, const float *queries, uint32_t nq, int32_t dim, size_t size,
                              float epsilon, float result_expansion, float radius, uint32_t *ids,
                              float *dists, uint32_t *n, NGTError);

#ifdef __cplusplus
}
#endif
#endif
