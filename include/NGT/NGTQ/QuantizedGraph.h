/*
 * NGT/NGTQ/QuantizedGraph.h -- the NGTQG C++ API of NGT 1.13.8
 * (NGTQG::SearchContainer, NGTQG::SearchQuery, NGTQG::Index;
 * lib/NGT/NGTQ/QuantizedGraph.h:27-39, 168-185, 354-372, 456-475) served by the
 * MI355X build.  Header-only over the C ABI of libngt_amd.so
 * (include/NGT/NGTQ/Capi.h): the quantized-graph search
 * (NGTQG::Index::search(SearchQuery&) -> getSeedsFromTree +
 * searchQuantizedGraph) runs on the GPU; NGTQG::Index also is an NGT::Index
 * over the same directory, so exact searches work on it as well.
 */
#ifndef NGT_AMD_CXX_QUANTIZED_GRAPH_H
#define NGT_AMD_CXX_QUANTIZED_GRAPH_H

#include <string>
#include <vector>

#include "../Index.h"
#include "Capi.h"

namespace NGTQG {

// QuantizedGraph.h:27-35 (the reference leaves resultExpansion unset by the
// default constructor; the C API's default is 3.0, NGTQ/Capi.cpp:40-46)
class SearchContainer : public NGT::SearchContainer {
 public:
  SearchContainer() : resultExpansion(3.0f) {}
  explicit SearchContainer(NGT::Object& f) : NGT::SearchContainer(f), resultExpansion(3.0f) {}
  void setResultExpansion(float re) { resultExpansion = re; }
  float resultExpansion;
};

class SearchQuery : public NGT::QueryContainer, public NGTQG::SearchContainer {
 public:
  template <typename QTYPE>
  explicit SearchQuery(const std::vector<QTYPE>& q) : NGT::QueryContainer(q) {}
};

class Index : public NGT::Index {
 public:
  // NGTQG::Index(indexPath, maxNoOfEdges) (QuantizedGraph.h:168-185): opens
  // <index>/qg and loads qg/grp, or constructs the quantized graph keeping at
  // most maxNoOfEdges neighbours per node
  explicit Index(const std::string& indexPath, size_t maxNoOfEdges = 128) : NGT::Index(indexPath, false) {
    NGT::detail::Err err;
    qg = ngtqg_open_index_with_max_edges(indexPath.c_str(), (uint32_t)maxNoOfEdges, err);
    if (qg == nullptr) err.raise("NGTQG::Index::Index");
  }
  ~Index() override {
    if (qg) ngtqg_close_index(qg);
  }

  // NGTQG::Index::search(SearchQuery&) (QuantizedGraph.h:354-372)
  void search(NGTQG::SearchQuery& sq) {
    NGT::ObjectDistances& out = sq.getResult();
    out.clear();
    std::vector<float> q(sq.getQueryValues());
    NGTQGQuery query;
    ngtqg_initialize_query(&query);
    query.query = q.data();
    query.size = sq.size;
    query.epsilon = (float)((double)sq.explorationCoefficient - 1.0);
    query.result_expansion = sq.resultExpansion;
    query.radius = sq.radius;
    NGT::detail::Err err;
    NGTObjectDistances r = ngt_create_empty_results(err);
    if (!ngtqg_search_index(qg, query, r, err)) {
      ngt_destroy_results(r);
      err.raise("NGTQG::Index::search");
    }
    const uint32_t n = ngt_get_result_size(r, err);
    for (uint32_t i = 0; i < n; i++) {
      NGTObjectDistance d = ngt_get_result(r, i, err);
      out.push_back(NGT::ObjectDistance(d.id, d.distance));
    }
    ngt_destroy_results(r);
  }
  using NGT::Index::search;

  // NGTQG::Index::quantize (QuantizedGraph.h:456-475): codebooks, codes and
  // the quantized graph of the index at indexPath, written to <index>/qg
  static void quantize(const std::string& indexPath, float dimensionOfSubvector, size_t maxNumberOfEdges) {
    NGTQGQuantizationParameters p;
    ngtqg_initialize_quantization_parameters(&p);
    p.dimension_of_subvector = dimensionOfSubvector;
    p.max_number_of_edges = maxNumberOfEdges;
    NGT::detail::Err err;
    if (!ngtqg_quantize(indexPath.c_str(), p, err)) err.raise("NGTQG::Index::quantize");
  }

 private:
  NGTQGIndex qg = nullptr;
};

}  // namespace NGTQG

#endif
