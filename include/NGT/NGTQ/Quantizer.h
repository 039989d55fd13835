/*
 * NGT/NGTQ/Quantizer.h -- the NGTQ (IVF-ADC) search API of NGT 1.13.8
 * (NGTQ::AggregationMode, NGTQ::Index: lib/NGT/NGTQ/Quantizer.h:180-186,
 * 2819-2930) served by the MI355X build.  Header-only over the C ABI of
 * libngt_amd.so (include/ngt_amd.h, ngt_amd_ngtq_*): NGTQ::Index(path) loads
 * an index directory made by `ngtq create` into HBM, and
 * search(object, objs, size, expansion, aggregationMode, epsilon) runs the
 * global-codebook search and the inverted-list aggregation on the GPU.
 * Index construction (create/append/rebuild) is not part of this build.
 */
#ifndef NGT_AMD_CXX_NGTQ_QUANTIZER_H
#define NGT_AMD_CXX_NGTQ_QUANTIZER_H

#include <cfloat>
#include <string>
#include <vector>

#include "../../ngt_amd.h"
#include "../Index.h"

namespace NGTQ {

enum AggregationMode {
  AggregationModeApproximateDistance = NGT_AMD_NGTQ_APPROXIMATE,
  AggregationModeApproximateDistanceWithLookupTable = NGT_AMD_NGTQ_LOOKUP_TABLE,
  AggregationModeApproximateDistanceWithCache = NGT_AMD_NGTQ_CACHE,
  AggregationModeExactDistanceThroughApproximateDistance = NGT_AMD_NGTQ_REFINE,
  AggregationModeExactDistance = NGT_AMD_NGTQ_EXACT
};

class Index {
 public:
  Index() {}
  explicit Index(const std::string& index) { open(index); }
  ~Index() { close(); }
  Index(const Index&) = delete;
  Index& operator=(const Index&) = delete;

  void open(const std::string& index, int device = 0) {
    close();
    if (ngt_amd_ngtq_open(index.c_str(), device, &ix) != 0)
      throw NGT::Exception(std::string("NGTQ::Index::open: ") + ngt_amd_last_error());
    dimension = ngt_amd_index_padded_dimension(ix);
  }
  void close() {
    if (ix) ngt_amd_index_destroy(ix);
    ix = nullptr;
  }

  // Quantizer::allocateObject (Quantizer.h:2856-2862): the query as floats
  NGT::Object* allocateObject(std::vector<double>& obj) {
    NGT::Object* o = new NGT::Object();
    o->values.assign(obj.begin(), obj.end());
    return o;
  }
  NGT::Object* allocateObject(const std::vector<float>& obj) {
    NGT::Object* o = new NGT::Object();
    o->values = obj;
    return o;
  }
  void deleteObject(NGT::Object* object) { delete object; }

  // NGTQ::Index::search (Quantizer.h:2877-2883); epsilon >= FLT_MAX searches
  // the global codebook linearly (the CLI's "-e -")
  void search(NGT::Object* object, NGT::ObjectDistances& objs, size_t size, float expansion,
              AggregationMode aggregationMode, double epsilon) {
    if (!ix) throw NGT::Exception("NGTQ::Index: Not open.");
    ngt_amd_ngtq_search_params p;
    p.size = (uint32_t)size;
    p.expansion = expansion;
    p.epsilon = epsilon >= FLT_MAX ? -1.0f : (float)epsilon;
    p.mode = (int32_t)aggregationMode;
    std::vector<uint32_t> ids(size);
    std::vector<float> ds(size);
    uint32_t n = 0;
    if (ngt_amd_ngtq_search(ix, &p, object->values.data(), 1, ids.data(), ds.data(), &n) != 0)
      throw NGT::Exception(std::string("NGTQ::Index::search: ") + ngt_amd_last_error());
    objs.clear();
    for (uint32_t i = 0; i < n; i++) objs.push_back(NGT::ObjectDistance(ids[i], ds[i]));
  }

 private:
  ngt_amd_index* ix = nullptr;
  size_t dimension = 0;
};

}  // namespace NGTQ

#endif
