// kmeans_harness.cpp -- test infrastructure (never shipped, never run on the
// GPU box): runs ngt_amd's restatement of NGT::Clustering::kmeansWithNGT
// (ngt_amd/csrc/kmeans_ngt.h) with the REFERENCE's own NGT search as the
// search callback, over a sample index built the way NGTQ builds a local
// codebook index (lib/NGT/NGTQ/Quantizer.h:1678-1719, local property
// :2041-2058: ANNG, E 10, batch 500, insertion coefficient 1.1, edge size for
// search 40; createIndex(objects, ids, range = -1) in the insertion batches of
// buildQuantizedObjects: 1000 then 600 objects).  It pins the host logic
// against the reference's local codebooks in tests/golden/*_qg.
// build: oracle/ref.mk (target oracle/_ref/kmeans_harness).
// usage: kmeans_harness <in.bin> <constraint 0|1>   in.bin: u32 n, u32 dim, n*dim f32
// prints the centroids, one per line.
#include <stdio.h>
#include <stdlib.h>

#include "NGT/Index.h"
#include "NGT/Clustering.h"
#include "kmeans_ngt.h"

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  uint32_t n = 0, dim = 0;
  if (!f || fread(&n, 4, 1, f) != 1 || fread(&dim, 4, 1, f) != 1) return 2;
  std::vector<std::vector<float>> vectors(n, std::vector<float>(dim));
  for (auto& v : vectors)
    if (fread(v.data(), 4, dim, f) != dim) return 2;
  fclose(f);
  NGT::Property p;
  p.setDefault();
  p.dimension = dim;
  p.objectType = NGT::Property::ObjectType::Float;
  p.distanceType = NGT::Property::DistanceType::DistanceTypeL2;
  p.indexType = NGT::Property::IndexType::GraphAndTree;
  p.graphType = NGT::Property::GraphType::GraphTypeANNG;
  p.edgeSizeForCreation = 10;
  p.edgeSizeForSearch = 40;
  p.batchSizeForCreation = argc > 4 ? atoi(argv[4]) : 200;  // lp.set(localProperty) restores the default 200 (the quantizer's local prf)
  p.insertionRadiusCoefficient = 1.1;
  NGT::Index index(p);
  NGT::GraphAndTreeIndex& g = static_cast<NGT::GraphAndTreeIndex&>(index.getIndex());
  size_t done = 0;
  for (size_t chunk : {(size_t)1000, (size_t)600}) {
    std::vector<std::pair<NGT::Object*, size_t>> objs;
    for (size_t i = done; i < done + chunk && i < n; i++) objs.push_back({index.allocateObject(vectors[i]), i + 1});
    if (objs.empty()) break;
    std::vector<NGT::Index::InsertionResult> ids;
    g.createIndex(objs, ids, -1.0f, 24);
    done += objs.size();
  }
  ngt_amd::kmeans::SearchFn search = [&](const std::vector<std::vector<float>>& qs, size_t size, float eps,
                                         std::vector<std::vector<std::pair<uint32_t, float>>>& out) {
    out.assign(qs.size(), {});
    for (size_t qi = 0; qi < qs.size(); qi++) {
      std::vector<float> qv = qs[qi];
      NGT::Object* q = index.allocateObject(qv);
      NGT::SearchContainer sc(*q);
      NGT::ObjectDistances res;
      sc.setResults(&res);
      sc.setEpsilon(eps);
      sc.setSize(size);
      index.search(sc);
      for (auto& r : res) out[qi].push_back({r.id, r.distance});
      index.deleteObject(q);
    }
    return true;
  };
  if (argc > 3 && std::string(argv[3]) == "save") {  // the sample index itself, for builder comparisons
    index.save(argv[5]);
    return 0;
  }
  if (argc > 3) {  // the reference's own Clustering::kmeansWithNGT on the same index
    NGT::Clustering clustering;
    clustering.epsilonFrom = 0.10;
    clustering.epsilonTo = 0.50;
    clustering.epsilonStep = 0.05;
    clustering.maximumIteration = 20;
    clustering.clusterSizeConstraint = atoi(argv[2]) != 0;
    std::vector<NGT::Clustering::Cluster> clusters;
    const double diff = clustering.kmeansWithNGT(index, 16, clusters);
    for (auto& c : clusters) {
      for (size_t i = 0; i < c.centroid.size(); i++) printf(i ? "\t%.9g" : "%.9g", c.centroid[i]);
      printf("\n");
    }
    fprintf(stderr, "diff %g\n", diff);
    return 0;
  }
  ngt_amd::kmeans::Params prm;
  prm.cluster_size_constraint = atoi(argv[2]) != 0;
  std::vector<std::vector<float>> cents;
  std::string err;
  const double diff = ngt_amd::kmeans::kmeans_with_ngt(search, vectors, 16, prm, cents, err);
  if (diff < 0) {
    fprintf(stderr, "%s\n", err.c_str());
    return 1;
  }
  for (auto& c : cents) {
    for (size_t i = 0; i < c.size(); i++) printf(i ? "\t%.9g" : "%.9g", c[i]);
    printf("\n");
  }
  fprintf(stderr, "diff %g\n", diff);
  return 0;
}
