// ngt_sample.cpp -- a program written against the reference's C++ API in the
// style of samples/cosine-float/cosine-float.cpp:17-100 (create -> append ->
// createIndex -> save, then open -> SearchQuery -> search -> getObject),
// compiled against include/ and linked with libngt_amd.so.  Test
// infrastructure: tests/test_cxx_api.py builds it and compares its output
// with the reference's own results and with the oracle.
//
//   ngt_sample create <index> <data.tsv> <dim> <L2|Cosine|...> [edgeSizeForSearch]
//   ngt_sample search <index> <queries.tsv> <k> <epsilon> [graph]
//   ngt_sample linear <index> <queries.tsv> <k>
//   ngt_sample qg <index> <queries.tsv> <k> <epsilon> <expansion>
//   ngt_sample accuracy <index> <expected accuracy>
// Output lines: "<query> <rank> <id> <distance bits as hex>" then, per query,
// "# <query> distances=<distanceComputationCount>".
#include <cfloat>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "NGT/Index.h"
#include "NGT/NGTQ/QuantizedGraph.h"
#include "NGT/NGTQ/Quantizer.h"

using namespace std;

static vector<vector<float>> read_tsv(const string& path, size_t dim) {
  vector<vector<float>> out;
  ifstream is(path);
  string line;
  while (getline(is, line)) {
    vector<float> v;
    stringstream ls(line);
    float x;
    while (ls >> x) v.push_back(x);
    if (v.empty()) continue;
    v.resize(dim);
    out.push_back(v);
  }
  return out;
}

static void print(size_t qi, const NGT::ObjectDistances& r) {
  for (size_t i = 0; i < r.size(); i++) {
    uint32_t bits;
    memcpy(&bits, &r[i].distance, 4);
    printf("%zu %zu %u %08x\n", qi, i + 1, r[i].id, bits);
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    cerr << "usage: see the header" << endl;
    return 2;
  }
  const string mode = argv[1], path = argv[2];
  try {
    if (mode == "create") {
      NGT::Property property;
      property.dimension = atoi(argv[4]);
      property.objectType = NGT::ObjectSpace::ObjectType::Float;
      property.distanceType = NGT::Property::distanceOf(argv[5]);
      if (argc > 6) property.edgeSizeForSearch = atoi(argv[6]);  // `ngt create -S` (default 40 there)
      NGT::Index::create(path, property);
      NGT::Index index(path);
      for (auto& obj : read_tsv(argv[3], property.dimension)) index.append(obj);
      index.createIndex(16);
      index.save();
      printf("objects %zu\n", index.getObjectRepositorySize() - 1);
      return 0;
    }
    if (mode == "accuracy") {
      NGT::Index index(path);
      printf("%.9g\n", index.getEpsilonFromExpectedAccuracy(atof(argv[3])));
      return 0;
    }
    if (mode == "ngtq") {
      // the `ngtq search` flow (NGTQCommand.h:272-420): allocateObject, then
      // NGTQ::Index::search(object, objects, size, expansion, mode, epsilon)
      NGTQ::Index index(path);
      auto queries = read_tsv(argv[3], 128);
      const char m = argv[6][0];
      NGTQ::AggregationMode am = m == 'r'   ? NGTQ::AggregationModeExactDistanceThroughApproximateDistance
                                 : m == 'e' ? NGTQ::AggregationModeExactDistance
                                 : m == 'l' ? NGTQ::AggregationModeApproximateDistanceWithLookupTable
                                 : m == 'c' ? NGTQ::AggregationModeApproximateDistanceWithCache
                                            : NGTQ::AggregationModeApproximateDistance;
      const double epsilon = string(argv[7]) == "-" ? FLT_MAX : atof(argv[7]);
      for (size_t qi = 0; qi < queries.size(); qi++) {
        std::vector<double> q(queries[qi].begin(), queries[qi].end());
        NGT::Object* query = index.allocateObject(q);
        NGT::ObjectDistances objects;
        index.search(query, objects, atoi(argv[4]), (float)atof(argv[5]), am, epsilon);
        print(qi, objects);
        index.deleteObject(query);
      }
      return 0;
    }
    if (mode == "qg") {
      NGTQG::Index index(path);
      NGT::Property property;
      index.getProperty(property);
      auto queries = read_tsv(argv[3], property.dimension);
      for (size_t qi = 0; qi < queries.size(); qi++) {
        NGTQG::SearchQuery sq(queries[qi]);
        NGT::ObjectDistances objects;
        sq.setResults(&objects);
        sq.setSize(atoi(argv[4]));
        sq.setEpsilon(atof(argv[5]));
        sq.setResultExpansion(atof(argv[6]));
        index.search(sq);
        print(qi, objects);
      }
      return 0;
    }
    NGT::Index index(path);
    NGT::Property property;
    index.getProperty(property);
    auto queries = read_tsv(argv[3], property.dimension);
    for (size_t qi = 0; qi < queries.size(); qi++) {
      NGT::ObjectDistances objects;
      if (mode == "linear") {
        NGT::SearchQuery sq(queries[qi]);
        sq.setResults(&objects);
        sq.setSize(atoi(argv[4]));
        index.linearSearch(sq);
      } else if (argc > 6 && string(argv[6]) == "graph") {
        // the SearchContainer form: an allocated object, graph-only seeds
        NGT::Object* query = index.allocateObject(queries[qi]);
        NGT::SearchContainer sc(*query);
        sc.setResults(&objects);
        sc.setSize(atoi(argv[4]));
        sc.setEpsilon(atof(argv[5]));
        index.searchUsingOnlyGraph(sc);
        index.deleteObject(query);
      } else {
        NGT::SearchQuery sq(queries[qi]);
        sq.setResults(&objects);
        sq.setSize(atoi(argv[4]));
        sq.setEpsilon(atof(argv[5]));
        index.search(sq);
        printf("# %zu distances=%zu\n", qi, sq.distanceComputationCount);
      }
      print(qi, objects);
      // getObjectSpace().getObject: the borrowed row of the first result
      if (!objects.empty()) {
        float* o = static_cast<float*>(index.getObjectSpace().getObject(objects[0].id));
        uint32_t bits;
        memcpy(&bits, &o[0], 4);
        printf("@ %zu %08x\n", qi, bits);
      }
    }
  } catch (NGT::Exception& err) {
    cerr << "Error " << err.what() << endl;
    return 1;
  }
  return 0;
}
