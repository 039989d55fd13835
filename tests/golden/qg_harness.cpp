// qg_harness.cpp -- golden-vector generator for the NGTQG path (runs only in the
// development container, against the reference library built in /tmp/ngt-build;
// never shipped, never run on the GPU box).  Only its output files are committed.
//
// For every query it records what NGTQG::Index::searchQuantizedGraph
// (lib/NGT/NGTQ/QuantizedGraph.h:192-320) computes:
//   * the uint8 distance LUT, scales[0] and totalOffset built by
//     QuantizedObjectDistance::createDistanceLookup (Quantizer.h:709-760),
//   * ADC distances of the packed neighbour codes of a few nodes
//     (QuantizedObjectDistanceFloat::operator(), Quantizer.h:957-1062),
//   * final search results of NGTQG::Index::search for (k, epsilon, expansion)
//     triples (the path ngtqg_search_index takes, NGTQ/Capi.cpp:69-83).
//
// build: see make_qg_goldens.py (g++ with the reference's own flags).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "NGT/NGTQ/QuantizedGraph.h"

static void die(const char* m) {
  fprintf(stderr, "qg_harness: %s\n", m);
  exit(1);
}

int main(int argc, char** argv) {
  if (argc < 7) die("usage: qg_harness index queries.f32 nq dim outdir nodes.u32 [k:eps:exp ...]");
  std::string path = argv[1];
  size_t nq = strtoul(argv[3], 0, 10), dim = strtoul(argv[4], 0, 10);
  std::string out = argv[5];
  std::vector<float> qs(nq * dim);
  {
    FILE* f = fopen(argv[2], "rb");
    if (!f || fread(qs.data(), 4, qs.size(), f) != qs.size()) die("cannot read queries");
    fclose(f);
  }
  std::vector<uint32_t> nodes;
  {
    FILE* f = fopen(argv[6], "rb");
    if (!f) die("cannot read nodes");
    uint32_t v;
    while (fread(&v, 4, 1, f) == 1) nodes.push_back(v);
    fclose(f);
  }

  NGTQG::Index index(path);
  NGTQ::Quantizer& quantizer = index.quantizedIndex.getQuantizer();
  NGTQ::QuantizedObjectDistance& qod = quantizer.getQuantizedObjectDistance();
  size_t M = quantizer.divisionNo;
  size_t Me = ((M - 1) / 2 + 1) * 2;

  FILE* flut = fopen((out + "/lut.bin").c_str(), "wb");
  FILE* fsc = fopen((out + "/scale.bin").c_str(), "wb");
  FILE* fadc = fopen((out + "/adc.bin").c_str(), "wb");
  for (size_t qi = 0; qi < nq; qi++) {
    std::vector<float> q(qs.begin() + qi * dim, qs.begin() + (qi + 1) * dim);
    NGT::Object* obj = index.allocateObject(q);
    NGTQ::QuantizedObjectDistance::DistanceLookupTableUint8 lut;
    qod.initialize(lut);
    qod.createDistanceLookup(*obj, 1, lut);
    fwrite(lut.localDistanceLookup, 1, Me * 16, flut);
    float sc[2] = {lut.scales[0], lut.totalOffset};
    fwrite(sc, 4, 2, fsc);
    for (uint32_t id : nodes) {
      size_t n = index.quantizedGraph.getIDs(id).size();
      std::vector<float> ds(n + NGTQ_SIMD_BLOCK_SIZE, 0.0f);
      if (n > 0) qod(index.quantizedGraph.get(id), ds.data(), n, lut);
      fwrite(ds.data(), 4, n, fadc);
    }
    index.deleteObject(obj);
  }
  fclose(flut);
  fclose(fsc);
  fclose(fadc);

  for (int a = 7; a < argc; a++) {
    size_t k;
    float eps, exp;
    if (sscanf(argv[a], "%zu:%f:%f", &k, &eps, &exp) != 3) die("bad k:eps:exp");
    std::string fn = out + "/search_" + argv[a] + ".bin";
    FILE* fs = fopen(fn.c_str(), "wb");
    for (size_t qi = 0; qi < nq; qi++) {
      std::vector<float> q(qs.begin() + qi * dim, qs.begin() + (qi + 1) * dim);
      NGT::ObjectDistances res;
      NGTQG::SearchQuery sq(q);
      sq.setResults(&res);
      sq.setSize(k);
      sq.setRadius(FLT_MAX);
      sq.setEpsilon(eps);
      sq.setResultExpansion(exp);
      index.search(sq);
      uint32_t n = res.size();
      fwrite(&n, 4, 1, fs);
      for (size_t i = 0; i < k; i++) {
        uint32_t id = i < n ? res[i].id : 0;
        float d = i < n ? res[i].distance : 0.0f;
        fwrite(&id, 4, 1, fs);
        fwrite(&d, 4, 1, fs);
      }
    }
    fclose(fs);
  }
  return 0;
}
