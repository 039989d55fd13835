// ngtq_harness.cpp -- golden-vector generator for the NGTQ IVF-ADC search path
// (runs only in the development container, linked against the reference
// library that oracle/ref.mk builds from /root/reference; never shipped, never
// run on the GPU box).  Only its output files are committed.
//
// For every "mode:size:expansion:epsilon" spec and query it records what
// NGTQ::Index::search (lib/NGT/NGTQ/Quantizer.h:2877-2883) returns, i.e.
// QuantizerInstance::search (:2471-2549): the global-codebook search, the
// aggregation over inverted lists (aggregateObjects* :2266-2441) with the
// float-LUT ADC (:942-953, LUT :683-706), the per-subspace residual distances
// (:1102-1153, :579-608) or exact distances, and the refinement (:2450-2460).
// Also the float LUT of createDistanceLookup for global centroids 1..3.
//
// build: oracle/ref.mk (target oracle/_ref/ngtq_harness).
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "NGT/NGTQ/Quantizer.h"

static void die(const char* m) {
  fprintf(stderr, "ngtq_harness: %s\n", m);
  exit(1);
}

int main(int argc, char** argv) {
  if (argc < 6) die("usage: ngtq_harness index queries.f32 nq dim outdir [mode:size:expansion:eps ...]");
  std::string path = argv[1];
  size_t nq = strtoul(argv[3], 0, 10), dim = strtoul(argv[4], 0, 10);
  std::string out = argv[5];
  std::vector<float> qs(nq * dim);
  {
    FILE* f = fopen(argv[2], "rb");
    if (!f || fread(qs.data(), 4, qs.size(), f) != qs.size()) die("cannot read queries");
    fclose(f);
  }
  NGTQ::Index index(path);
  NGTQ::Quantizer& quantizer = index.getQuantizer();
  NGTQ::QuantizedObjectDistance& qod = quantizer.getQuantizedObjectDistance();
  {
    FILE* fl = fopen((out + "/flut.bin").c_str(), "wb");
    for (size_t qi = 0; qi < nq; qi++) {
      std::vector<double> q(qs.begin() + qi * dim, qs.begin() + (qi + 1) * dim);
      NGT::Object* obj = index.allocateObject(q);
      for (size_t g = 1; g <= 3; g++) {
        NGTQ::QuantizedObjectDistance::DistanceLookupTable lut;
        qod.initialize(lut);
        qod.createDistanceLookup(*obj, g, lut);
        fwrite(lut.localDistanceLookup, sizeof(float), lut.size, fl);
      }
      index.deleteObject(obj);
    }
    fclose(fl);
  }
  for (int a = 6; a < argc; a++) {
    char mode;
    size_t size;
    float expansion, eps;
    if (sscanf(argv[a], "%c:%zu:%f:%f", &mode, &size, &expansion, &eps) != 4) die("bad spec");
    NGTQ::AggregationMode am;
    switch (mode) {
      case 'r': am = NGTQ::AggregationModeExactDistanceThroughApproximateDistance; break;
      case 'e': am = NGTQ::AggregationModeExactDistance; break;
      case 'l': am = NGTQ::AggregationModeApproximateDistanceWithLookupTable; break;
      case 'c': am = NGTQ::AggregationModeApproximateDistanceWithCache; break;
      case 'a': am = NGTQ::AggregationModeApproximateDistance; break;
      default: die("bad mode");
    }
    const double epsilon = eps < 0 ? FLT_MAX : eps;  // "-e -": linear global-codebook search
    std::string fn = out + "/search_" + argv[a] + ".bin";
    FILE* fs = fopen(fn.c_str(), "wb");
    for (size_t qi = 0; qi < nq; qi++) {
      std::vector<double> q(qs.begin() + qi * dim, qs.begin() + (qi + 1) * dim);
      NGT::Object* obj = index.allocateObject(q);
      NGT::ObjectDistances res;
      index.search(obj, res, size, expansion, am, epsilon);
      uint32_t n = res.size();
      fwrite(&n, 4, 1, fs);
      for (size_t i = 0; i < size; i++) {
        uint32_t id = i < n ? res[i].id : 0;
        float d = i < n ? res[i].distance : 0.0f;
        fwrite(&id, 4, 1, fs);
        fwrite(&d, 4, 1, fs);
      }
      index.deleteObject(obj);
    }
    fclose(fs);
  }
  return 0;
}
