// comparator_harness.cpp -- golden-vector generator for the distance
// comparators and query normalization.  Test infrastructure only: compiled by
// oracle/ref.mk against the reference headers under /root/reference (never
// shipped, never run on the GPU box); only its output files are committed.
//
//   comparator_harness dist <metric> <f|c> <dp> <a.bin> <b.bin> <n> <out.f32>
//       out[i] = (float) PrimitiveComparator::<metric>(a[i], b[i], dp)
//       (lib/NGT/PrimitiveComparator.h:105-648; the value is stored as the
//       float NGT::Distance, Common.h:47, exactly as the search loop does)
//   comparator_harness normalize <dim> <in.f32> <n> <out.f32>
//       ObjectSpace::normalize (lib/NGT/ObjectSpace.h:251-266) of each row,
//       as allocateNormalizedObject applies it (ObjectSpaceRepository.h:560-566)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <typeinfo>
#include <vector>

#include "NGT/ObjectSpaceRepository.h"

using NGT::PrimitiveComparator;

static void die(const char* m) {
  fprintf(stderr, "comparator_harness: %s\n", m);
  exit(1);
}

static std::vector<char> slurp(const char* path, size_t bytes) {
  std::vector<char> v(bytes);
  FILE* f = fopen(path, "rb");
  if (!f || fread(v.data(), 1, bytes, f) != bytes) die(path);
  fclose(f);
  return v;
}

template <typename T>
static double dist(const std::string& m, const T* a, const T* b, size_t dp) {
  if (m == "l1") return PrimitiveComparator::compareL1(a, b, dp);
  if (m == "l2") return PrimitiveComparator::compareL2(a, b, dp);
  if (m == "angle") return PrimitiveComparator::compareAngleDistance(a, b, dp);
  if (m == "cosine") return PrimitiveComparator::compareCosineSimilarity(a, b, dp);
  if (m == "normalized_angle") return PrimitiveComparator::compareNormalizedAngleDistance(a, b, dp);
  if (m == "normalized_cosine") return PrimitiveComparator::compareNormalizedCosineSimilarity(a, b, dp);
  if (m == "normalized_l2") return PrimitiveComparator::compareNormalizedL2(a, b, dp);
  if (m == "dot") return PrimitiveComparator::compareDotProduct(a, b, dp);
  die(("metric " + m).c_str());
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) die("usage: see the header");
  const std::string mode = argv[1];
  if (mode == "dist") {
    if (argc != 9) die("dist <metric> <f|c> <dp> <a.bin> <b.bin> <n> <out.f32>");
    const std::string m = argv[2];
    const bool fl = argv[3][0] == 'f';
    const size_t dp = strtoul(argv[4], 0, 10), n = strtoul(argv[7], 0, 10);
    const size_t es = fl ? 4 : 1;
    std::vector<char> a = slurp(argv[5], n * dp * es), b = slurp(argv[6], n * dp * es);
    std::vector<float> out(n);
    for (size_t i = 0; i < n; i++) {
      double d;
      if (fl) {
        const float* x = reinterpret_cast<const float*>(a.data()) + i * dp;
        const float* y = reinterpret_cast<const float*>(b.data()) + i * dp;
        if (m == "sparse_jaccard") d = PrimitiveComparator::compareSparseJaccardDistance(x, y, dp);
        else if (m == "poincare") d = PrimitiveComparator::comparePoincareDistance(x, y, dp);
        else if (m == "lorentz") d = PrimitiveComparator::compareLorentzDistance(x, y, dp);
        else d = dist<float>(m, x, y, dp);
      } else {
        const uint8_t* x = reinterpret_cast<const uint8_t*>(a.data()) + i * dp;
        const uint8_t* y = reinterpret_cast<const uint8_t*>(b.data()) + i * dp;
        if (m == "hamming") d = PrimitiveComparator::compareHammingDistance(x, y, dp);
        else if (m == "jaccard") d = PrimitiveComparator::compareJaccardDistance(x, y, dp);
        else d = dist<uint8_t>(m, x, y, dp);
      }
      out[i] = static_cast<float>(d);
    }
    FILE* f = fopen(argv[8], "wb");
    if (!f || fwrite(out.data(), 4, n, f) != n) die(argv[8]);
    fclose(f);
    return 0;
  }
  if (mode == "normalize") {
    if (argc != 6) die("normalize <dim> <in.f32> <n> <out.f32>");
    const size_t dim = strtoul(argv[2], 0, 10), n = strtoul(argv[4], 0, 10);
    std::vector<char> in = slurp(argv[3], n * dim * 4);
    std::vector<float> rows(reinterpret_cast<float*>(in.data()), reinterpret_cast<float*>(in.data()) + n * dim);
    NGT::ObjectSpaceRepository<float, double> os(dim, typeid(float), NGT::ObjectSpace::DistanceTypeNormalizedCosine);
    NGT::ObjectSpace& base = os;  // the template ObjectSpace::normalize(T*, size_t)
    for (size_t i = 0; i < n; i++) base.normalize(rows.data() + i * dim, dim);
    FILE* f = fopen(argv[5], "wb");
    if (!f || fwrite(rows.data(), 4, n * dim, f) != n * dim) die(argv[5]);
    fclose(f);
    return 0;
  }
  die("unknown mode");
  return 1;
}
