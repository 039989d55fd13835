// Fixture harness (test infrastructure, built by oracle/ref.mk against the
// reference's headers): Index::AccuracyTable::getEpsilon (lib/NGT/Index.h:
// 293-346) for the AccuracyTable string of a prf file and each expected
// accuracy given, as ngtpy's search passes it (a float widened to double).
// Prints one line per accuracy: "<accuracy as float bits> <epsilon as float bits>".
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>

#include "NGT/Index.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <prf> <accuracy>...\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1]);
  std::string line, table;
  while (std::getline(f, line))
    if (line.compare(0, 14, "AccuracyTable\t") == 0) table = line.substr(14);
  NGT::Index::AccuracyTable t(table);
  for (int i = 2; i < argc; i++) {
    const float a = strtof(argv[i], nullptr);
    const float e = t.getEpsilon(a);
    uint32_t ab, eb;
    memcpy(&ab, &a, 4);
    memcpy(&eb, &e, 4);
    printf("%u %u\n", ab, eb);
  }
  return 0;
}
