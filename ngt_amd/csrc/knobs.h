// Test and measurement knobs of libngt_amd.so.
//
// The library reads its NGT_AMD_* tuning variables only through knob(), and
// knob() answers only when NGT_AMD_TEST_KNOBS=1 is set as well: a stray
// variable in a caller's environment cannot change a kernel path of the
// drop-in library.  The tests set the master switch (tests/conftest.py); the
// table of knobs and what they force is DESIGN.md section 8.  NGT_AMD_DEVICE
// (the device a C-API index opens on) is a public setting, not a knob.
#pragma once

#include <cstdlib>

namespace ngt_amd {

inline bool test_knobs_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("NGT_AMD_TEST_KNOBS");
    return v != nullptr && std::atoi(v) != 0;
  }();
  return on;
}

inline const char* knob(const char* name) { return test_knobs_enabled() ? std::getenv(name) : nullptr; }

}  // namespace ngt_amd
