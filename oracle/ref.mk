# Builds the reference NGT 1.13.8 from its own sources under /root/reference
# (read-only) into oracle/_ref/ -- test infrastructure only: it regenerates
# the golden fixtures under tests/golden/ and validates the oracle
# restatement.  Nothing here ships or runs on the GPU box.
#
#   make -f oracle/ref.mk            (from the repo root)
#
# Generated headers come from the reference's own generators: NGT/defines.h
# via CMake's configure_file on lib/NGT/defines.h.in (configure_defines.cmake,
# options at their OFF defaults) and NGT/version_defs.h via the reference's
# utils/mk_version_defs_h.sh.  Compiler flags follow CMakeLists.txt:54
# (-Ofast -march=native), so the AVX-512 comparator paths are the ones built,
# as in the survey's build.
REF ?= /root/reference
OUT ?= oracle/_ref
GEN = $(OUT)/gen
CXX ?= g++
CXXFLAGS = -Ofast -march=native -fopenmp -std=c++17 -fPIC -w -I$(GEN) -I$(GEN)/NGT -I$(REF)/lib
SRCS = $(wildcard $(REF)/lib/NGT/*.cpp) $(wildcard $(REF)/lib/NGT/NGTQ/*.cpp)
OBJS = $(patsubst $(REF)/lib/%.cpp,$(OUT)/obj/%.o,$(SRCS))

all: $(OUT)/libngt_ref.so $(OUT)/ngt $(OUT)/ngtq $(OUT)/ngtqg $(OUT)/qg_harness $(OUT)/ngtq_harness $(OUT)/comparator_harness $(OUT)/kmeans_harness $(OUT)/accuracy_harness

$(GEN)/NGT/defines.h: $(REF)/lib/NGT/defines.h.in oracle/configure_defines.cmake
	@mkdir -p $(GEN)/NGT
	cmake -DREF=$(REF) -DOUT=$(abspath $(GEN)) -P oracle/configure_defines.cmake

$(GEN)/NGT/version_defs.h: $(REF)/VERSION
	@mkdir -p $(GEN)/NGT
	cd $(REF) && sh utils/mk_version_defs_h.sh $(REF) $(abspath $(GEN))/NGT/version_defs.h

$(OUT)/obj/%.o: $(REF)/lib/%.cpp $(GEN)/NGT/defines.h $(GEN)/NGT/version_defs.h
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OUT)/libngt_ref.so: $(OBJS)
	$(CXX) -shared -fopenmp -o $@ $(OBJS) -lrt

$(OUT)/ngt: $(REF)/bin/ngt/ngt.cpp $(OUT)/libngt_ref.so
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(OUT) -lngt_ref -Wl,-rpath,$(abspath $(OUT))

$(OUT)/ngtqg: $(REF)/bin/ngtqg/ngtqg.cpp $(OUT)/libngt_ref.so
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(OUT) -lngt_ref -Wl,-rpath,$(abspath $(OUT))

# fixture harnesses (committed under tests/golden/, compiled against the reference headers)
$(OUT)/qg_harness: tests/golden/qg_harness.cpp $(OUT)/libngt_ref.so
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(OUT) -lngt_ref -Wl,-rpath,$(abspath $(OUT))

$(OUT)/comparator_harness: tests/golden/comparator_harness.cpp $(GEN)/NGT/defines.h
	$(CXX) $(CXXFLAGS) -o $@ $<

clean:
	rm -rf $(OUT)

$(OUT)/ngtq: $(REF)/bin/ngtq/ngtq.cpp $(OUT)/libngt_ref.so
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(OUT) -lngt_ref -Wl,-rpath,$(abspath $(OUT))

$(OUT)/ngtq_harness: tests/golden/ngtq_harness.cpp $(OUT)/libngt_ref.so
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(OUT) -lngt_ref -Wl,-rpath,$(abspath $(OUT))

$(OUT)/kmeans_harness: tests/golden/kmeans_harness.cpp ngt_amd/csrc/kmeans_ngt.h $(OUT)/libngt_ref.so
	$(CXX) $(CXXFLAGS) -Ingt_amd/csrc -o $@ $< -L$(OUT) -lngt_ref -Wl,-rpath,$(abspath $(OUT))

$(OUT)/accuracy_harness: tests/golden/accuracy_harness.cpp $(OUT)/libngt_ref.so
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(OUT) -lngt_ref -Wl,-rpath,$(abspath $(OUT))
