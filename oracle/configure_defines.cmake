# Generates NGT/defines.h from the reference's lib/NGT/defines.h.in with
# CMake's own configure_file -- exactly what lib/NGT/CMakeLists.txt:3 does --
# with every #cmakedefine option at its default (unset = OFF:
# NGT_SHARED_MEMORY_ALLOCATOR OFF per lib/NGT/CMakeLists.txt:2).
# Usage: cmake -DREF=/root/reference -DOUT=<dir> -P configure_defines.cmake
if(NOT DEFINED REF OR NOT DEFINED OUT)
  message(FATAL_ERROR "pass -DREF=<reference root> -DOUT=<output dir>")
endif()
configure_file(${REF}/lib/NGT/defines.h.in ${OUT}/NGT/defines.h)
