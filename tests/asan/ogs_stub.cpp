// ogs_stub.cpp — a host-only stand-in for libopenr_gpu.so, for the CPU
// sanitizer build of the drop-in's host code (make asan; tests/asan/
// host_asan.cpp). Device memory is host memory, copies are memcpy, and every
// compute entry point returns OGS_E_NODEVICE: the harness exercises only the
// host paths (ingestion, flattening, prefix tables, materialisation, the
// route-update and thrift conversions), never a route computation. Not a
// CPU fallback: nothing in the product links it.
#include <cstdlib>
#include <cstring>
#include <initializer_list>

#include "openr_gpu.h"

extern "C" {
const char* ogs_last_error(void) { return "host-only stub: no device"; }
int ogs_malloc(void** dptr, size_t bytes) {
  *dptr = std::malloc(bytes ? bytes : 1);
  return *dptr ? OGS_OK : OGS_E_NOMEM;
}
int ogs_free(void* dptr) {
  std::free(dptr);
  return OGS_OK;
}
int ogs_host_alloc(void** hptr, size_t bytes) { return ogs_malloc(hptr, bytes); }
int ogs_host_free(void* hptr) { return ogs_free(hptr); }
int ogs_memcpy_h2d(void* dst, const void* src, size_t bytes, void*) {
  std::memcpy(dst, src, bytes);
  return OGS_OK;
}
int ogs_memcpy_d2h(void* dst, const void* src, size_t bytes, void*) {
  std::memcpy(dst, src, bytes);
  return OGS_OK;
}
int ogs_stream_sync(void*) { return OGS_OK; }
int ogs_nh_words_for_degree(int degree) {
  if (degree < 0) return OGS_E_INVALID;
  const int words = (degree + 31) / 32;
  for (int w : {1, 2, 4, 8, 16}) {
    if (words <= w) return w;
  }
  return words;
}
#define NODEV(name, ...) \
  int name(__VA_ARGS__) { return OGS_E_NODEVICE; }
NODEV(ogs_csr_patch, uint64_t*, const uint32_t*, const uint64_t*, int32_t, void*)
NODEV(ogs_ksp_paths, const ogs_graph*, const ogs_path_unit*, int32_t, const uint32_t*, uint32_t,
      uint32_t, ogs_path_out*, void*)
NODEV(ogs_ksp2_paths, const ogs_graph*, const ogs_unit*, int32_t, const ogs_path_unit*, int32_t,
      uint32_t, ogs_path_out*, ogs_path_out*, void*)
NODEV(ogs_rib_policy_apply, const ogs_prefix_table*, const ogs_rib_policy*, int32_t, int32_t,
      int32_t, const uint32_t*, uint32_t*, uint16_t*, uint16_t*, void*)
NODEV(ogs_route_changes_gather, const uint32_t*, int32_t, int32_t, const ogs_spf_out*, int32_t,
      const ogs_route_changes*, void*)
NODEV(ogs_routes_from_spf, const ogs_graph*, const ogs_prefix_table*, const ogs_unit*, int32_t,
      const void*, const uint32_t*, const uint32_t*, uint32_t, int32_t, ogs_spf_out*, void*)
NODEV(ogs_routes_multiarea, const ogs_graph*, const ogs_prefix_table*, const ogs_area_table*,
      const uint32_t*, int32_t, const uint32_t*, const void*, const uint32_t*, uint32_t, int32_t,
      ogs_spf_out*, void*)
NODEV(ogs_spf_routes, const ogs_graph*, const ogs_prefix_table*, const ogs_unit*, int32_t,
      uint32_t, int32_t, ogs_spf_out*, void*)
NODEV(ogs_spf_routes_groups, const ogs_graph*, const ogs_prefix_table*, const ogs_route_group*,
      int32_t, uint32_t, void*)
NODEV(ogs_spf_routes_variants, const ogs_graph*, const ogs_prefix_table*, const ogs_unit*,
      int32_t, const ogs_unit_mods*, ogs_route_diff*, uint32_t, int32_t, ogs_spf_out*, void*)
}
