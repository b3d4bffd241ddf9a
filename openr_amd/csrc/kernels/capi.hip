// capi.hip — extern "C" entry points of libopenr_gpu.so (include/openr_gpu.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "openr_gpu.h"
#include "engine.h"

namespace ogs {
hipError_t launch_spf_routes(const ogs_graph& g, const ogs_prefix_table* pt,
                             const ogs_unit* units, int nUnits, uint32_t flags,
                             int W, const ogs_spf_out& out, hipStream_t stream,
                             int* unsupported);
hipError_t launch_spf_routes_groups(const ogs_graph& g, const ogs_prefix_table* pt,
                                    const ogs_route_group* groups, int n, uint32_t flags,
                                    hipStream_t stream, int* unsupported);
hipError_t launch_routes_multiarea(const ogs_graph& g, const ogs_prefix_table& pt,
                                   const ogs_area_table& at,
                                   const uint32_t* units, int n,
                                   const uint32_t* spfRow, const void* dist,
                                   const uint32_t* nh, uint32_t flags, int W,
                                   const ogs_spf_out& out, hipStream_t stream);
hipError_t launch_variants(const ogs_graph& g, const ogs_prefix_table& pt,
                           const ogs_unit* units, int nUnits,
                           const ogs_unit_mods* mods, ogs_route_diff* diff,
                           uint32_t flags, int W, const ogs_spf_out& out,
                           hipStream_t stream, int* unsupported);
hipError_t launch_rib_policy(const ogs_prefix_table& pt, const ogs_rib_policy& pol,
                             int A, int nUnits, int W, const uint32_t* meta,
                             uint32_t* mask, uint16_t* applied, uint16_t* counter,
                             hipStream_t stream);
hipError_t launch_route_changes(const uint32_t* changed, int nUnits, int Sp, int W,
                                const uint32_t* meta, const uint32_t* metric,
                                const uint32_t* mask, const ogs_route_changes& out,
                                hipStream_t stream);
hipError_t launch_csr_patch(uint64_t* edges, const uint32_t* idx, const uint64_t* val,
                            int n, hipStream_t stream);
hipError_t launch_routes_from_spf(const ogs_graph& g, const ogs_prefix_table& pt,
                                  const ogs_unit* units, int n, const void* dist,
                                  const uint32_t* nh, const uint32_t* reach, uint32_t flags,
                                  int W, const ogs_spf_out& out, hipStream_t stream);
hipError_t launch_ksp(const ogs_graph& g, const ogs_path_unit* units,
                      int nUnits, const uint32_t* masks, uint32_t maskWords,
                      uint32_t flags, const ogs_path_out& out,
                      hipStream_t stream, int* unsupported);
hipError_t launch_ksp2(const ogs_graph& g, const ogs_unit* sources,
                       int nSources, const ogs_path_unit* units, int nUnits,
                       uint32_t flags, const ogs_path_out& o1,
                       const ogs_path_out& o2, hipStream_t stream,
                       int* unsupported);
}

namespace {
thread_local std::string g_lastError;

int fail(int code, const std::string& msg) {
  g_lastError = msg;
  return code;
}

int hipFail(hipError_t e, const char* what) {
  return fail(OGS_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

extern "C" {

const char* ogs_version(void) { return "openr-gpu-spf 0.3 (gfx950)"; }
int ogs_abi_version(void) { return OGS_ABI_VERSION; }

const char* ogs_last_error(void) { return g_lastError.c_str(); }

int ogs_device_count(int* count) {
  if (!count) return fail(OGS_E_INVALID, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return fail(OGS_E_NODEVICE, std::string("hipGetDeviceCount: ") +
                                    hipGetErrorString(e));
  }
  *count = n;
  return n > 0 ? OGS_OK : fail(OGS_E_NODEVICE, "no HIP device visible");
}

int ogs_set_device(int device) {
  hipError_t e = hipSetDevice(device);
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipSetDevice");
}

int ogs_malloc(void** dptr, size_t bytes) {
  if (!dptr) return fail(OGS_E_INVALID, "dptr is NULL");
  *dptr = nullptr;
  if (bytes == 0) return OGS_OK;
  hipError_t e = hipMalloc(dptr, bytes);
  if (e == hipErrorOutOfMemory) return fail(OGS_E_NOMEM, "hipMalloc: out of memory");
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipMalloc");
}

int ogs_free(void* dptr) {
  if (!dptr) return OGS_OK;
  hipError_t e = hipFree(dptr);
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipFree");
}

int ogs_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return OGS_OK;
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice,
                                static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipMemcpyAsync(H2D)");
}

int ogs_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return OGS_OK;
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost,
                                static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipMemcpyAsync(D2H)");
}

int ogs_memset(void* dst, int value, size_t bytes, void* stream) {
  if (bytes == 0) return OGS_OK;
  hipError_t e =
      hipMemsetAsync(dst, value, bytes, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipMemsetAsync");
}

int ogs_host_alloc(void** hptr, size_t bytes) {
  if (!hptr) return fail(OGS_E_INVALID, "hptr is NULL");
  *hptr = nullptr;
  if (bytes == 0) return OGS_OK;
  hipError_t e = hipHostMalloc(hptr, bytes, hipHostMallocDefault);
  if (e == hipErrorOutOfMemory) return fail(OGS_E_NOMEM, "hipHostMalloc: out of memory");
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipHostMalloc");
}

int ogs_host_free(void* hptr) {
  if (!hptr) return OGS_OK;
  hipError_t e = hipHostFree(hptr);
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipHostFree");
}

int ogs_stream_sync(void* stream) {
  hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "hipStreamSynchronize");
}

}  // extern "C"

// one knob of `o` (the default context's, or a context's own)
static int set_option(ogs::EngineOptions& o, const char* name, int64_t value) {
  if (!name) return fail(OGS_E_INVALID, "option name is NULL");
  if (std::strcmp(name, "unit_width") == 0) {
    if (value != -1 && value != 0 && value != 1 && value != 2 && value != 3 &&
        value != 64 && value != 128 && value != 256) {
      return fail(OGS_E_INVALID, "unit_width must be -1, 0, 1, 2, 3, 64, 128 or 256");
    }
    o.unitWidth = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "ms_group") == 0) {
    if (value != 0 && value != 1 && value != 2 && value != 4) {
      return fail(OGS_E_INVALID, "ms_group must be 0, 1, 2 or 4");
    }
    o.msGroup = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "route_stream") == 0) {
    if (value != 1 && value != 2 && value != 4 && value != 5) {
      return fail(OGS_E_INVALID, "route_stream must be 1, 2, 4 or 5");
    }
    o.routeStream = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "lds_parts") == 0) {
    if (value < 0 || value > 64) return fail(OGS_E_INVALID, "lds_parts must be in [0, 64]");
    o.ldsParts = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "lds_tail") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "lds_tail must be 0 or 1");
    o.ldsTail = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "lds_lead") == 0) {
    if (value < -1 || value > 65536) return fail(OGS_E_INVALID, "lds_lead must be in [-1, 65536]");
    o.ldsLead = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "lds_tail_parts") == 0) {
    if (value < 0 || value > 64) return fail(OGS_E_INVALID, "lds_tail_parts must be in [0, 64]");
    o.ldsTailParts = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "lds_pull") == 0) {
    if (value < 0 || value > 15) return fail(OGS_E_INVALID, "lds_pull must be in [0, 15]");
    o.ldsPull = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "lds_bfs_exit") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "lds_bfs_exit must be 0 or 1");
    o.ldsBfsExit = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "lds_key16") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "lds_key16 must be 0 or 1");
    o.ldsKey16 = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "lds_grid") == 0) {
    if (value < 0 || value > 4096) return fail(OGS_E_INVALID, "lds_grid must be in [0, 4096]");
    o.ldsGrid = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_packed_scan") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "spf_packed_scan must be 0 or 1");
    o.spfPackedScan = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "route_store_nt") == 0) {
    if (value < 0 || value > 3) return fail(OGS_E_INVALID, "route_store_nt must be in [0, 3]");
    o.routeStoreNt = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "frontier_block") == 0) {
    if (value != 0 && value != 256 && value != 512 && value != 1024) {
      return fail(OGS_E_INVALID, "frontier_block must be 0, 256, 512 or 1024");
    }
    o.frontierBlock = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "frontier_parts") == 0) {
    if (value < 0 || value > 16) return fail(OGS_E_INVALID, "frontier_parts must be in [0, 16]");
    o.frontierParts = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_lane_walk") == 0) {
    if (value < -1 || value > 1) return fail(OGS_E_INVALID, "spf_lane_walk must be -1, 0 or 1");
    o.spfLaneWalk = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_preload") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "spf_preload must be 0 or 1");
    o.spfPreload = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "frontier_parts_wide") == 0) {
    if (value < 0 || value > 16) {
      return fail(OGS_E_INVALID, "frontier_parts_wide must be in [0, 16]");
    }
    o.frontierPartsWide = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_seed_row") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "spf_seed_row must be 0 or 1");
    o.spfSeedRow = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_frontier") == 0) {
    if (value != 0 && value != 1) {
      return fail(OGS_E_INVALID, "spf_frontier must be 0 or 1");
    }
    o.spfFrontier = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_global") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "spf_global must be 0 or 1");
    o.spfGlobal = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "ksp_queue") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "ksp_queue must be 0 or 1");
    o.kspQueue = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_global_sync") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "spf_global_sync must be 0 or 1");
    o.spfGlobalSync = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_global_lds") == 0) {
    if (value < 0 || value > 3) return fail(OGS_E_INVALID, "spf_global_lds must be 0..3");
    o.spfGlobalLds = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "c4_desc") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "c4_desc must be 0 or 1");
    o.c4Desc = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "ksp_hbm") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "ksp_hbm must be 0 or 1");
    o.kspHbm = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "ksp_stage") == 0) {
    if (value < -1 || value > 2) return fail(OGS_E_INVALID, "ksp_stage must be -1, 0, 1 or 2");
    o.kspStage = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_ninfo") == 0) {
    if (value < -1 || value > 1) return fail(OGS_E_INVALID, "spf_ninfo must be -1, 0 or 1");
    o.spfNinfo = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "spf_queue") == 0) {
    if (value != -1 && value != 0) return fail(OGS_E_INVALID, "spf_queue must be -1 or 0");
    o.spfQueue = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "wave_upb") == 0) {
    if (value != 4 && value != 8 && value != 16) {
      return fail(OGS_E_INVALID, "wave_upb must be 4, 8 or 16");
    }
    o.waveUpb = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "ksp_prune") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "ksp_prune must be 0 or 1");
    o.kspPrune = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "ksp_wave_trace") == 0) {
    if (value != 0 && value != 1) return fail(OGS_E_INVALID, "ksp_wave_trace must be 0 or 1");
    o.kspWaveTrace = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "wave_opt") == 0) {
    if (value < 0 || value > 3) return fail(OGS_E_INVALID, "wave_opt must be in [0, 3]");
    o.waveOpt = int(value);
    return OGS_OK;
  }
  if (std::strcmp(name, "wave_wg_lds") == 0) {
    if (value < 0 || value > 160 * 1024) {
      return fail(OGS_E_INVALID, "wave_wg_lds must be in [0, 163840]");
    }
    o.waveWgLds = int(value);
    return OGS_OK;
  }
  return fail(OGS_E_INVALID, std::string("unknown option ") + name);
}

extern "C" {

int ogs_set_option(const char* name, int64_t value) {
  return set_option(ogs::default_options(), name, value);
}

// ---- contexts (ABI 6) ------------------------------------------------------
struct ogs_ctx {
  ogs::EngineContext e;
};

int ogs_ctx_create(int32_t device, ogs_ctx** out) {
  if (!out) return fail(OGS_E_INVALID, "out is NULL");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return fail(OGS_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return fail(OGS_E_INVALID, "device out of range");
  ogs_ctx* c = new (std::nothrow) ogs_ctx;
  if (!c) return fail(OGS_E_NOMEM, "context allocation");
  c->e.device = device;
  c->e.opts = ogs::default_options();  // starts from the process defaults
  *out = c;
  return OGS_OK;
}

int ogs_ctx_destroy(ogs_ctx* ctx) {
  if (!ctx) return OGS_OK;
  ogs::DeviceGuard dev(ctx->e.device);  // the caller's device comes back
  delete ctx;  // frees its scratch (hipFree waits for the device)
  return OGS_OK;
}

int ogs_ctx_set_option(ogs_ctx* ctx, const char* name, int64_t value) {
  if (!ctx) return fail(OGS_E_INVALID, "ctx is NULL");
  return set_option(ctx->e.opts, name, value);
}

// any width from ceil(degree/32) up is valid for a call; this is the
// smallest power-of-two width (the templated kernels) up to 16 words
int ogs_nh_words_for_degree(int degree) {
  if (degree < 0) return OGS_E_INVALID;
  const int words = (degree + 31) / 32;
  for (int w : {1, 2, 4, 8, 16}) {
    if (words <= w) return w;
  }
  return words;  // sources of more than 512 links: exact width
}

// Shape checks shared by ogs_spf_routes and ogs_spf_routes_groups.
static int check_routes_args(const ogs_graph* graph, const ogs_prefix_table* prefixes,
                             uint32_t flags) {
  if (!graph->node_base || !graph->row_ptr || !graph->node_flags) {
    return fail(OGS_E_INVALID, "graph arrays are NULL");
  }
  if (graph->max_nodes <= 0 ||
      uint32_t(graph->max_nodes) > OGS_MAX_NODES_PER_TOPO) {
    return fail(OGS_E_UNSUPPORTED, "max_nodes outside (0, 2^21]");
  }
  if (graph->slot_node && graph->slot_stride != 64 &&
      graph->slot_stride != 128 && graph->slot_stride != 256) {
    return fail(OGS_E_INVALID, "slot_stride must be 64, 128 or 256");
  }
  if (graph->slot_node && graph->slot_stride < graph->max_nodes) {
    return fail(OGS_E_INVALID, "slot_stride < max_nodes");
  }
  if (graph->slot_edges &&
      (!graph->slot_node || (graph->slot_degree != 4 && graph->slot_degree != 8))) {
    return fail(OGS_E_INVALID, "slot_edges needs slot_node and slot_degree 4 or 8");
  }
  if (prefixes && (!prefixes->pfx_base || !prefixes->adv_off ||
                   !prefixes->adv_node || !prefixes->adv_metrics ||
                   !prefixes->adv_min_nh || !prefixes->pfx_flags)) {
    return fail(OGS_E_INVALID, "prefix table arrays are NULL");
  }
  if ((flags & OGS_F_EXACT_ORDER) && !(flags & OGS_F_WIDE_METRIC)) {
    return fail(OGS_E_INVALID, "OGS_F_EXACT_ORDER needs OGS_F_WIDE_METRIC");
  }
  return OGS_OK;
}

int ogs_spf_routes_groups(const ogs_graph* graph, const ogs_prefix_table* prefixes,
                          const ogs_route_group* groups, int32_t n_groups, uint32_t flags,
                          void* stream) {
  if (!graph || (!groups && n_groups > 0)) return fail(OGS_E_INVALID, "graph/groups is NULL");
  if (n_groups < 0) return fail(OGS_E_INVALID, "n_groups < 0");
  int live = 0;
  for (int32_t i = 0; i < n_groups; ++i) {
    if (groups[i].n_units < 0) return fail(OGS_E_INVALID, "n_units < 0");
    if (groups[i].n_units == 0) continue;
    if (!groups[i].units) return fail(OGS_E_INVALID, "group units are NULL");
    if (groups[i].nh_words < 1) return fail(OGS_E_INVALID, "nh_words < 1");
    ++live;
  }
  if (live == 0) return OGS_OK;
  const int rc = check_routes_args(graph, prefixes, flags);
  if (rc != OGS_OK) return rc;
  int unsupported = 0;
  hipError_t e = ogs::launch_spf_routes_groups(*graph, prefixes, groups, n_groups, flags,
                                               static_cast<hipStream_t>(stream), &unsupported);
  if (unsupported) {
    return fail(OGS_E_UNSUPPORTED, "no SPF path for these shapes");
  }
  return e == hipSuccess ? OGS_OK : hipFail(e, "spf_route launch");
}

int ogs_spf_routes(const ogs_graph* graph, const ogs_prefix_table* prefixes,
                   const ogs_unit* units, int32_t n_units, uint32_t flags,
                   int32_t nh_words, ogs_spf_out* out, void* stream) {
  if (!graph || !out) return fail(OGS_E_INVALID, "graph/out is NULL");
  if (n_units < 0) return fail(OGS_E_INVALID, "n_units < 0");
  if (n_units == 0) return OGS_OK;
  if (!units || !graph->node_base || !graph->row_ptr || !graph->node_flags) {
    return fail(OGS_E_INVALID, "graph arrays are NULL");
  }
  if (graph->max_nodes <= 0 ||
      uint32_t(graph->max_nodes) > OGS_MAX_NODES_PER_TOPO) {
    return fail(OGS_E_UNSUPPORTED, "max_nodes outside (0, 2^21]");
  }
  if (graph->slot_node && graph->slot_stride != 64 &&
      graph->slot_stride != 128 && graph->slot_stride != 256) {
    return fail(OGS_E_INVALID, "slot_stride must be 64, 128 or 256");
  }
  if (graph->slot_node && graph->slot_stride < graph->max_nodes) {
    return fail(OGS_E_INVALID, "slot_stride < max_nodes");
  }
  if (graph->slot_edges &&
      (!graph->slot_node || (graph->slot_degree != 4 && graph->slot_degree != 8))) {
    return fail(OGS_E_INVALID, "slot_edges needs slot_node and slot_degree 4 or 8");
  }
  if (prefixes && (!prefixes->pfx_base || !prefixes->adv_off ||
                   !prefixes->adv_node || !prefixes->adv_metrics ||
                   !prefixes->adv_min_nh || !prefixes->pfx_flags)) {
    return fail(OGS_E_INVALID, "prefix table arrays are NULL");
  }
  if (nh_words < 1) {
    return fail(OGS_E_INVALID, "nh_words < 1");
  }
  if ((flags & OGS_F_EXACT_ORDER) && !(flags & OGS_F_WIDE_METRIC)) {
    return fail(OGS_E_INVALID, "OGS_F_EXACT_ORDER needs OGS_F_WIDE_METRIC");
  }
  int unsupported = 0;
  hipError_t e = ogs::launch_spf_routes(
      *graph, prefixes, units, n_units, flags, nh_words, *out,
      static_cast<hipStream_t>(stream), &unsupported);
  if (unsupported) {
    return fail(OGS_E_UNSUPPORTED, "no SPF path for these shapes");
  }
  return e == hipSuccess ? OGS_OK : hipFail(e, "spf_route launch");
}

int ogs_routes_from_spf(const ogs_graph* graph, const ogs_prefix_table* prefixes,
                        const ogs_unit* units, int32_t n_units, const void* spf_dist,
                        const uint32_t* spf_nh, const uint32_t* spf_reached, uint32_t flags,
                        int32_t nh_words, ogs_spf_out* out, void* stream) {
  if (!graph || !prefixes || !out) return fail(OGS_E_INVALID, "graph/prefixes/out is NULL");
  if (n_units < 0) return fail(OGS_E_INVALID, "n_units < 0");
  if (n_units == 0 || prefixes->max_prefixes <= 0) return OGS_OK;
  if (!units || !spf_dist || !spf_nh || !graph->node_base || !graph->node_flags ||
      !prefixes->pfx_base || !prefixes->adv_off || !prefixes->adv_node ||
      !prefixes->adv_metrics || !prefixes->adv_min_nh || !prefixes->pfx_flags) {
    return fail(OGS_E_INVALID, "input arrays are NULL");
  }
  if (nh_words < 1) {
    return fail(OGS_E_INVALID, "nh_words < 1");
  }
  hipError_t e = ogs::launch_routes_from_spf(*graph, *prefixes, units, n_units, spf_dist,
                                            spf_nh, spf_reached, flags, nh_words, *out,
                                            static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "routes-from-spf launch");
}

int ogs_ksp_paths(const ogs_graph* graph, const ogs_path_unit* units,
                  int32_t n_units, const uint32_t* masks, uint32_t mask_words,
                  uint32_t flags, ogs_path_out* out, void* stream) {
  if (!graph || !out) return fail(OGS_E_INVALID, "graph/out is NULL");
  if (n_units < 0) return fail(OGS_E_INVALID, "n_units < 0");
  if (n_units == 0) return OGS_OK;
  if (!units || !graph->node_base || !graph->row_ptr || !out->path_count ||
      !out->path_len || !out->path_edges) {
    return fail(OGS_E_INVALID, "graph/unit/output arrays are NULL");
  }
  if (graph->max_nodes <= 0 ||
      uint32_t(graph->max_nodes) > OGS_MAX_NODES_PER_TOPO) {
    return fail(OGS_E_UNSUPPORTED, "max_nodes outside (0, 2^21]");
  }
  if (masks && mask_words < uint32_t((graph->max_edges + 31) / 32)) {
    return fail(OGS_E_INVALID, "mask_words too small for max_edges");
  }
  if (graph->max_degree >= OGS_MAX_DEGREE && !graph->rslot_ext) {
    return fail(OGS_E_INVALID, "rows of 512+ edges need graph->rslot_ext");
  }
  int unsupported = 0;
  hipError_t e = ogs::launch_ksp(*graph, units, n_units, masks, mask_words,
                                 flags, *out, static_cast<hipStream_t>(stream),
                                 &unsupported);
  if (unsupported) {
    return fail(OGS_E_INVALID, "OGS_F_EXACT_ORDER needs OGS_F_WIDE_METRIC");
  }
  return e == hipSuccess ? OGS_OK : hipFail(e, "ksp launch");
}

int ogs_ksp2_paths(const ogs_graph* graph, const ogs_unit* sources,
                   int32_t n_sources, const ogs_path_unit* units,
                   int32_t n_units, uint32_t flags, ogs_path_out* k1,
                   ogs_path_out* k2, void* stream) {
  if (!graph || !k1 || !k2) return fail(OGS_E_INVALID, "graph/outputs are NULL");
  if (n_units < 0 || n_sources < 0) return fail(OGS_E_INVALID, "negative count");
  if (n_units == 0) return OGS_OK;
  if (n_sources == 0 || !sources || !units || !graph->node_base ||
      !graph->row_ptr || !graph->edges) {
    return fail(OGS_E_INVALID, "graph/source/unit arrays are NULL");
  }
  for (const ogs_path_out* o : {k1, k2}) {
    if (!o->path_count || !o->path_len || !o->path_edges) {
      return fail(OGS_E_INVALID, "path output arrays are NULL");
    }
  }
  if (graph->max_nodes <= 0 ||
      uint32_t(graph->max_nodes) > OGS_MAX_NODES_PER_TOPO) {
    return fail(OGS_E_UNSUPPORTED, "max_nodes outside (0, 2^21]");
  }
  if (graph->max_degree >= OGS_MAX_DEGREE && !graph->rslot_ext) {
    return fail(OGS_E_INVALID, "rows of 512+ edges need graph->rslot_ext");
  }
  int unsupported = 0;
  hipError_t e = ogs::launch_ksp2(*graph, sources, n_sources, units, n_units,
                                  flags, *k1, *k2,
                                  static_cast<hipStream_t>(stream), &unsupported);
  if (unsupported) {
    return fail(OGS_E_INVALID, "OGS_F_EXACT_ORDER needs OGS_F_WIDE_METRIC");
  }
  return e == hipSuccess ? OGS_OK : hipFail(e, "ksp2 launch");
}

int ogs_spf_routes_variants(const ogs_graph* graph,
                            const ogs_prefix_table* prefixes,
                            const ogs_unit* units, int32_t n_units,
                            const ogs_unit_mods* mods,
                            ogs_route_diff* diff, uint32_t flags,
                            int32_t nh_words, ogs_spf_out* out, void* stream) {
  if (!graph || !prefixes || !out) return fail(OGS_E_INVALID, "graph/prefixes/out is NULL");
  if (n_units < 0) return fail(OGS_E_INVALID, "n_units < 0");
  if (n_units == 0) return OGS_OK;
  if (!units || !graph->node_base || !graph->row_ptr || !graph->edges ||
      !graph->node_flags || !prefixes->pfx_base || !prefixes->adv_off ||
      !prefixes->adv_node || !prefixes->adv_metrics || !prefixes->adv_min_nh ||
      !prefixes->pfx_flags) {
    return fail(OGS_E_INVALID, "graph / prefix table arrays are NULL");
  }
  if (mods && (!mods->dead_edges || mods->dead_per_unit < 1 || mods->dead_per_unit > 8)) {
    return fail(OGS_E_INVALID, "mods: dead_edges NULL or dead_per_unit outside [1, 8]");
  }
  if (diff && (!diff->base_meta || !diff->base_metric || !diff->base_mask ||
               !diff->changed || !diff->counts)) {
    return fail(OGS_E_INVALID, "diff arrays are NULL");
  }
  if ((flags & OGS_F_INCREMENTAL) && (!mods || !diff || !diff->base_dist || !diff->base_nh)) {
    return fail(OGS_E_INVALID, "OGS_F_INCREMENTAL needs mods and diff with base_dist / base_nh");
  }
  if ((flags & OGS_F_CHANGED_ONLY) && (!(flags & OGS_F_INCREMENTAL) || nh_words != 1)) {
    return fail(OGS_E_INVALID, "OGS_F_CHANGED_ONLY needs OGS_F_INCREMENTAL and nh_words 1");
  }
  if (graph->max_nodes <= 0 || uint32_t(graph->max_nodes) > OGS_MAX_NODES_PER_TOPO) {
    return fail(OGS_E_UNSUPPORTED, "max_nodes outside (0, 2^21]");
  }
  if (nh_words < 1) {
    return fail(OGS_E_INVALID, "nh_words < 1");
  }
  int unsupported = 0;
  hipError_t e = ogs::launch_variants(*graph, *prefixes, units, n_units, mods, diff,
                                      flags, nh_words, *out,
                                      static_cast<hipStream_t>(stream), &unsupported);
  if (unsupported) {
    return fail(OGS_E_UNSUPPORTED,
                "variants need the large-topology path (edge_src, nh_words <= 4, "
                "32-bit distances)");
  }
  return e == hipSuccess ? OGS_OK : hipFail(e, "variant launch");
}

int ogs_route_changes_gather(const uint32_t* changed, int32_t n_units,
                             int32_t max_prefixes, const ogs_spf_out* records,
                             int32_t nh_words, const ogs_route_changes* changes,
                             void* stream) {
  if (n_units < 0 || max_prefixes < 0) {
    return fail(OGS_E_INVALID, "n_units or max_prefixes < 0");
  }
  if (n_units == 0 || max_prefixes == 0) return OGS_OK;
  if (!changed || !records || !changes || !changes->offsets) {
    return fail(OGS_E_INVALID, "changed/records/changes/offsets is NULL");
  }
  if (!records->meta || !records->metric || !records->mask) {
    return fail(OGS_E_INVALID, "records need meta, metric and mask");
  }
  if (nh_words != 1 && nh_words != 2 && nh_words != 4) {
    return fail(OGS_E_UNSUPPORTED, "nh_words must be 1, 2 or 4");
  }
  if (changes->total == 0) return OGS_OK;
  if (!changes->prefix || !changes->meta || !changes->metric || !changes->mask) {
    return fail(OGS_E_INVALID, "change record arrays are NULL");
  }
  hipError_t e = ogs::launch_route_changes(
      changed, n_units, max_prefixes, nh_words, records->meta,
      reinterpret_cast<const uint32_t*>(records->metric), records->mask, *changes,
      static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "route changes gather");
}

int ogs_csr_patch(uint64_t* edges, const uint32_t* idx, const uint64_t* val,
                  int32_t n, void* stream) {
  if (n < 0) return fail(OGS_E_INVALID, "n < 0");
  if (n == 0) return OGS_OK;
  if (!edges || !idx || !val) return fail(OGS_E_INVALID, "edges/idx/val is NULL");
  hipError_t e = ogs::launch_csr_patch(edges, idx, val, n, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "csr patch");
}

int ogs_rib_policy_apply(const ogs_prefix_table* prefixes,
                         const ogs_rib_policy* policy, int32_t num_areas,
                         int32_t n_units, int32_t nh_words,
                         const uint32_t* meta, uint32_t* mask,
                         uint16_t* applied, uint16_t* counter, void* stream) {
  if (!prefixes || !policy || !meta || !mask) {
    return fail(OGS_E_INVALID, "prefixes/policy/meta/mask is NULL");
  }
  if (n_units < 0 || num_areas < 1) {
    return fail(OGS_E_INVALID, "n_units < 0 or num_areas < 1");
  }
  if (n_units == 0 || policy->num_statements == 0) return OGS_OK;
  if (policy->num_statements < 0 || policy->num_statements > 32 ||
      !policy->pfx_match || !policy->adv_tag_match || !policy->slot_nonzero ||
      !prefixes->pfx_base || !prefixes->adv_off) {
    return fail(OGS_E_INVALID, "policy tables NULL or more than 32 statements per chunk");
  }
  if (policy->statement_base < 0 ||
      policy->statement_base + policy->num_statements > int32_t(OGS_POLICY_NONE)) {
    return fail(OGS_E_INVALID, "statement_base + num_statements outside [0, 65535]");
  }
  if (policy->statement_base > 0 && (!applied || !counter)) {
    return fail(OGS_E_INVALID, "a continuation chunk needs applied / counter");
  }
  if (nh_words < 1) {
    return fail(OGS_E_INVALID, "nh_words < 1");
  }
  hipError_t e = ogs::launch_rib_policy(*prefixes, *policy, num_areas, n_units, nh_words,
                                        meta, mask, applied, counter,
                                        static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "rib policy launch");
}

int ogs_routes_multiarea(const ogs_graph* graph,
                         const ogs_prefix_table* prefixes,
                         const ogs_area_table* areas, const uint32_t* units,
                         int32_t n_units, const uint32_t* spf_row,
                         const void* spf_dist, const uint32_t* spf_nh,
                         uint32_t flags, int32_t nh_words, ogs_spf_out* out,
                         void* stream) {
  if (!graph || !prefixes || !areas || !out) {
    return fail(OGS_E_INVALID, "graph/prefixes/areas/out is NULL");
  }
  if (n_units < 0) return fail(OGS_E_INVALID, "n_units < 0");
  if (n_units == 0) return OGS_OK;
  if (!units || !spf_row || !spf_dist || !spf_nh || !graph->node_base ||
      !graph->node_flags || !areas->name_local || !areas->adv_area ||
      !areas->adv_name || !prefixes->pfx_base || !prefixes->adv_off ||
      !prefixes->adv_node || !prefixes->adv_metrics || !prefixes->adv_min_nh ||
      !prefixes->pfx_flags) {
    return fail(OGS_E_INVALID, "multi-area input arrays are NULL");
  }
  if (areas->num_areas <= 0 || areas->num_areas > graph->num_topos) {
    return fail(OGS_E_INVALID, "num_areas outside [1, num_topos]");
  }
  if (nh_words < 1) {
    return fail(OGS_E_INVALID, "nh_words < 1");
  }
  hipError_t e = ogs::launch_routes_multiarea(
      *graph, *prefixes, *areas, units, n_units, spf_row, spf_dist, spf_nh,
      flags, nh_words, *out, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? OGS_OK : hipFail(e, "multi-area route launch");
}


// Context forms of the compute entry points: the call runs with the
// context's device, options and scratch (engine.h), then the thread's
// previous context binding and its previous HIP device are restored
// (BoundContext). Same arguments and status as the plain entry point.
#define OGS_CTX_CALL(ctx, call)                                  \
  do {                                                           \
    if (!(ctx)) return fail(OGS_E_INVALID, "ctx is NULL");       \
    ogs::BoundContext bound_(&(ctx)->e);                         \
    if (!bound_.ok()) {                                          \
      return fail(OGS_E_HIP, "cannot switch to the ctx's device"); \
    }                                                            \
    return (call);                                               \
  } while (0)

int ogs_ctx_spf_routes(ogs_ctx* ctx, const ogs_graph* graph, const ogs_prefix_table* prefixes,
                       const ogs_unit* units, int32_t n_units, uint32_t flags,
                       int32_t nh_words, ogs_spf_out* out, void* stream) {
  OGS_CTX_CALL(ctx, ogs_spf_routes(graph, prefixes, units, n_units, flags, nh_words, out,
                                   stream));
}

int ogs_ctx_spf_routes_groups(ogs_ctx* ctx, const ogs_graph* graph,
                              const ogs_prefix_table* prefixes, const ogs_route_group* groups,
                              int32_t n_groups, uint32_t flags, void* stream) {
  OGS_CTX_CALL(ctx, ogs_spf_routes_groups(graph, prefixes, groups, n_groups, flags, stream));
}

int ogs_ctx_routes_from_spf(ogs_ctx* ctx, const ogs_graph* graph,
                            const ogs_prefix_table* prefixes, const ogs_unit* units,
                            int32_t n_units, const void* spf_dist, const uint32_t* spf_nh,
                            const uint32_t* spf_reached, uint32_t flags, int32_t nh_words,
                            ogs_spf_out* out, void* stream) {
  OGS_CTX_CALL(ctx, ogs_routes_from_spf(graph, prefixes, units, n_units, spf_dist, spf_nh,
                                        spf_reached, flags, nh_words, out, stream));
}

int ogs_ctx_spf_routes_variants(ogs_ctx* ctx, const ogs_graph* graph,
                                const ogs_prefix_table* prefixes, const ogs_unit* units,
                                int32_t n_units, const ogs_unit_mods* mods,
                                ogs_route_diff* diff, uint32_t flags, int32_t nh_words,
                                ogs_spf_out* out, void* stream) {
  OGS_CTX_CALL(ctx, ogs_spf_routes_variants(graph, prefixes, units, n_units, mods, diff, flags,
                                            nh_words, out, stream));
}

int ogs_ctx_ksp_paths(ogs_ctx* ctx, const ogs_graph* graph, const ogs_path_unit* units,
                      int32_t n_units, const uint32_t* masks, uint32_t mask_words,
                      uint32_t flags, ogs_path_out* out, void* stream) {
  OGS_CTX_CALL(ctx, ogs_ksp_paths(graph, units, n_units, masks, mask_words, flags, out, stream));
}

int ogs_ctx_ksp2_paths(ogs_ctx* ctx, const ogs_graph* graph, const ogs_unit* sources,
                       int32_t n_sources, const ogs_path_unit* units, int32_t n_units,
                       uint32_t flags, ogs_path_out* k1, ogs_path_out* k2, void* stream) {
  OGS_CTX_CALL(ctx, ogs_ksp2_paths(graph, sources, n_sources, units, n_units, flags, k1, k2,
                                   stream));
}

int ogs_ctx_routes_multiarea(ogs_ctx* ctx, const ogs_graph* graph,
                             const ogs_prefix_table* prefixes, const ogs_area_table* areas,
                             const uint32_t* units, int32_t n_units, const uint32_t* spf_row,
                             const void* spf_dist, const uint32_t* spf_nh, uint32_t flags,
                             int32_t nh_words, ogs_spf_out* out, void* stream) {
  OGS_CTX_CALL(ctx, ogs_routes_multiarea(graph, prefixes, areas, units, n_units, spf_row,
                                         spf_dist, spf_nh, flags, nh_words, out, stream));
}

int ogs_ctx_rib_policy_apply(ogs_ctx* ctx, const ogs_prefix_table* prefixes,
                             const ogs_rib_policy* policy, int32_t num_areas, int32_t n_units,
                             int32_t nh_words, const uint32_t* meta, uint32_t* mask,
                             uint16_t* applied, uint16_t* counter, void* stream) {
  OGS_CTX_CALL(ctx, ogs_rib_policy_apply(prefixes, policy, num_areas, n_units, nh_words, meta,
                                         mask, applied, counter, stream));
}

}  // extern "C"
