// spf_lds.h -- host interface of spf_lds.hip (the LDS-resident all-sources
// SPF and its one-launch SPF + RouteDb stream form), for route_stream.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "openr_gpu.h"

namespace ogs {

// One unit group of the one-launch form: units sharing a next-hop width W,
// their SPF rows (dist [n * S_n], nh [n * W * S_n]: scratch or the caller's)
// and RouteDb outputs.
struct LdsRouteGroup {
  const ogs_unit* units;
  int n;
  int W;
  uint32_t* dist;
  uint32_t* nh;
  ogs_spf_out out;
};

// Workspace bytes of the LDS forms for nUnits units of width <= W, or 0
// when the batch does not qualify (15-bit node ids, 16-bit chunk ids, image
// + state fit LDS).
size_t lds_scratch_bytes(const ogs_graph& g, int W, int nUnits);
// Prep launch: images, weight partials, counters, route keys (key may be
// nullptr: SPF only; key16: packed u16 keys, route_stream.h).
hipError_t launch_lds_prep(const ogs_graph& g, const ogs_prefix_table* pt, void* key,
                           bool key16, int W, int nUnits, void* scratch, hipStream_t stream);
// whether the one-launch form packs this graph's route keys into 16 bits
bool lds_key16(const ogs_graph& g);
// SPF of every unit into dist / nh (route_stream 4), after the prep.
hipError_t launch_spf_lds(const ogs_graph& g, const ogs_unit* units, int nUnits,
                          uint32_t flags, int W, uint32_t* dist, uint32_t* nh,
                          void* scratch, hipStream_t stream);
// SPF + RouteDb stream of up to 4 groups (widest first) in one persistent
// launch (route_stream 5), after the prep for the widest W and all units.
hipError_t launch_spf_lds_routes(const ogs_graph& g, const ogs_prefix_table& pt,
                                 const void* key, bool key16, const LdsRouteGroup* groups,
                                 int n, uint32_t flags, void* scratch, hipStream_t stream);

}  // namespace ogs
