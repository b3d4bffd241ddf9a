// route_global.h — one thread per (unit, prefix) RouteDb from SPF state in
// HBM (spf_global.hip, spf_exact.hip): route_one (route_core.h) against the
// unit's dist / next-hop rows, no per-node LDS staging, coalesced record
// stores. u32 or u64 distances.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "route_core.h"
#include "spf_core.h"

namespace ogs {

// Unit state in HBM as the route kernel reads it.
template <typename D, int W>
struct GlobalView {
  const D* d;
  const uint32_t* n;
  size_t Sn;
  const uint32_t* r;  // settled bitset (exact-order state) or nullptr
  __device__ __forceinline__ D dist(uint32_t v) const { return d[v]; }
  __device__ __forceinline__ bool reached(uint32_t v) const {
    return r ? ((r[v >> 5] >> (v & 31u)) & 1u) != 0u : d[v] != DistInf<D>::value;
  }
  __device__ __forceinline__ uint32_t nh(uint32_t v, int w) const {
    return n[size_t(w) * Sn + v];
  }
};

// One thread per (unit, prefix): route_one against the unit's HBM state
// (grid x = unit, y = prefix block of 256).
template <typename D, int W>
__global__ __launch_bounds__(kBlock) void route_global_kernel(
    ogs_graph g, ogs_prefix_table pt, const ogs_unit* __restrict__ units,
    uint32_t flags, const D* __restrict__ sDist, const uint32_t* __restrict__ sNh,
    const uint32_t* __restrict__ sReach, ogs_spf_out out) {
  const uint32_t u = blockIdx.x;
  const uint32_t p = blockIdx.y * kBlock + threadIdx.x;
  const ogs_unit unit = units[u];
  const uint32_t Sp = uint32_t(pt.max_prefixes);
  const uint32_t p0 = pt.pfx_base[unit.topo];
  const uint32_t P = pt.pfx_base[unit.topo + 1] - p0;
  if (p >= Sp) return;
  const size_t Sn = size_t(g.max_nodes);
  const size_t rec = size_t(u) * Sp + p;
  uint32_t meta = 0, selBits = 0, mask[W];
  D metric = DistInf<D>::value;
#pragma unroll
  for (int w = 0; w < W; ++w) mask[w] = 0u;
  if (p < P) {
    const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0, (flags & OGS_F_V4_OVER_V6) != 0,
                       (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
    const GlobalView<D, W> sv{sDist + u * Sn, sNh + size_t(u) * W * Sn, Sn,
                              sReach ? sReach + size_t(u) * ((Sn + 31) / 32) : nullptr};
    route_one<D, W>(pt, p0 + p, unit.src, g.node_flags + g.node_base[unit.topo], sv, cfg,
                    meta, metric, mask, selBits);
  }
  if (out.meta) out.meta[rec] = meta;
  if (out.metric) static_cast<D*>(out.metric)[rec] = metric;
  if (out.sel) out.sel[rec] = selBits;
  if (out.mask) {
#pragma unroll
    for (int w = 0; w < W; ++w) out.mask[(size_t(u) * W + w) * Sp + p] = mask[w];
  }
}

// route_global_kernel for next-hop sets wider than 16 words (sources of more
// than 512 links; runtime W, masks stored word by word).
template <typename D>
__global__ __launch_bounds__(kBlock) void route_global_wide_kernel(
    ogs_graph g, ogs_prefix_table pt, const ogs_unit* __restrict__ units,
    uint32_t flags, int W, const D* __restrict__ sDist, const uint32_t* __restrict__ sNh,
    const uint32_t* __restrict__ sReach, ogs_spf_out out) {
  const uint32_t u = blockIdx.x;
  const uint32_t p = blockIdx.y * kBlock + threadIdx.x;
  const ogs_unit unit = units[u];
  const uint32_t Sp = uint32_t(pt.max_prefixes);
  const uint32_t p0 = pt.pfx_base[unit.topo];
  const uint32_t P = pt.pfx_base[unit.topo + 1] - p0;
  if (p >= Sp) return;
  const size_t Sn = size_t(g.max_nodes);
  const size_t rec = size_t(u) * Sp + p;
  uint32_t meta = 0, selBits = 0;
  D metric = DistInf<D>::value;
  uint32_t* mask = out.mask ? out.mask + size_t(u) * W * Sp + p : nullptr;
  if (p < P) {
    const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0, (flags & OGS_F_V4_OVER_V6) != 0,
                       (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
    const GlobalView<D, 1> sv{sDist + u * Sn, sNh + size_t(u) * W * Sn, Sn,
                              sReach ? sReach + size_t(u) * ((Sn + 31) / 32) : nullptr};
    route_one_wide<D>(pt, p0 + p, unit.src, g.node_flags + g.node_base[unit.topo], sv, cfg, W,
                      meta, metric, mask, Sp, selBits);
  } else if (mask) {
    for (int w = 0; w < W; ++w) mask[size_t(w) * Sp] = 0u;
  }
  if (out.meta) out.meta[rec] = meta;
  if (out.metric) static_cast<D*>(out.metric)[rec] = metric;
  if (out.sel) out.sel[rec] = selBits;
}

template <typename D>
hipError_t launch_route_global_wide(const ogs_graph& g, const ogs_prefix_table& pt,
                                    const ogs_unit* units, int nUnits, uint32_t flags, int W,
                                    const D* dist, const uint32_t* nh, const ogs_spf_out& out,
                                    hipStream_t stream, const uint32_t* reach = nullptr) {
  const unsigned by = unsigned((pt.max_prefixes + kBlock - 1) / kBlock);
  hipLaunchKernelGGL((route_global_wide_kernel<D>), dim3(unsigned(nUnits), by), dim3(kBlock), 0,
                     stream, g, pt, units, flags, W, dist, nh, reach, out);
  return hipGetLastError();
}

template <typename D, int W>
hipError_t launch_route_global(const ogs_graph& g, const ogs_prefix_table& pt,
                               const ogs_unit* units, int nUnits, uint32_t flags,
                               const D* dist, const uint32_t* nh, const ogs_spf_out& out,
                               hipStream_t stream, const uint32_t* reach = nullptr) {
  const unsigned by = unsigned((pt.max_prefixes + kBlock - 1) / kBlock);
  hipLaunchKernelGGL((route_global_kernel<D, W>), dim3(unsigned(nUnits), by), dim3(kBlock), 0,
                     stream, g, pt, units, flags, dist, nh, reach, out);
  return hipGetLastError();
}

}  // namespace ogs
