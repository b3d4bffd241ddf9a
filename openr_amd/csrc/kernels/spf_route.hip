// spf_route.hip — batched ECMP SPF + fused per-prefix RouteDb for gfx950.
//
// One work unit = (topology, source). Small topologies (<= 256 nodes) run
// one WAVEFRONT per unit (4 independent units per 256-thread workgroup, no
// workgroup barriers); larger ones run one WORKGROUP per unit. The whole
// per-unit working set (distances, next-hop link-slot bitsets and, when it
// fits, the topology's CSR) lives in LDS.
//
// SPF (replaces LinkState::runSpf, LinkState.cpp:720-820). For metrics >= 1
// the reference's Dijkstra result equals the unique fixpoint of
//   dist(v) = min_{u in P(v)} dist(u) + w(u,v)
//   NH(v)   = U_{u tight pred of v} ( u == src ? {links src->v with
//             w == dist(v)} : NH(u) )
// where P(v) are neighbours over up links that relax (u == src or u not
// hard-drained, LinkState.cpp:741-752). Because only the source has an empty
// next-hop set, the reference's "if empty add otherNode" (808-811) is exactly
// "the predecessor is the source". Next-hop sets are kept over the SOURCE's
// link slots, so they already include the link filter of getNextHopsThrift
// (SpfSolver.cpp:705-743: up && maxMetric + (shortest - dist(nbr)) ==
// shortest <=> maxMetric == dist(nbr)). The fixpoint is reached by
// pull-style Bellman-Ford rounds over LDS with in-place (chaotic) updates;
// distances only decrease, so the loop stops at the first round in which no
// node of the unit changes (wave ballot / workgroup barrier-OR).
//
// RouteDb (replaces SpfSolver::createRouteForPrefix, SpfSolver.cpp:160-311,
// 455-639, and LsdbUtil selectRoutes/selectBestNodeArea, LsdbUtil.cpp:
// 700-823), single area: one lane per prefix walks the prefix's advertiser
// segment a few times (reachability + hard-drain filter, best-route
// selection, shortest distance, next-hop union, min-nexthop) and writes one
// compact route record (flags|best, metric, link-slot mask).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "openr_gpu.h"
#include "route_core.h"
#include "spf_core.h"
#include "engine.h"

namespace ogs {

template <typename D, int W, int UT, bool STAGE>
__global__ __launch_bounds__(kBlock) void spf_route_kernel(
    ogs_graph g, ogs_prefix_table pt, int hasPrefixes,
    const ogs_unit* __restrict__ units, int nUnits, uint32_t flags,
    ogs_spf_out out, uint32_t ldsPerUnit) {
  constexpr int kUnitsPerBlock = kBlock / UT;
  const int uib = threadIdx.x / UT;
  const int lane = threadIdx.x % UT;
  const int uidx = blockIdx.x * kUnitsPerBlock + uib;
  if (uidx >= nUnits) return;  // whole unit exits together

  const ogs_unit unit = units[uidx];
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const uint32_t s = unit.src;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* base = smem + uib * ldsPerUnit;
  D* dist = reinterpret_cast<D*>(base);
  const uint32_t distBytes = (N * sizeof(D) + 15u) & ~15u;
  uint32_t* nh = reinterpret_cast<uint32_t*>(base + distBytes);
  const uint32_t nhBytes = (N * W * 4u + 15u) & ~15u;

  UnitCsr csr;
  if constexpr (STAGE) {
    uint32_t* lrow = reinterpret_cast<uint32_t*>(base + distBytes + nhBytes);
    const uint32_t rowBytes = ((N + 1) * 4u + 15u) & ~15u;
    uint64_t* ledg =
        reinterpret_cast<uint64_t*>(base + distBytes + nhBytes + rowBytes);
    const uint32_t e0 = gRow[0];
    const uint32_t E = gRow[N] - e0;
    for (uint32_t i = lane; i <= N; i += UT) lrow[i] = gRow[i] - e0;
    for (uint32_t i = lane; i < E; i += UT) ledg[i] = g.edges[e0 + i];
    csr = UnitCsr{lrow, ledg, 0u, nullptr};
  } else {
    csr = UnitCsr{gRow, g.edges, gRow[0], nullptr};
  }
  // staging writes are ordered before the first reads by the init sync
  spf_fixpoint<D, W, UT, true, false>(N, s, lane, csr,
                                      (flags & OGS_F_HOP_METRIC) != 0, dist,
                                      nh, nullptr);

  // ---- SPF outputs (coalesced) -------------------------------------------
  const uint32_t Sn = g.max_nodes;
  if (out.dist) {
    D* od = reinterpret_cast<D*>(out.dist) + size_t(uidx) * Sn;
    for (uint32_t v = lane; v < N; v += UT) od[v] = dist[v];
  }
  if (out.nh) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint32_t* on = out.nh + (size_t(uidx) * W + w) * Sn;
      for (uint32_t v = lane; v < N; v += UT) on[v] = nh[v * W + w];
    }
  }
  if (!hasPrefixes) return;

  // ---- fused RouteDb ------------------------------------------------------
  const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0,
                     (flags & OGS_F_V4_OVER_V6) != 0,
                     (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
  const uint32_t p0 = pt.pfx_base[unit.topo];
  const uint32_t P = pt.pfx_base[unit.topo + 1] - p0;
  const uint32_t Sp = pt.max_prefixes;
  for (uint32_t p = lane; p < P; p += UT) {
    uint32_t meta, selBits;
    D metric;
    uint32_t mask[W];
    route_one<D, W>(pt, p0 + p, s, nflags, SplitView<D, W>{dist, nh}, cfg,
                    meta, metric, mask, selBits);
    const size_t o = size_t(uidx) * Sp + p;
    if (out.meta) out.meta[o] = meta;
    if (out.metric) reinterpret_cast<D*>(out.metric)[o] = metric;
    if (out.sel) out.sel[o] = selBits;
    if (out.mask) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        out.mask[(size_t(uidx) * W + w) * Sp + p] = mask[w];
      }
    }
  }
}

// ---- host-side launch selection -------------------------------------------
template <typename D, int W, int UT, bool STAGE>
hipError_t launch_one(const ogs_graph& g, const ogs_prefix_table& pt,
                      int hasPrefixes, const ogs_unit* units, int nUnits,
                      uint32_t flags, const ogs_spf_out& out,
                      uint32_t ldsPerUnit, hipStream_t stream) {
  constexpr int upb = kBlock / UT;
  const int grid = (nUnits + upb - 1) / upb;
  const size_t lds = size_t(ldsPerUnit) * upb;
  auto k = spf_route_kernel<D, W, UT, STAGE>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(k),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), lds, stream, g, pt,
                     hasPrefixes, units, nUnits, flags, out, ldsPerUnit);
  return hipGetLastError();
}

uint32_t lds_per_unit(int maxNodes, int maxEdges, int W, int distBytes,
                      bool stage) {
  uint64_t b = align16(uint64_t(maxNodes) * distBytes) +
      align16(uint64_t(maxNodes) * W * 4);
  if (stage) b += align16(uint64_t(maxNodes + 1) * 4) + align16(uint64_t(maxEdges) * 8);
  return static_cast<uint32_t>(b);
}

template <typename D, int W>
hipError_t dispatch_w(const ogs_graph& g, const ogs_prefix_table& pt,
                      int hasPrefixes, const ogs_unit* units, int nUnits,
                      uint32_t flags, const ogs_spf_out& out,
                      hipStream_t stream, int* unsupported) {
  const int wave = g.max_nodes <= 256;
  const uint32_t staged = lds_per_unit(g.max_nodes, g.max_edges, W, sizeof(D), true);
  const uint32_t bare = lds_per_unit(g.max_nodes, g.max_edges, W, sizeof(D), false);
  constexpr uint32_t kBudget = 160 * 1024;
  if (wave && staged * 4 <= kBudget / 2) {
    return launch_one<D, W, 64, true>(g, pt, hasPrefixes, units, nUnits, flags,
                                      out, staged, stream);
  }
  if (staged <= kBudget / 2) {
    return launch_one<D, W, kBlock, true>(g, pt, hasPrefixes, units, nUnits,
                                          flags, out, staged, stream);
  }
  if (bare <= kBudget) {
    return launch_one<D, W, kBlock, false>(g, pt, hasPrefixes, units, nUnits,
                                           flags, out, bare, stream);
  }
  *unsupported = 1;  // > ~10k nodes per topology: needs the global path
  return hipSuccess;
}

template <typename D>
hipError_t dispatch_d(int W, const ogs_graph& g, const ogs_prefix_table& pt,
                      int hasPrefixes, const ogs_unit* units, int nUnits,
                      uint32_t flags, const ogs_spf_out& out,
                      hipStream_t stream, int* unsupported) {
  switch (W) {
    case 1: return dispatch_w<D, 1>(g, pt, hasPrefixes, units, nUnits, flags, out, stream, unsupported);
    case 2: return dispatch_w<D, 2>(g, pt, hasPrefixes, units, nUnits, flags, out, stream, unsupported);
    case 4: return dispatch_w<D, 4>(g, pt, hasPrefixes, units, nUnits, flags, out, stream, unsupported);
    case 8: return dispatch_w<D, 8>(g, pt, hasPrefixes, units, nUnits, flags, out, stream, unsupported);
    case 16: return dispatch_w<D, 16>(g, pt, hasPrefixes, units, nUnits, flags, out, stream, unsupported);
    default: *unsupported = 1; return hipSuccess;
  }
}

template <typename D, int W>
bool try_small(const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes,
               const ogs_unit* units, int nUnits, uint32_t flags,
               const ogs_spf_out& out, int maxDegree, uint32_t maxA,
               int unitWidth, hipStream_t stream, hipError_t* err);

bool try_wave(const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes,
              const ogs_unit* units, int nUnits, uint32_t flags,
              const ogs_spf_out& out, uint32_t maxA, hipStream_t stream,
              hipError_t* err);

bool try_frontier(const ogs_graph& g, const ogs_unit* units, int nUnits,
                  uint32_t flags, int W, uint32_t* dist, uint32_t* nh,
                  hipStream_t stream, hipError_t* err);
bool try_ms_stream(const ogs_graph& g, const ogs_prefix_table& pt,
                   const ogs_unit* units, int nUnits, uint32_t flags, int W,
                   const ogs_spf_out& out, hipStream_t stream, hipError_t* err);
bool try_ms(const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes,
            const ogs_unit* units, int nUnits, uint32_t flags, int W,
            const ogs_spf_out& out, hipStream_t stream, hipError_t* err);

// unit_width option / OGS_UNIT_WIDTH env: -1 automatic, 0 generic kernel
// only, 1 wave kernel, 2 small kernel (automatic width), 3 multi-source
// edge-parallel kernel, 64/128/256 small kernel at that unit width.
// EngineOptions::unitWidth (engine.h), default $OGS_UNIT_WIDTH or -1
int small_unit_width() { return opts().unitWidth; }

bool use_global(const ogs_graph& g, int W, uint32_t flags);
hipError_t launch_spf_routes_exact(const ogs_graph& g, const ogs_prefix_table* pt,
                                   const ogs_unit* units, int nUnits, uint32_t flags,
                                   int W, const ogs_spf_out& out, hipStream_t stream);
hipError_t launch_spf_routes_global(const ogs_graph& g, const ogs_prefix_table* pt,
                                    const ogs_unit* units, int nUnits, uint32_t flags,
                                    int W, const ogs_spf_out& out, hipStream_t stream);
hipError_t launch_spf_routes_global_wide(const ogs_graph& g, const ogs_prefix_table* pt,
                                         const ogs_unit* units, int nUnits, uint32_t flags,
                                         int W, const ogs_spf_out& out, hipStream_t stream);

hipError_t launch_spf_routes(const ogs_graph& g, const ogs_prefix_table* pt,
                             const ogs_unit* units, int nUnits,
                             uint32_t flags, int W, const ogs_spf_out& out,
                             hipStream_t stream, int* unsupported) {
  // zero / negative metrics: the reference's extraction order, replayed
  if (flags & OGS_F_EXACT_ORDER) {
    return launch_spf_routes_exact(g, pt, units, nUnits, flags, W, out, stream);
  }
  // sources of more than 512 links: next-hop sets past 16 words, state in
  // HBM, runtime word count (push-style rounds: no reverse-slot reads)
  if (W > 16) {
    return launch_spf_routes_global_wide(g, pt, units, nUnits, flags, W, out, stream);
  }
  // exact widths that are not a power of two (three words for 65..96 links):
  // the fused frontier + route stream when it takes the launch, else the
  // runtime-width HBM kernels
  if (W & (W - 1)) {
    hipError_t err = hipSuccess;
    if (pt && try_ms_stream(g, *pt, units, nUnits, flags, W, out, stream, &err)) return err;
    return launch_spf_routes_global_wide(g, pt, units, nUnits, flags, W, out, stream);
  }
  // units too large for LDS (or the "spf_global" option): state in HBM
  if (use_global(g, W, flags)) {
    return launch_spf_routes_global(g, pt, units, nUnits, flags, W, out, stream);
  }
  ogs_prefix_table empty{};
  const ogs_prefix_table& p = pt ? *pt : empty;
  const int hasPrefixes = pt ? 1 : 0;
  const int uw = small_unit_width();
  const uint32_t maxA = hasPrefixes ? uint32_t(p.max_advertisements) : 0u;
  if (W == 1 && (uw == -1 || uw == 1)) {
    hipError_t err = hipSuccess;
    if (try_wave(g, p, hasPrefixes, units, nUnits, flags, out, maxA, stream,
                 &err)) {
      return err;
    }
  }
  // large shared topologies: multi-source edge-parallel kernel
  if ((uw == -1 && g.max_nodes > 256) || uw == 3) {
    hipError_t err = hipSuccess;
    if (hasPrefixes &&
        try_ms_stream(g, p, units, nUnits, flags, W, out, stream, &err)) {
      return err;
    }
    if (!hasPrefixes && !out.meta && !out.metric && !out.mask && !out.sel &&
        try_frontier(g, units, nUnits, flags, W, static_cast<uint32_t*>(out.dist),
                     out.nh, stream, &err)) {
      return err;
    }
    if (try_ms(g, p, hasPrefixes, units, nUnits, flags, W, out, stream, &err)) {
      return err;
    }
  }
  if (W == 1 && uw != 0 && uw != 3) {
    hipError_t err = hipSuccess;
    const int width = uw >= 64 ? uw : 0;
    const bool done = (flags & OGS_F_WIDE_METRIC)
        ? try_small<uint64_t, 1>(g, p, hasPrefixes, units, nUnits, flags, out,
                                 g.max_degree, maxA, width, stream, &err)
        : try_small<uint32_t, 1>(g, p, hasPrefixes, units, nUnits, flags, out,
                                 g.max_degree, maxA, width, stream, &err);
    if (done) return err;
  }
  if (flags & OGS_F_WIDE_METRIC) {
    return dispatch_d<uint64_t>(W, g, p, hasPrefixes, units, nUnits, flags,
                                out, stream, unsupported);
  }
  return dispatch_d<uint32_t>(W, g, p, hasPrefixes, units, nUnits, flags, out,
                              stream, unsupported);
}

}  // namespace ogs
