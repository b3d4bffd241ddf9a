// route_stream.hip — RouteDb streaming for large shared topologies (C3
// fabric all-sources: 2,080 sources x 208,000 prefixes = 432 M routes, 5.7 GB
// of route records per whole-node build; C4/C5 WAN batches).
//
// The route phase of an all-sources build is a pure HBM write stream: every
// (source, prefix) pair gets a compact record (flags|best, metric, link-slot
// mask). Doing it inside the SPF workgroup (spf_route_ms.hip's fused form)
// leaves it latency-bound: a few resident waves per CU, each walking the
// prefix table through a chain of dependent loads. Here it is its own
// launch, after the SPF launch has left dist / next-hop sets in HBM:
//
//  1. pfx_key_kernel — once per call, one thread per (topology, prefix):
//     folds the advertiser segment into one u32 key:
//       bits 0..20  the single advertiser's node id,
//       bit  30     prefix is IPv4 (the v4 gate is applied at run time),
//       bit  31     SLOW: several advertisements, minNexthop set, or an
//                   advertiser without adjacency DB -> full route_one.
//  2. route_stream_kernel — one workgroup per unit: turns the unit's SPF
//     state into one record per NODE in LDS (a single-advertiser prefix's
//     route depends only on its advertiser: SpfSolver.cpp:160-311 with a
//     one-entry segment), then streams the unit's prefix rows: per lane four
//     consecutive prefixes = one 16-B key load, LDS gathers, and one 16-B
//     non-temporal store per output array. SLOW prefixes run route_one
//     (route_core.h) against the unit's SPF state in HBM/L2.
// Results are identical to the fused kernels' (same route_core semantics;
// tests/test_gpu_parity.py compares both against the oracle).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "openr_gpu.h"
#include "route_core.h"
#include "route_stream.h"
#include "spf_lds.h"
#include "spf_core.h"
#include "engine.h"

namespace ogs {

__global__ __launch_bounds__(kBlock) void pfx_key_kernel(
    ogs_prefix_table pt, int numTopos, uint32_t* __restrict__ key) {
  const uint32_t Sp = uint32_t(pt.max_prefixes);
  const uint32_t t = blockIdx.y;
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (t >= uint32_t(numTopos) || p >= Sp) return;
  const uint32_t k = prefix_key(pt, t, p);
  key[size_t(t) * Sp + p] = k;
}

// Unit's SPF state as left in HBM by the SPF launch (ogs_spf_out layout).
template <int W>
struct HbmView {
  const uint32_t* d;  // dist + u*Sn
  const uint32_t* n;  // nh + u*W*Sn
  uint32_t Sn;
  __device__ __forceinline__ uint32_t dist(uint32_t v) const { return d[v]; }
  __device__ __forceinline__ uint32_t nh(uint32_t v, int w) const {
    return n[size_t(w) * Sn + v];
  }
};

// `parts` workgroups per unit, each streaming one 4-aligned prefix range.
template <int W>
__global__ __launch_bounds__(kBlock) void route_stream_kernel(
    ogs_graph g, ogs_prefix_table pt, const uint32_t* __restrict__ key,
    const ogs_unit* __restrict__ units, uint32_t flags,
    const uint32_t* __restrict__ sDist, const uint32_t* __restrict__ sNh,
    ogs_spf_out out, uint32_t parts) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  const uint32_t u = blockIdx.x / parts, part = blockIdx.x - u * parts;
  const ogs_unit unit = units[u];
  const uint32_t t = unit.topo, s = unit.src;
  const uint32_t nb = g.node_base[t];
  const uint32_t N = g.node_base[t + 1] - nb;
  const uint32_t Sn = uint32_t(g.max_nodes);
  const uint32_t Sp = uint32_t(pt.max_prefixes);
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const HbmView<W> sv{sDist + size_t(u) * Sn, sNh + size_t(u) * W * Sn, Sn};
  const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0,
                     (flags & OGS_F_V4_OVER_V6) != 0,
                     (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};

  // per-node records in LDS
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* rMeta = reinterpret_cast<uint32_t*>(smem);
  uint32_t* rMetric = rMeta + Sn;
  uint32_t* rMask = rMetric + Sn;  // [W][Sn]
  for (uint32_t v = tid; v < N; v += kBlock) {
    const uint32_t d = sv.dist(v);
    uint32_t m[W], cnt = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      m[w] = sv.nh(v, w);  // 0 for the source and unreachable nodes
      cnt += __popc(m[w]);
    }
    rMeta[v] = node_route_meta(v, s, d != kInf, cnt, nflags[v]);
    rMetric[v] = (v == s) ? kInf : d;
#pragma unroll
    for (int w = 0; w < W; ++w) rMask[w * Sn + v] = m[w];
  }
  __syncthreads();

  const uint32_t p0 = pt.pfx_base[t];
  const uint32_t P = pt.pfx_base[t + 1] - p0;
  const uint32_t span = ((P + parts - 1u) / parts + 3u) & ~3u;
  const uint32_t lo = min(P, part * span), hi = min(P, lo + span);
  auto rec = [&](uint32_t v, Rec<W>& r) {
    r.meta = rMeta[v];
    r.metric = rMetric[v];
#pragma unroll
    for (int w = 0; w < W; ++w) r.mask[w] = rMask[w * Sn + v];
  };
  if (out.meta && out.metric && out.mask && !out.sel) {  // unconditional 16-B stores
    stream_routes<W, false, true>(pt, key + size_t(t) * Sp, p0, P, Sp, u, s, nflags, sv, cfg,
                                  out, rec, nullptr, (flags & kFlagNtStores) != 0, lo, hi);
  } else {
    stream_routes<W>(pt, key + size_t(t) * Sp, p0, P, Sp, u, s, nflags, sv, cfg, out, rec,
                     nullptr, (flags & kFlagNtStores) != 0, lo, hi);
  }
}

// "route_stream" option for large shared topologies: 5 (default) the
// LDS-resident SPF and the route stream in one persistent launch
// (spf_lds.hip, spf_lds_route_kernel; topologies whose image does not fit
// LDS take form 2); 2 fused frontier SPF + route stream, one launch; 1 SPF
// launch then route-stream launch (dist / next-hop sets through HBM); 4 the
// LDS-resident SPF then the route stream over parts. C3 (profiles/
// r04_lds_groups_ab.log): 5 at 1.10 / 0.57 / 0.31 / 0.17 ms for 1 / 2 / 4 / 8
// shards vs 2 at 1.22 / 0.72 / 0.41 / 0.26. (0, the fused multi-source
// kernel as the C3 form, and 3, the split pipelined over unit chunks on two
// streams -- 1.40-1.64 vs 1.33 ms on C3, profiles/r03_c3_pipelined_split_
// ab.log -- were removed in round 4; the multi-source kernel remains the
// fallback where neither form applies.)
// EngineOptions::routeStream (engine.h), default 5
// "route_store_nt" option, bits: 1 the RouteDb stream's 16-B stores are
// non-temporal (else ordinary write-back stores), 2 the wave kernel's output
// stores are. Default 2. The bare C3 store pattern drains faster with
// ordinary stores (tools/store_pattern.hip: 5.4 vs 5.0 TB/s); the C3 build
// gains 0.5-2 % from them (1.278 vs 1.283 ms mean of 5, 1.282-1.295 vs
// 1.303-1.325 ms), the C2 wave kernel loses 3 % (10.9 vs 10.6 us):
// profiles/r03_store_pattern.log, r03_store_nt_ab.log.
// EngineOptions::routeStoreNt (engine.h), default 2

bool try_ms(const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes,
            const ogs_unit* units, int nUnits, uint32_t flags, int W,
            const ogs_spf_out& out, hipStream_t stream, hipError_t* err);
bool frontier_fits(const ogs_graph& g, uint32_t flags, int W);
size_t chunk_scratch_bytes(const ogs_graph& g);
size_t desc_scratch_bytes(const ogs_graph& g);
hipError_t launch_frontier_spf(const ogs_graph& g, const ogs_unit* units,
                               int nUnits, uint32_t flags, int W,
                               uint32_t* dist, uint32_t* nh, void* scratch,
                               hipStream_t stream);
hipError_t launch_frontier_routes(const ogs_graph& g, const ogs_prefix_table& pt,
                                  const uint32_t* key, const ogs_unit* units,
                                  int nUnits, uint32_t flags, int W,
                                  const ogs_spf_out& out, void* scratch,
                                  hipStream_t stream);
void stream_parts(int nUnits, int W, int P, int* parts);

template <int W>
hipError_t launch_route_stream(const ogs_graph& g, const ogs_prefix_table& pt,
                               const uint32_t* key, const ogs_unit* units,
                               int nUnits, uint32_t flags, const uint32_t* dist,
                               const uint32_t* nh, const ogs_spf_out& out,
                               hipStream_t stream, int parts = 1) {
  const size_t lds = size_t(g.max_nodes) * (2 + W) * 4;
  auto k = route_stream_kernel<W>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       int(lds));
    if (e != hipSuccess) return e;
  }
  if (opts().routeStoreNt & 1) flags |= kFlagNtStores;
  hipLaunchKernelGGL(k, dim3(unsigned(nUnits) * unsigned(parts)), dim3(kBlock), lds, stream, g,
                     pt, key, units, flags, dist, nh, out, uint32_t(parts));
  return hipGetLastError();
}

static size_t round256(size_t x) { return (x + 255) & ~size_t(255); }

// SPF only through the frontier kernel (callers without a prefix table).
bool try_frontier(const ogs_graph& g, const ogs_unit* units, int nUnits,
                  uint32_t flags, int W, uint32_t* dist, uint32_t* nh,
                  hipStream_t stream, hipError_t* err) {
  if (!dist || !nh || !g.edge_src || !frontier_fits(g, flags, W)) return false;
  if (W != 1 && W != 2 && W != 4 && W != 8) return false;
  void* ws = nullptr;
  *err = workspace(chunk_scratch_bytes(g), stream, &ws);
  if (*err != hipSuccess) return true;
  *err = launch_frontier_spf(g, units, nUnits, flags, W, dist, nh, ws, stream);
  return true;
}

hipError_t launch_frontier_variants(const ogs_graph& g, const ogs_prefix_table& pt,
                                    const uint32_t* key, const ogs_unit* units,
                                    int n, uint32_t flags, int W,
                                    const ogs_spf_out& out,
                                    const ogs_unit_mods* mods,
                                    ogs_route_diff* diff, void* scratch,
                                    hipStream_t stream);

// ogs_spf_routes_variants: key fold + zeroed diff bitmap + fused frontier
// SPF / RouteDb / diff launch. *unsupported when outside the frontier path.
hipError_t launch_variants(const ogs_graph& g, const ogs_prefix_table& pt,
                           const ogs_unit* units, int nUnits,
                           const ogs_unit_mods* mods, ogs_route_diff* diff,
                           uint32_t flags, int W, const ogs_spf_out& out,
                           hipStream_t stream, int* unsupported) {
  if (!g.edge_src || (flags & OGS_F_WIDE_METRIC) || !frontier_fits(g, flags, W) ||
      (W != 1 && W != 2 && W != 4)) {
    *unsupported = 1;
    return hipSuccess;
  }
  const size_t Sp = size_t(pt.max_prefixes);
  const size_t keyBytes = round256(size_t(g.num_topos) * Sp * 4);
  void* ws = nullptr;
  // after the keys: the chunk lists (full recompute) or the repair's
  // descendant rows (OGS_F_INCREMENTAL) -- one launch uses one of them
  const size_t scratchBytes = std::max(chunk_scratch_bytes(g), desc_scratch_bytes(g));
  hipError_t e = workspace(keyBytes + scratchBytes, stream, &ws);
  if (e != hipSuccess) return e;
  uint32_t* key = static_cast<uint32_t*>(ws);
  if (diff) {
    e = hipMemsetAsync(diff->changed, 0, size_t(nUnits) * ((Sp + 31) / 32) * 4, stream);
    if (e != hipSuccess) return e;
  }
  if (Sp > 0) {
    hipLaunchKernelGGL(pfx_key_kernel, dim3(unsigned((Sp + kBlock - 1) / kBlock),
                                            unsigned(g.num_topos)),
                       dim3(kBlock), 0, stream, pt, g.num_topos, key);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return launch_frontier_variants(g, pt, key, units, nUnits, flags, W, out, mods,
                                  diff, static_cast<char*>(ws) + keyBytes, stream);
}

// Large shared topologies with a prefix table: key fold, then either the
// fused frontier SPF + stream launch (route_stream 2), or an SPF launch
// (frontier / multi-source sweep) and a route-stream launch (route_stream 1).
bool try_ms_stream(const ogs_graph& g, const ogs_prefix_table& pt,
                   const ogs_unit* units, int nUnits, uint32_t flags, int W,
                   const ogs_spf_out& out, hipStream_t stream, hipError_t* err) {
  if (!g.edge_src || (flags & OGS_F_WIDE_METRIC)) return false;
  if (W != 1 && W != 2 && W != 3 && W != 4) return false;
  if (size_t(g.max_nodes) * (2 + W) * 4 > 160 * 1024) return false;
  const size_t Sn = size_t(g.max_nodes), Sp = size_t(pt.max_prefixes);
  const bool frontier = frontier_fits(g, flags, W);
  // route_stream 4: SPF with the topology in LDS (spf_lds.hip), then the
  // stream over `parts` workgroups per unit; 5: both in one persistent launch
  const bool ldsForm = (opts().routeStream == 4 || opts().routeStream == 5) && Sp > 0;
  const size_t ldsBytes = ldsForm ? lds_scratch_bytes(g, W, nUnits) : 0;
  const bool ldsSplit = ldsBytes != 0;
  const bool fused = (opts().routeStream == 2 || (ldsForm && !ldsSplit)) && frontier;
  // three-word sets (65..96 links: C3 FSWs) through the frontier forms only
  if (W == 3 && !fused && !ldsSplit) return false;
  const size_t keyBytes = round256(size_t(g.num_topos) * Sp * 4);
  const size_t chunkBytes = ldsSplit ? round256(ldsBytes) : frontier ? chunk_scratch_bytes(g) : 0;
  const size_t distBytes = (fused || out.dist) ? 0 : round256(size_t(nUnits) * Sn * 4);
  const size_t nhBytes = (fused || out.nh) ? 0 : round256(size_t(nUnits) * W * Sn * 4);
  void* ws = nullptr;
  *err = workspace(keyBytes + chunkBytes + distBytes + nhBytes, stream, &ws);
  if (*err != hipSuccess) return true;
  char* base = static_cast<char*>(ws);
  uint32_t* key = reinterpret_cast<uint32_t*>(base);
  void* chunkScratch = base + keyBytes;
  ogs_spf_out spf{};
  spf.dist = out.dist ? out.dist : base + keyBytes + chunkBytes;
  spf.nh = out.nh ? out.nh
                  : reinterpret_cast<uint32_t*>(base + keyBytes + chunkBytes + distBytes);
  if (ldsSplit) {
    uint32_t* d = static_cast<uint32_t*>(spf.dist);
    if (opts().routeStream == 5) {  // the prep is part of that launch (or its own, A/B)
      const LdsRouteGroup one{units, nUnits, W, d, spf.nh, out};
      *err = launch_spf_lds_routes(g, pt, key, lds_key16(g), &one, 1, flags, chunkScratch,
                                   stream);
      return true;
    }
    // form 4: one prep launch (LDS images, weight partials, counters, u32
    // route keys), the SPF launch, the stream launch
    *err = launch_lds_prep(g, &pt, key, false, W, nUnits, chunkScratch, stream);
    if (*err != hipSuccess) return true;
    *err = launch_spf_lds(g, units, nUnits, flags, W, d, spf.nh, chunkScratch, stream);
    if (*err != hipSuccess) return true;
    int parts = 1;
    stream_parts(nUnits, W, int(Sp), &parts);
    switch (W) {
      case 1: *err = launch_route_stream<1>(g, pt, key, units, nUnits, flags, d, spf.nh, out, stream, parts); break;
      case 2: *err = launch_route_stream<2>(g, pt, key, units, nUnits, flags, d, spf.nh, out, stream, parts); break;
      case 3: *err = launch_route_stream<3>(g, pt, key, units, nUnits, flags, d, spf.nh, out, stream, parts); break;
      default: *err = launch_route_stream<4>(g, pt, key, units, nUnits, flags, d, spf.nh, out, stream, parts); break;
    }
    return true;
  }
  if (Sp > 0) {
    hipLaunchKernelGGL(pfx_key_kernel, dim3(unsigned((Sp + kBlock - 1) / kBlock),
                                            unsigned(g.num_topos)),
                       dim3(kBlock), 0, stream, pt, g.num_topos, key);
    *err = hipGetLastError();
    if (*err != hipSuccess) return true;
  }
  if (fused) {
    *err = launch_frontier_routes(g, pt, key, units, nUnits, flags, W, out,
                                  chunkScratch, stream);
    return true;
  }
  if (frontier) {
    *err = launch_frontier_spf(g, units, nUnits, flags, W,
                               static_cast<uint32_t*>(spf.dist), spf.nh,
                               chunkScratch, stream);
  } else if (!try_ms(g, pt, 0, units, nUnits, flags, W, spf, stream, err)) {
    return false;
  }
  if (*err != hipSuccess || Sp == 0) return true;
  const uint32_t* d = static_cast<const uint32_t*>(spf.dist);
  switch (W) {
    case 1: *err = launch_route_stream<1>(g, pt, key, units, nUnits, flags, d, spf.nh, out, stream); break;
    case 2: *err = launch_route_stream<2>(g, pt, key, units, nUnits, flags, d, spf.nh, out, stream); break;
    default: *err = launch_route_stream<4>(g, pt, key, units, nUnits, flags, d, spf.nh, out, stream); break;
  }
  return true;
}


hipError_t launch_spf_routes(const ogs_graph& g, const ogs_prefix_table* pt,
                             const ogs_unit* units, int nUnits, uint32_t flags, int W,
                             const ogs_spf_out& out, hipStream_t stream, int* unsupported);
int small_unit_width();
bool use_global(const ogs_graph& g, int W, uint32_t flags);

// ogs_spf_routes_groups: every group's RouteDbs over one graph / prefix
// table. With route_stream 5 on a large shared topology whose image fits
// LDS for the widest group: ONE persistent launch for all groups (widest
// first), the prep as its first items. Otherwise one launch_spf_routes per group, in
// order on the stream -- the same outputs either way.
hipError_t launch_spf_routes_groups(const ogs_graph& g, const ogs_prefix_table* pt,
                                    const ogs_route_group* groups, int n, uint32_t flags,
                                    hipStream_t stream, int* unsupported) {
  std::vector<LdsRouteGroup> lg;
  int Wmax = 1, U = 0;
  for (int i = 0; i < n; ++i) {
    if (groups[i].n_units <= 0) continue;
    lg.push_back(LdsRouteGroup{groups[i].units, groups[i].n_units, groups[i].nh_words,
                               nullptr, nullptr, groups[i].out});
    Wmax = std::max(Wmax, groups[i].nh_words);
    U += groups[i].n_units;
  }
  const size_t Sp = pt ? size_t(pt->max_prefixes) : 0;
  // the same gating as launch_spf_routes before its large-topology forms:
  // topologies of <= 256 nodes go to the wave / small kernels, and
  // use_global() (deep graphs past the frontier's LDS budget, or the
  // "spf_global" option) to the HBM-state frontier -- so a group gets the
  // same engine here as through ogs_spf_routes
  bool one = opts().routeStream == 5 && pt && Sp > 0 && g.edge_src && g.max_nodes > 256 &&
      !(flags & (OGS_F_EXACT_ORDER | OGS_F_WIDE_METRIC)) && small_unit_width() == -1 &&
      !lg.empty() && lg.size() <= 4 && Wmax <= 4 && !use_global(g, Wmax, flags);
  const size_t ldsBytes = one ? lds_scratch_bytes(g, Wmax, U) : 0;
  if (!ldsBytes) {
    for (const LdsRouteGroup& x : lg) {
      const hipError_t e = launch_spf_routes(g, pt, x.units, x.n, flags, x.W, x.out, stream,
                                             unsupported);
      if (e != hipSuccess || *unsupported) return e;
    }
    return hipSuccess;
  }
  std::stable_sort(lg.begin(), lg.end(),
                   [](const LdsRouteGroup& a, const LdsRouteGroup& b) { return a.W > b.W; });
  const size_t Sn = size_t(g.max_nodes);
  const size_t keyBytes = round256(size_t(g.num_topos) * Sp * 4);
  size_t rows = 0;
  for (const LdsRouteGroup& x : lg) {
    if (!x.out.dist) rows += round256(size_t(x.n) * Sn * 4);
    if (!x.out.nh) rows += round256(size_t(x.n) * x.W * Sn * 4);
  }
  void* ws = nullptr;
  hipError_t e = workspace(keyBytes + round256(ldsBytes) + rows, stream, &ws);
  if (e != hipSuccess) return e;
  char* base = static_cast<char*>(ws);
  uint32_t* key = reinterpret_cast<uint32_t*>(base);
  void* scratch = base + keyBytes;
  char* at = base + keyBytes + round256(ldsBytes);
  for (LdsRouteGroup& x : lg) {
    if (x.out.dist) {
      x.dist = static_cast<uint32_t*>(x.out.dist);
    } else {
      x.dist = reinterpret_cast<uint32_t*>(at);
      at += round256(size_t(x.n) * Sn * 4);
    }
    if (x.out.nh) {
      x.nh = x.out.nh;
    } else {
      x.nh = reinterpret_cast<uint32_t*>(at);
      at += round256(size_t(x.n) * x.W * Sn * 4);
    }
  }
  return launch_spf_lds_routes(g, *pt, key, lds_key16(g), lg.data(), int(lg.size()), flags,
                               scratch, stream);
}
}  // namespace ogs
