// spf_route_ms.hip — multi-source SPF + RouteDb for large shared topologies
// (C3 fabric all-sources: N = 2080, E = 43,008, 208,000 prefixes; C4/C5
// WAN graphs).
//
// One WORKGROUP per group of G units that share a topology (all-sources
// batches list (topology, source) units consecutively). Same results as
// spf_route.hip (reference mapping and fixpoint argument in its header and
// spf_core.h); the work is laid out for a graph that does not fit in LDS but
// is shared by thousands of sources, so its CSR stays L2-resident:
//  * SPF is EDGE-parallel: each round every thread streams a coalesced slice
//    of the topology's directed edges (ogs_graph.edges + edge_src, the row
//    owner of each edge) and relaxes all G sources from one edge read:
//      dist phase: atomicMin(dist_g[v], dist_g[u] + w) until a round
//                  changes nothing (chaotic Bellman-Ford);
//      nh phase:   for tight edges (dist_g[u] + w == dist_g[v]) OR the
//                  predecessor's next-hop set, or the source's link slot when
//                  u is the source (LinkState.cpp:795-812), into nh_g[v]
//                  until no bit is added (the least fixpoint = the union of
//                  the shortest-path DAG, exactly the reference's NH sets);
//    edges out of hard-drained non-source nodes never relax
//    (LinkState.cpp:741-752);
//  * RouteDb: one thread per prefix reads the shared prefix table ONCE and
//    writes the G sources' route records (single-advertiser prefixes take a
//    straight-line path), with non-temporal stores so the write stream does
//    not evict the CSR / prefix table from L2.
// LDS per workgroup: dist[N][G] u32 + nh[N][G][W] u32.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "route_core.h"
#include "spf_core.h"
#include "engine.h"

namespace ogs {

// SPF state of source g inside the interleaved multi-source arrays.
template <int G, int W>
struct MsView {
  const uint32_t* d;  // dist[v * G + g]
  const uint32_t* n;  // nh[(v * G + g) * W + w]
  int g;
  __device__ __forceinline__ uint32_t dist(uint32_t v) const {
    return d[v * G + g];
  }
  __device__ __forceinline__ uint32_t nh(uint32_t v, int w) const {
    return n[(v * G + g) * W + w];
  }
};

template <typename T>
__device__ __forceinline__ void nt_store(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}

// Route for a prefix with exactly one advertisement, any next-hop width
// (same result as route_one on a one-entry segment).
template <int W, typename View>
__device__ __forceinline__ void route_single_w(uint32_t n, int64_t minNh,
                                               uint32_t s, uint8_t nf,
                                               const View& sv, uint32_t& meta,
                                               uint32_t& metric,
                                               uint32_t (&mask)[W]) {
  meta = (n == s) ? OGS_ROUTE_LOCAL : 0u;
  metric = 0xFFFFFFFFu;
#pragma unroll
  for (int w = 0; w < W; ++w) mask[w] = 0u;
  const uint32_t d = (n != OGS_NODE_NONE) ? sv.dist(n) : 0xFFFFFFFFu;
  if (d == 0xFFFFFFFFu) {
    meta |= OGS_REASON_UNREACHABLE << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  meta |= OGS_ROUTE_SELECTED;  // best index 0
  if (nf & (OGS_NODE_OVERLOADED | OGS_NODE_METRICINC)) meta |= OGS_ROUTE_DRAINED;
  if (n == s) {
    meta |= OGS_REASON_SELF << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    mask[w] = sv.nh(n, w);
    cnt += __popc(mask[w]);
  }
  metric = d;
  if (cnt == 0) {
    meta |= OGS_REASON_NO_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
  } else if (minNh != INT64_MIN && static_cast<uint64_t>(minNh) > cnt) {
    meta |= OGS_REASON_MIN_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
  } else {
    meta |= OGS_ROUTE_VALID;
  }
}

template <int G, int W>
__global__ __launch_bounds__(kBlock) void spf_route_ms_kernel(
    ogs_graph g, ogs_prefix_table pt, int hasPrefixes,
    const ogs_unit* __restrict__ units, int nUnits, uint32_t flags,
    ogs_spf_out out) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  const int uBeg = blockIdx.x * G;
  const int uEnd = min(uBeg + G, nUnits);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t Nmax = g.max_nodes;
  uint32_t* dist = reinterpret_cast<uint32_t*>(smem);
  uint32_t* nh = dist + ((Nmax * G + 3u) & ~3u);
  const bool hop = flags & OGS_F_HOP_METRIC;
  const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0,
                     (flags & OGS_F_V4_OVER_V6) != 0,
                     (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};

  // consecutive units sharing a topology are solved together
  for (int first = uBeg; first < uEnd;) {
    const uint32_t topo = units[first].topo;
    uint32_t src[G];
    int gc = 0;
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const bool take = first + k < uEnd && gc == k &&
          units[first + k].topo == topo;
      src[k] = take ? units[first + k].src : 0xFFFFFFFFu;
      gc += take ? 1 : 0;
    }
    const uint32_t nb = g.node_base[topo];
    const uint32_t N = g.node_base[topo + 1] - nb;
    const uint32_t e0 = g.row_ptr[nb];
    const uint32_t E = g.row_ptr[nb + N] - e0;
    const uint64_t* __restrict__ edges = g.edges + e0;
    const uint32_t* __restrict__ esrc = g.edge_src + e0;

    for (uint32_t v = tid; v < N; v += kBlock) {
#pragma unroll
      for (int k = 0; k < G; ++k) {
        dist[v * G + k] = (v == src[k]) ? 0u : kInf;
#pragma unroll
        for (int w = 0; w < W; ++w) nh[(v * G + k) * W + w] = 0u;
      }
    }
    __syncthreads();

    // ---- dist phase ---------------------------------------------------------
    for (;;) {
      bool changed = false;
      for (uint32_t e = tid; e < E; e += kBlock) {
        const uint64_t x = edges[e];
        const uint32_t v = esrc[e];
        const uint32_t lo = static_cast<uint32_t>(x);
        if (lo & OGS_EDGE_DOWN) continue;
        const uint32_t u = edge_dst(lo);
        const bool ovl = lo & OGS_EDGE_DST_OVERLOADED;
        const uint32_t w = hop ? 1u : static_cast<uint32_t>(x >> 32);
#pragma unroll
        for (int k = 0; k < G; ++k) {
          if (k >= gc || (ovl && u != src[k])) continue;
          const uint32_t du = dist[u * G + k];
          if (du == kInf) continue;
          const uint32_t cand = du + w;
          if (cand < dist[v * G + k]) {
            atomicMin(&dist[v * G + k], cand);
            changed = true;
          }
        }
      }
      if (!__syncthreads_or(changed)) break;
    }

    // ---- next-hop phase (least fixpoint over the shortest-path DAG) -------
    for (;;) {
      bool changed = false;
      for (uint32_t e = tid; e < E; e += kBlock) {
        const uint64_t x = edges[e];
        const uint32_t v = esrc[e];
        const uint32_t lo = static_cast<uint32_t>(x);
        if (lo & OGS_EDGE_DOWN) continue;
        const uint32_t u = edge_dst(lo);
        const bool ovl = lo & OGS_EDGE_DST_OVERLOADED;
        const uint32_t w = hop ? 1u : static_cast<uint32_t>(x >> 32);
#pragma unroll
        for (int k = 0; k < G; ++k) {
          if (k >= gc || (ovl && u != src[k])) continue;
          const uint32_t du = dist[u * G + k];
          if (du == kInf || du + w != dist[v * G + k]) continue;
          uint32_t* nv = &nh[(v * G + k) * W];
          if (u == src[k]) {
            const uint32_t r = edge_rslot(lo);
            const uint32_t bit = 1u << (r & 31u);
            if (int(r >> 5) < W && !(nv[r >> 5] & bit)) {
              atomicOr(&nv[r >> 5], bit);
              changed = true;
            }
          } else {
            const uint32_t* nu = &nh[(u * G + k) * W];
#pragma unroll
            for (int wd = 0; wd < W; ++wd) {
              const uint32_t add = nu[wd] & ~nv[wd];
              if (add) {
                atomicOr(&nv[wd], add);
                changed = true;
              }
            }
          }
        }
      }
      if (!__syncthreads_or(changed)) break;
    }

    // ---- SPF outputs ----------------------------------------------------------
    const uint32_t Sn = g.max_nodes;
    for (int k = 0; k < gc; ++k) {
      const size_t u = size_t(first + k);
      for (uint32_t v = tid; v < N; v += kBlock) {
        if (out.dist) nt_store(static_cast<uint32_t*>(out.dist) + u * Sn + v, dist[v * G + k]);
        if (out.nh) {
#pragma unroll
          for (int w = 0; w < W; ++w) {
            nt_store(out.nh + (u * W + w) * Sn + v, nh[(v * G + k) * W + w]);
          }
        }
      }
    }

    // ---- fused RouteDb: prefix table read once for all sources --------------
    if (hasPrefixes) {
      const uint8_t* __restrict__ nflags = g.node_flags + nb;
      const uint32_t p0 = pt.pfx_base[topo];
      const uint32_t P = pt.pfx_base[topo + 1] - p0;
      const uint32_t Sp = pt.max_prefixes;
      for (uint32_t p = tid; p < P; p += kBlock) {
        const uint32_t gp = p0 + p;
        const uint32_t a0 = pt.adv_off[gp], a1 = pt.adv_off[gp + 1];
        const uint8_t pf = pt.pfx_flags[gp];
        const bool gated = (pf & OGS_PFX_V4) && !cfg.enableV4 && !cfg.v4OverV6;
        const bool single = a1 - a0 == 1 && !gated;
        uint32_t n = OGS_NODE_NONE;
        int64_t minNh = INT64_MIN;
        uint8_t nf = 0;
        if (single) {
          n = pt.adv_node[a0];
          if (pf & OGS_PFX_HAS_MIN_NH) minNh = pt.adv_min_nh[a0];
          if (n != OGS_NODE_NONE) nf = nflags[n];
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
          if (k >= gc) continue;
          const MsView<G, W> sv{dist, nh, k};
          uint32_t meta, metric, selBits, mask[W];
          if (single) {
            route_single_w<W>(n, minNh, src[k], nf, sv, meta, metric, mask);
            selBits = (meta & OGS_ROUTE_SELECTED) ? 1u : 0u;
          } else {
            route_one<uint32_t, W>(pt, gp, src[k], nflags, sv, cfg, meta, metric,
                                   mask, selBits);
          }
          const size_t u = size_t(first + k);
          const size_t o = u * Sp + p;
          if (out.meta) nt_store(out.meta + o, meta);
          if (out.metric) nt_store(static_cast<uint32_t*>(out.metric) + o, metric);
          if (out.sel) nt_store(out.sel + o, selBits);
          if (out.mask) {
#pragma unroll
            for (int w = 0; w < W; ++w) nt_store(out.mask + (u * W + w) * Sp + p, mask[w]);
          }
        }
      }
    }
    first += gc;
    __syncthreads();  // LDS reused by the next group of this workgroup
  }
}

uint32_t ms_lds_bytes(int maxNodes, int G, int W) {
  const uint64_t d = (uint64_t(maxNodes) * G + 3u) & ~uint64_t(3u);
  return uint32_t((d + uint64_t(maxNodes) * G * W) * 4u);
}

template <int G, int W>
hipError_t launch_ms(const ogs_graph& g, const ogs_prefix_table& pt,
                     int hasPrefixes, const ogs_unit* units, int nUnits,
                     uint32_t flags, const ogs_spf_out& out, hipStream_t stream) {
  const size_t lds = ms_lds_bytes(g.max_nodes, G, W);
  auto k = spf_route_ms_kernel<G, W>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       int(lds));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3((nUnits + G - 1) / G), dim3(kBlock), lds, stream,
                     g, pt, hasPrefixes, units, nUnits, flags, out);
  return hipGetLastError();
}

// "ms_group" option: 0 automatic, else force G (1, 2 or 4) when it fits.
// EngineOptions::msGroup (engine.h), default 0

template <int W>
bool try_ms_w(const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes,
              const ogs_unit* units, int nUnits, uint32_t flags,
              const ogs_spf_out& out, hipStream_t stream, hipError_t* err) {
  constexpr uint32_t kBudget = 80 * 1024;  // two workgroups per CU
  constexpr uint32_t kMax = 160 * 1024;
  const int N = g.max_nodes;
  for (int G : {4, 2, 1}) {
    if (opts().msGroup && G != opts().msGroup) continue;
    const uint32_t b = ms_lds_bytes(N, G, W);
    if (b > (G == 1 || opts().msGroup ? kMax : kBudget)) continue;
    switch (G) {
      case 4: *err = launch_ms<4, W>(g, pt, hasPrefixes, units, nUnits, flags, out, stream); return true;
      case 2: *err = launch_ms<2, W>(g, pt, hasPrefixes, units, nUnits, flags, out, stream); return true;
      default: *err = launch_ms<1, W>(g, pt, hasPrefixes, units, nUnits, flags, out, stream); return true;
    }
  }
  return false;
}

bool try_ms(const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes,
            const ogs_unit* units, int nUnits, uint32_t flags, int W,
            const ogs_spf_out& out, hipStream_t stream, hipError_t* err) {
  if (!g.edge_src || (flags & OGS_F_WIDE_METRIC)) return false;
  switch (W) {
    case 1: return try_ms_w<1>(g, pt, hasPrefixes, units, nUnits, flags, out, stream, err);
    case 2: return try_ms_w<2>(g, pt, hasPrefixes, units, nUnits, flags, out, stream, err);
    case 4: return try_ms_w<4>(g, pt, hasPrefixes, units, nUnits, flags, out, stream, err);
    default: return false;
  }
}

}  // namespace ogs
