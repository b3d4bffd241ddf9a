// route_multiarea.hip — RouteDb of a multi-area routing domain (one
// LinkState per area), one thread per (source,
// prefix), from the per-(source, area) SPF results of a prior launch.
//
// Reference: SpfSolver::createRouteForPrefix (SpfSolver.cpp:160-311):
//  1. v4 gate (169-176);
//  2. an entry (node, area) survives iff node is in the source's SPF of
//     ITS area; the source itself always is (runSpf records the source
//     first even in an area without its adjacency DB, LinkState.cpp:
//     730-734); localPrefixConsidered if any entry is the source (194-214);
//  3. selectBestRoutes (455-486): hard-drain filter by each entry's own
//     area (filterHardDrainedNodes 526-541), best-route selection
//     (LsdbUtil.cpp:760-823, SHORTEST_DISTANCE; soft drain = metric
//     increment > 0 in the entry's area) or all; bestNodeArea = the
//     source's entry if selected under best-route selection
//     (selectBestNodeArea, LsdbUtil.cpp:700-711), else the smallest
//     (node, area) key; drained iff the best node is overloaded or has a
//     metric increment in its area (543-551);
//  4. self selected -> no route (253-258);
//  5. for every area holding a selected entry (hasBestRoutesInArea,
//     LsdbUtil.cpp:374-389), getNextHopsWithMetric over ALL selected node
//     NAMES looked up in that area's SPF (648-688, the A.4 quirk), then the
//     link filter (690-767, folded into the link-slot bitsets);
//  6. keep the union of the areas with the smallest metric (290-301);
//  7. addBestPaths: no next hop / min-nexthop (595-639).
// Per-area next-hop masks are over the source's CSR row in that area.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "spf_core.h"

namespace ogs {

template <typename D, int W>
__global__ __launch_bounds__(kBlock) void route_multiarea_kernel(
    ogs_graph g, ogs_prefix_table pt, ogs_area_table at,
    const uint32_t* __restrict__ units, const uint32_t* __restrict__ spfRow,
    const D* __restrict__ sDist, const uint32_t* __restrict__ sNh,
    uint32_t flags, ogs_spf_out out, int Wr) {
  constexpr D kInf = DistInf<D>::value;
  // W == 0: next-hop sets of runtime width Wr (sources of 512+ links)
  const int WW = W > 0 ? W : Wr;
  const uint32_t u = blockIdx.y;
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t p0 = pt.pfx_base[0];
  const uint32_t P = pt.pfx_base[1] - p0;
  if (p >= P) return;
  const uint32_t A = uint32_t(at.num_areas);
  const uint32_t Sn = uint32_t(g.max_nodes);
  const uint32_t Sp = uint32_t(pt.max_prefixes);
  const uint32_t S = units[u];  // source name id
  const uint32_t* __restrict__ row = spfRow + size_t(u) * A;
  const bool enableV4 = flags & OGS_F_ENABLE_V4;
  const bool v4OverV6 = flags & OGS_F_V4_OVER_V6;
  const bool brs = flags & OGS_F_BEST_ROUTE_SELECTION;

  // SPF of (source, area b) looked up by node NAME
  auto distOf = [&](uint32_t b, uint32_t name) -> D {
    if (name == S) return D(0);
    const uint32_t r = row[b];
    const uint32_t v = at.name_local[size_t(name) * A + b];
    if (r == OGS_NODE_NONE || v == OGS_NODE_NONE) return kInf;
    return sDist[size_t(r) * Sn + v];
  };
  // reached in (source, area b)'s SPF: the settled bitset of exact-order
  // rows when given (a wrapped u64 distance may be all ones), else the
  // all-ones sentinel
  const size_t RW = (size_t(Sn) + 31) / 32;
  auto reachOf = [&](uint32_t b, uint32_t name) -> bool {
    if (name == S) return true;
    const uint32_t r = row[b];
    const uint32_t v = at.name_local[size_t(name) * A + b];
    if (r == OGS_NODE_NONE || v == OGS_NODE_NONE) return false;
    if (at.reached) return ((at.reached[size_t(r) * RW + (v >> 5)] >> (v & 31u)) & 1u) != 0u;
    return sDist[size_t(r) * Sn + v] != kInf;
  };
  auto nhOf = [&](uint32_t b, uint32_t name, int w) -> uint32_t {
    const uint32_t r = row[b];
    const uint32_t v = at.name_local[size_t(name) * A + b];
    if (name == S || r == OGS_NODE_NONE || v == OGS_NODE_NONE) return 0u;
    return sNh[(size_t(r) * WW + w) * Sn + v];
  };
  // node flags of an entry in its own area (no adjacency DB: none set)
  auto flagsOf = [&](uint32_t a) -> uint8_t {
    const uint32_t v = pt.adv_node[a];
    if (v == OGS_NODE_NONE) return 0;
    return g.node_flags[g.node_base[at.adv_area[a]] + v];
  };

  const uint32_t gp = p0 + p;
  uint32_t meta = 0, selBits = 0;
  const size_t o = size_t(u) * Sp + p;
  auto finish = [&](uint32_t m, D d) {
    if (out.meta) out.meta[o] = m;
    if (out.metric) static_cast<D*>(out.metric)[o] = d;
    if (out.sel) out.sel[o] = selBits;
  };
  auto clearMasks = [&]() {
    if (!out.mask) return;
    for (uint32_t b = 0; b < A; ++b) {
      for (int w = 0; w < WW; ++w) out.mask[((size_t(u) * A + b) * WW + w) * Sp + p] = 0u;
    }
  };

  const uint8_t pflags = pt.pfx_flags[gp];
  if ((pflags & OGS_PFX_V4) && !enableV4 && !v4OverV6) {
    clearMasks();
    finish(OGS_REASON_V4_DISABLED << OGS_ROUTE_REASON_SHIFT, kInf);
    return;
  }
  const uint32_t a0 = pt.adv_off[gp], a1 = pt.adv_off[gp + 1];

  // pass 1: reachability in the entry's own area, local, hard-drain census
  bool local = false;
  uint32_t nReach = 0, nReachUp = 0;
  for (uint32_t a = a0; a < a1; ++a) {
    const uint32_t name = at.adv_name[a];
    if (name == S) local = true;
    if (reachOf(at.adv_area[a], name)) {
      ++nReach;
      nReachUp += (flagsOf(a) & OGS_NODE_OVERLOADED) ? 0u : 1u;
    }
  }
  if (local) meta |= OGS_ROUTE_LOCAL;
  if (nReach == 0) {
    clearMasks();
    finish(meta | (OGS_REASON_UNREACHABLE << OGS_ROUTE_REASON_SHIFT), kInf);
    return;
  }
  const bool dropOverloaded = nReachUp != 0;
  auto filtered = [&](uint32_t a) {
    return reachOf(at.adv_area[a], at.adv_name[a]) &&
        !(dropOverloaded && (flagsOf(a) & OGS_NODE_OVERLOADED));
  };
  int32_t bD = INT32_MIN, bP = INT32_MIN, bS = INT32_MIN, bDist = INT32_MAX;
  auto drainKey = [&](uint32_t a, const int4& m) {
    return -((m.x != 0 || (flagsOf(a) & OGS_NODE_SOFTDRAIN)) ? 1 : 0);
  };
  if (brs) {
    for (uint32_t a = a0; a < a1; ++a) {
      if (!filtered(a)) continue;
      const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
      const int32_t d = drainKey(a, m);
      if (d > bD || (d == bD && (m.y > bP || (m.y == bP && m.z > bS)))) {
        bD = d;
        bP = m.y;
        bS = m.z;
      }
    }
    for (uint32_t a = a0; a < a1; ++a) {
      if (!filtered(a)) continue;
      const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
      if (drainKey(a, m) == bD && m.y == bP && m.z == bS && m.w < bDist) bDist = m.w;
    }
  }
  auto selected = [&](uint32_t a) {
    if (!filtered(a)) return false;
    if (!brs) return true;
    const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
    return drainKey(a, m) == bD && m.y == bP && m.z == bS && m.w == bDist;
  };

  // selected set: best entry, self, areas holding selected entries
  bool self = false;
  uint32_t bestIdx = 0xFFFFFFFFu, selfIdx = 0xFFFFFFFFu;
  for (uint32_t a = a0; a < a1; ++a) {
    if (!selected(a)) continue;
    if (a - a0 < 32) selBits |= 1u << (a - a0);
    if (bestIdx == 0xFFFFFFFFu) bestIdx = a - a0;  // entries in key order
    if (at.adv_name[a] == S) {
      self = true;
      if (selfIdx == 0xFFFFFFFFu) selfIdx = a - a0;
    }
  }
  if (brs && self) bestIdx = selfIdx;  // selectBestNodeArea
  meta |= OGS_ROUTE_SELECTED | (bestIdx << OGS_ROUTE_BEST_SHIFT);
  if (flagsOf(a0 + bestIdx) & (OGS_NODE_OVERLOADED | OGS_NODE_METRICINC)) {
    meta |= OGS_ROUTE_DRAINED;
  }
  if (self) {
    clearMasks();
    finish(meta | (OGS_REASON_SELF << OGS_ROUTE_REASON_SHIFT), kInf);
    return;
  }

  // per area: shortest over all selected names in that area's SPF, next-hop
  // union over the closest ones; keep the areas with the smallest metric
  // (any number of areas: an area counts iff it holds a selected entry,
  // hasBestRoutesInArea, and is re-derived per pass instead of a bitmask)
  auto holds = [&](uint32_t b) {
    for (uint32_t a = a0; a < a1; ++a) {
      if (at.adv_area[a] == b && selected(a)) return true;
    }
    return false;
  };
  auto areaShortest = [&](uint32_t b) {
    D sb = kInf;
    for (uint32_t a = a0; a < a1; ++a) {
      if (!selected(a) || !reachOf(b, at.adv_name[a])) continue;
      const D d = distOf(b, at.adv_name[a]);
      if (d < sb) sb = d;
    }
    return sb;
  };
  D shortest = kInf;
  uint32_t cnt = 0;
  for (uint32_t b = 0; b < A; ++b) {
    if (!holds(b)) continue;
    const D sb = areaShortest(b);
    if (sb < shortest) shortest = sb;
  }
  for (uint32_t b = 0; b < A; ++b) {
    const bool use = holds(b) && areaShortest(b) == shortest;
    if constexpr (W > 0) {
      uint32_t m[W > 0 ? W : 1];
#pragma unroll
      for (int w = 0; w < W; ++w) m[w] = 0u;
      if (use) {
        for (uint32_t a = a0; a < a1; ++a) {
          if (!selected(a)) continue;
          const uint32_t name = at.adv_name[a];
          if (!reachOf(b, name) || distOf(b, name) != shortest) continue;
#pragma unroll
          for (int w = 0; w < W; ++w) m[w] |= nhOf(b, name, w);
        }
      }
#pragma unroll
      for (int w = 0; w < W; ++w) {
        cnt += __popc(m[w]);
        if (out.mask) out.mask[((size_t(u) * A + b) * W + w) * Sp + p] = m[w];
      }
    } else {  // one word at a time
      for (int w = 0; w < WW; ++w) {
        uint32_t m = 0u;
        if (use) {
          for (uint32_t a = a0; a < a1; ++a) {
            if (!selected(a)) continue;
            const uint32_t name = at.adv_name[a];
            if (!reachOf(b, name) || distOf(b, name) != shortest) continue;
            m |= nhOf(b, name, w);
          }
        }
        cnt += __popc(m);
        if (out.mask) out.mask[((size_t(u) * A + b) * WW + w) * Sp + p] = m;
      }
    }
  }
  // minimum next-hop threshold over the selected entries (496-509, 612)
  bool anyMinNh = false;
  int64_t minNh = INT64_MIN;
  if (pflags & OGS_PFX_HAS_MIN_NH) {
    for (uint32_t a = a0; a < a1; ++a) {
      if (!selected(a)) continue;
      const int64_t t = pt.adv_min_nh[a];
      if (t != INT64_MIN && (!anyMinNh || t > minNh)) {
        anyMinNh = true;
        minNh = t;
      }
    }
  }
  if (cnt == 0) {
    meta |= OGS_REASON_NO_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
  } else if (anyMinNh && static_cast<uint64_t>(minNh) > cnt) {
    meta |= OGS_REASON_MIN_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
  } else {
    meta |= OGS_ROUTE_VALID;
  }
  finish(meta, shortest);
}

template <int W>
hipError_t launch_ma(const ogs_graph& g, const ogs_prefix_table& pt,
                     const ogs_area_table& at, const uint32_t* units, int n,
                     const uint32_t* spfRow, const void* dist,
                     const uint32_t* nh, uint32_t flags, const ogs_spf_out& out,
                     hipStream_t stream, int Wr = 0) {
  const unsigned bx = unsigned((pt.max_prefixes + kBlock - 1) / kBlock);
  if (flags & OGS_F_WIDE_METRIC) {
    hipLaunchKernelGGL((route_multiarea_kernel<uint64_t, W>), dim3(bx, unsigned(n)),
                       dim3(kBlock), 0, stream, g, pt, at, units, spfRow,
                       static_cast<const uint64_t*>(dist), nh, flags, out, Wr);
  } else {
    hipLaunchKernelGGL((route_multiarea_kernel<uint32_t, W>), dim3(bx, unsigned(n)),
                       dim3(kBlock), 0, stream, g, pt, at, units, spfRow,
                       static_cast<const uint32_t*>(dist), nh, flags, out, Wr);
  }
  return hipGetLastError();
}

hipError_t launch_routes_multiarea(const ogs_graph& g, const ogs_prefix_table& pt,
                                   const ogs_area_table& at,
                                   const uint32_t* units, int n,
                                   const uint32_t* spfRow, const void* dist,
                                   const uint32_t* nh, uint32_t flags, int W,
                                   const ogs_spf_out& out, hipStream_t stream) {
  if (pt.max_prefixes <= 0) return hipSuccess;
  switch (W) {
    case 1: return launch_ma<1>(g, pt, at, units, n, spfRow, dist, nh, flags, out, stream);
    case 2: return launch_ma<2>(g, pt, at, units, n, spfRow, dist, nh, flags, out, stream);
    case 4: return launch_ma<4>(g, pt, at, units, n, spfRow, dist, nh, flags, out, stream);
    case 8: return launch_ma<8>(g, pt, at, units, n, spfRow, dist, nh, flags, out, stream);
    case 16: return launch_ma<16>(g, pt, at, units, n, spfRow, dist, nh, flags, out, stream);
    default: return launch_ma<0>(g, pt, at, units, n, spfRow, dist, nh, flags, out, stream, W);
  }
}

}  // namespace ogs
