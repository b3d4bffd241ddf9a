// route_core.h — per-prefix route selection + next-hop union (device code).
//
// Replaces SpfSolver::createRouteForPrefix (SpfSolver.cpp:160-311),
// selectBestRoutes / filterHardDrainedNodes / getSoftDrainedNodes /
// isNodeDrained (455-551), getNextHopsWithMetric (648-688), the link filter
// of getNextHopsThrift (690-767, folded into the link-slot bitsets),
// addBestPaths + getMinNextHopThreshold (496-509, 595-639) and LsdbUtil's
// selectRoutes / selectBestNodeArea (LsdbUtil.cpp:700-823), single area.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "spf_core.h"

namespace ogs {

struct RouteCfg {
  bool enableV4, v4OverV6, bestRouteSel;
};

// SPF state views: split arrays (dist[N], nh[N*W]) or one packed 64-bit
// word per node (dist | nh << 32, 32-bit distances, W == 1).
template <typename D, int W>
struct SplitView {
  const D* d;
  const uint32_t* n;
  __device__ __forceinline__ D dist(uint32_t v) const { return d[v]; }
  __device__ __forceinline__ uint32_t nh(uint32_t v, int w) const {
    return n[v * W + w];
  }
};
struct PackedView {
  const uint64_t* dn;
  __device__ __forceinline__ uint32_t dist(uint32_t v) const {
    return static_cast<uint32_t>(dn[v]);
  }
  __device__ __forceinline__ uint32_t nh(uint32_t v, int) const {
    return static_cast<uint32_t>(dn[v] >> 32);
  }
};

// Is node v reached in the unit's SPF? Views over exact-order state carry
// the settled bitset (a wrapped u64 distance may be all ones, LinkState.cpp:
// 789 -- the reference keeps such a node with metric UINT64_MAX); every
// other view uses the all-ones sentinel.
template <typename D, typename View>
__device__ __forceinline__ auto view_reached(const View& sv, uint32_t v, int)
    -> decltype(sv.reached(v)) {
  return sv.reached(v);
}
template <typename D, typename View>
__device__ __forceinline__ bool view_reached(const View& sv, uint32_t v, long) {
  return sv.dist(v) != DistInf<D>::value;
}

// Route for one prefix from the unit's SPF state.
template <typename D, int W, typename View>
__device__ void route_one(const ogs_prefix_table& pt, uint32_t gp, uint32_t s,
                          const uint8_t* __restrict__ nflags, const View& sv,
                          const RouteCfg& cfg, uint32_t& meta, D& metric,
                          uint32_t (&mask)[W], uint32_t& selBits) {
  constexpr D kInf = DistInf<D>::value;
  meta = 0;
  metric = kInf;
  selBits = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) mask[w] = 0;

  // v4 gate (SpfSolver.cpp:169-176)
  const uint8_t pflags = pt.pfx_flags[gp];
  const bool isV4 = pflags & OGS_PFX_V4;
  const bool hasMinNh = pflags & OGS_PFX_HAS_MIN_NH;
  if (isV4 && !cfg.enableV4 && !cfg.v4OverV6) {
    meta = OGS_REASON_V4_DISABLED << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  const uint32_t a0 = pt.adv_off[gp], a1 = pt.adv_off[gp + 1];

  // pass 1: reachability in the advertiser's area (single area => this
  // SPF), localPrefixConsidered, hard-drain census (SpfSolver.cpp:194-214,
  // 526-541)
  bool local = false;
  uint32_t nReach = 0, nReachUp = 0;
  for (uint32_t a = a0; a < a1; ++a) {
    const uint32_t n = pt.adv_node[a];
    if (n == s) local = true;
    if (n != OGS_NODE_NONE && view_reached<D>(sv, n, 0)) {
      ++nReach;
      nReachUp += (nflags[n] & OGS_NODE_OVERLOADED) ? 0u : 1u;
    }
  }
  if (local) meta |= OGS_ROUTE_LOCAL;
  if (nReach == 0) {
    meta |= OGS_REASON_UNREACHABLE << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  const bool dropOverloaded = nReachUp != 0;
  auto filtered = [&](uint32_t n) {
    return n != OGS_NODE_NONE && view_reached<D>(sv, n, 0) &&
        !(dropOverloaded && (nflags[n] & OGS_NODE_OVERLOADED));
  };

  // best-route selection (LsdbUtil.cpp:760-823, SHORTEST_DISTANCE):
  // max (-(drained), path_pref, source_pref), then min distance
  int32_t bD = INT32_MIN, bP = INT32_MIN, bS = INT32_MIN, bDist = INT32_MAX;
  if (cfg.bestRouteSel) {
    for (uint32_t a = a0; a < a1; ++a) {
      const uint32_t n = pt.adv_node[a];
      if (!filtered(n)) continue;
      const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
      const int32_t d =
          -((m.x != 0 || (nflags[n] & OGS_NODE_SOFTDRAIN)) ? 1 : 0);
      if (d > bD || (d == bD && (m.y > bP || (m.y == bP && m.z > bS)))) {
        bD = d;
        bP = m.y;
        bS = m.z;
      }
    }
    for (uint32_t a = a0; a < a1; ++a) {
      const uint32_t n = pt.adv_node[a];
      if (!filtered(n)) continue;
      const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
      const int32_t d =
          -((m.x != 0 || (nflags[n] & OGS_NODE_SOFTDRAIN)) ? 1 : 0);
      if (d == bD && m.y == bP && m.z == bS && m.w < bDist) bDist = m.w;
    }
  }
  auto selected = [&](uint32_t a, uint32_t n) {
    if (!filtered(n)) return false;
    if (!cfg.bestRouteSel) return true;
    const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
    const int32_t d = -((m.x != 0 || (nflags[n] & OGS_NODE_SOFTDRAIN)) ? 1 : 0);
    return d == bD && m.y == bP && m.z == bS && m.w == bDist;
  };

  // selected set: self?, best = smallest (node, area) key (node ids are name
  // ranks), shortest distance over all selected names (SpfSolver.cpp:664-677)
  bool self = false;
  uint32_t bestIdx = 0, bestNode = 0xFFFFFFFFu, selfIdx = 0;
  D shortest = kInf;
  for (uint32_t a = a0; a < a1; ++a) {
    const uint32_t n = pt.adv_node[a];
    if (!selected(a, n)) continue;
    if (a - a0 < 32) selBits |= 1u << (a - a0);
    if (n == s && !self) {
      self = true;
      selfIdx = a - a0;
    }
    if (n < bestNode) {
      bestNode = n;
      bestIdx = a - a0;
    }
    const D dn = sv.dist(n);
    if (dn < shortest) shortest = dn;
  }
  if (cfg.bestRouteSel && self) {  // selectBestNodeArea (LsdbUtil.cpp:700-711)
    bestNode = s;
    bestIdx = selfIdx;
  }
  meta |= OGS_ROUTE_SELECTED | (bestIdx << OGS_ROUTE_BEST_SHIFT);
  if (nflags[bestNode] & (OGS_NODE_OVERLOADED | OGS_NODE_METRICINC)) {
    meta |= OGS_ROUTE_DRAINED;  // isNodeDrained (SpfSolver.cpp:543-551)
  }
  if (self) {
    meta |= OGS_REASON_SELF << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  // next-hop union over the min-cost destinations + min-nexthop threshold
  bool anyMinNh = false;
  int64_t minNh = INT64_MIN;
  for (uint32_t a = a0; a < a1; ++a) {
    const uint32_t n = pt.adv_node[a];
    if (!selected(a, n)) continue;
    const int64_t t = hasMinNh ? pt.adv_min_nh[a] : INT64_MIN;
    if (t != INT64_MIN && (!anyMinNh || t > minNh)) {
      anyMinNh = true;
      minNh = t;
    }
    if (sv.dist(n) != shortest) continue;
#pragma unroll
    for (int w = 0; w < W; ++w) mask[w] |= sv.nh(n, w);
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) cnt += __popc(mask[w]);
  metric = shortest;
  if (cnt == 0) {
    meta |= OGS_REASON_NO_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  if (anyMinNh && static_cast<uint64_t>(minNh) > cnt) {  // SpfSolver.cpp:612
    meta |= OGS_REASON_MIN_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  meta |= OGS_ROUTE_VALID;
}

}  // namespace ogs
