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

// Store flavour of route / SPF output writes (launch flag bit kFlagNtStores,
// set per kernel family from the "route_store_nt" option bits):
// non-temporal stores, or ordinary write-back ones.
constexpr uint32_t kFlagNtStores = 1u << 28;

template <typename T>
__device__ __forceinline__ void store_out(T* p, T v, bool nt) {
  if (nt) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

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

// Selection state of one prefix (everything route_one decides before the
// next-hop union): SpfSolver.cpp:160-311 up to getNextHopsWithMetric.
template <typename D>
struct RouteSel {
  uint32_t a0, a1;
  bool dropOverloaded;
  int32_t bD, bP, bS, bDist;
  D shortest;
};

// drained key of an advertisement (SpfSolver.cpp:518-519, LsdbUtil.cpp:760)
__device__ __forceinline__ int32_t drain_key(const int4& m, uint8_t nf) {
  return -((m.x != 0 || (nf & OGS_NODE_SOFTDRAIN)) ? 1 : 0);
}

template <typename D, typename View>
__device__ __forceinline__ bool route_filtered(const RouteSel<D>& rs, const uint8_t* nflags,
                                               const View& sv, uint32_t n) {
  return n != OGS_NODE_NONE && view_reached<D>(sv, n, 0) &&
      !(rs.dropOverloaded && (nflags[n] & OGS_NODE_OVERLOADED));
}

template <typename D, typename View>
__device__ __forceinline__ bool route_selected(const RouteSel<D>& rs, const ogs_prefix_table& pt,
                                               const uint8_t* nflags, const View& sv,
                                               const RouteCfg& cfg, uint32_t a, uint32_t n) {
  if (!route_filtered(rs, nflags, sv, n)) return false;
  if (!cfg.bestRouteSel) return true;
  const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
  return drain_key(m, nflags[n]) == rs.bD && m.y == rs.bP && m.z == rs.bS && m.w == rs.bDist;
}

// Everything up to the next-hop union: v4 gate, reachability, hard-drain
// filter, best-route selection, best entry, self check, shortest metric.
// Returns false when the route is decided already (meta holds the reason).
template <typename D, typename View>
__device__ bool route_select(const ogs_prefix_table& pt, uint32_t gp, uint32_t s,
                             const uint8_t* __restrict__ nflags, const View& sv,
                             const RouteCfg& cfg, uint32_t& meta, uint32_t& selBits,
                             RouteSel<D>& rs) {
  constexpr D kInf = DistInf<D>::value;
  meta = 0;
  selBits = 0;
  rs.shortest = kInf;
  // v4 gate (SpfSolver.cpp:169-176)
  const uint8_t pflags = pt.pfx_flags[gp];
  const bool isV4 = pflags & OGS_PFX_V4;
  if (isV4 && !cfg.enableV4 && !cfg.v4OverV6) {
    meta = OGS_REASON_V4_DISABLED << OGS_ROUTE_REASON_SHIFT;
    return false;
  }
  rs.a0 = pt.adv_off[gp];
  rs.a1 = pt.adv_off[gp + 1];
  const uint32_t a0 = rs.a0, a1 = rs.a1;

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
    return false;
  }
  rs.dropOverloaded = nReachUp != 0;

  // best-route selection (LsdbUtil.cpp:760-823, SHORTEST_DISTANCE):
  // max (-(drained), path_pref, source_pref), then min distance
  rs.bD = INT32_MIN;
  rs.bP = INT32_MIN;
  rs.bS = INT32_MIN;
  rs.bDist = INT32_MAX;
  if (cfg.bestRouteSel) {
    for (uint32_t a = a0; a < a1; ++a) {
      const uint32_t n = pt.adv_node[a];
      if (!route_filtered(rs, nflags, sv, n)) continue;
      const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
      const int32_t d = drain_key(m, nflags[n]);
      if (d > rs.bD || (d == rs.bD && (m.y > rs.bP || (m.y == rs.bP && m.z > rs.bS)))) {
        rs.bD = d;
        rs.bP = m.y;
        rs.bS = m.z;
      }
    }
    for (uint32_t a = a0; a < a1; ++a) {
      const uint32_t n = pt.adv_node[a];
      if (!route_filtered(rs, nflags, sv, n)) continue;
      const int4 m = reinterpret_cast<const int4*>(pt.adv_metrics)[a];
      if (drain_key(m, nflags[n]) == rs.bD && m.y == rs.bP && m.z == rs.bS && m.w < rs.bDist) {
        rs.bDist = m.w;
      }
    }
  }

  // selected set: self?, best = smallest (node, area) key (node ids are name
  // ranks), shortest distance over all selected names (SpfSolver.cpp:664-677)
  bool self = false;
  uint32_t bestIdx = 0, bestNode = 0xFFFFFFFFu, selfIdx = 0;
  D shortest = kInf;
  for (uint32_t a = a0; a < a1; ++a) {
    const uint32_t n = pt.adv_node[a];
    if (!route_selected(rs, pt, nflags, sv, cfg, a, n)) continue;
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
  rs.shortest = shortest;
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
    return false;
  }
  return true;
}

// After the union: no next hop, or fewer than the largest minNexthop of the
// selected entries (addBestPaths, SpfSolver.cpp:605-619)
template <typename D, typename View>
__device__ void route_finish(const RouteSel<D>& rs, const ogs_prefix_table& pt, uint32_t gp,
                             const uint8_t* __restrict__ nflags, const View& sv,
                             const RouteCfg& cfg, uint32_t cnt, uint32_t& meta) {
  bool anyMinNh = false;
  int64_t minNh = INT64_MIN;
  if (pt.pfx_flags[gp] & OGS_PFX_HAS_MIN_NH) {
    for (uint32_t a = rs.a0; a < rs.a1; ++a) {
      if (!route_selected(rs, pt, nflags, sv, cfg, a, pt.adv_node[a])) continue;
      const int64_t t = pt.adv_min_nh[a];
      if (t != INT64_MIN && (!anyMinNh || t > minNh)) {
        anyMinNh = true;
        minNh = t;
      }
    }
  }
  if (cnt == 0) {
    meta |= OGS_REASON_NO_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
  } else if (anyMinNh && static_cast<uint64_t>(minNh) > cnt) {  // SpfSolver.cpp:612
    meta |= OGS_REASON_MIN_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
  } else {
    meta |= OGS_ROUTE_VALID;
  }
}

// Route for one prefix from the unit's SPF state.
template <typename D, int W, typename View>
__device__ void route_one(const ogs_prefix_table& pt, uint32_t gp, uint32_t s,
                          const uint8_t* __restrict__ nflags, const View& sv,
                          const RouteCfg& cfg, uint32_t& meta, D& metric,
                          uint32_t (&mask)[W], uint32_t& selBits) {
#pragma unroll
  for (int w = 0; w < W; ++w) mask[w] = 0;
  RouteSel<D> rs;
  const bool go = route_select<D>(pt, gp, s, nflags, sv, cfg, meta, selBits, rs);
  metric = DistInf<D>::value;
  if (!go) return;
  // next-hop union over the min-cost destinations (getNextHopsWithMetric)
  for (uint32_t a = rs.a0; a < rs.a1; ++a) {
    const uint32_t n = pt.adv_node[a];
    if (!route_selected(rs, pt, nflags, sv, cfg, a, n) || sv.dist(n) != rs.shortest) continue;
#pragma unroll
    for (int w = 0; w < W; ++w) mask[w] |= sv.nh(n, w);
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) cnt += __popc(mask[w]);
  metric = rs.shortest;
  route_finish<D>(rs, pt, gp, nflags, sv, cfg, cnt, meta);
}

// route_one for next-hop sets of any width (sources of more than 512
// links): the union is formed one word at a time and stored straight to
// mask[w * maskStride].
template <typename D, typename View>
__device__ void route_one_wide(const ogs_prefix_table& pt, uint32_t gp, uint32_t s,
                               const uint8_t* __restrict__ nflags, const View& sv,
                               const RouteCfg& cfg, int W, uint32_t& meta, D& metric,
                               uint32_t* mask, size_t maskStride, uint32_t& selBits) {
  RouteSel<D> rs;
  const bool go = route_select<D>(pt, gp, s, nflags, sv, cfg, meta, selBits, rs);
  metric = DistInf<D>::value;
  uint32_t cnt = 0;
  for (int w = 0; w < W; ++w) {
    uint32_t m = 0u;
    if (go) {
      for (uint32_t a = rs.a0; a < rs.a1; ++a) {
        const uint32_t n = pt.adv_node[a];
        if (!route_selected(rs, pt, nflags, sv, cfg, a, n) || sv.dist(n) != rs.shortest) continue;
        m |= sv.nh(n, w);
      }
    }
    cnt += __popc(m);
    if (mask) mask[size_t(w) * maskStride] = m;
  }
  if (!go) return;
  metric = rs.shortest;
  route_finish<D>(rs, pt, gp, nflags, sv, cfg, cnt, meta);
}

}  // namespace ogs
