// spf_core.h — unit-scope SPF fixpoint shared by the RouteDb and KSP2
// kernels (device code only; included by the .hip translation units).
//
// Reference semantics: LinkState::runSpf (LinkState.cpp:720-820). For link
// metrics >= 1 the reference's Dijkstra result is the unique fixpoint of
//   dist(v) = min over usable predecessors u of dist(u) + w(u, v)
//   NH(v)   = U over tight predecessors u of (u == src ? slot(src->v) : NH(u))
// with u usable iff the link is up (LinkState.cpp:762), not in
// linksToIgnore (763) and u relaxes (u == src or u not hard-drained,
// 741-752). Distances only decrease across rounds, so the loop ends at the
// first round in which no node of the unit changes.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"

namespace ogs {

constexpr int kBlock = 256;

template <typename D>
struct DistInf {
  static constexpr D value = ~D(0);
};

template <int UT>
struct UnitScope;

template <>
struct UnitScope<64> {  // one wavefront per unit: lockstep, no s_barrier
  static __device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  static __device__ __forceinline__ bool any(bool x) {
    sync();
    return __ballot(x) != 0ull;
  }
};

template <>
struct UnitScope<kBlock> {  // one workgroup per unit
  static __device__ __forceinline__ void sync() { __syncthreads(); }
  static __device__ __forceinline__ bool any(bool x) {
    return __syncthreads_or(x) != 0;
  }
};

__device__ __forceinline__ uint32_t edge_dst(uint32_t lo) {
  return lo & OGS_EDGE_DST_MASK;
}
__device__ __forceinline__ uint32_t edge_rslot(uint32_t lo) {
  return (lo >> OGS_EDGE_RSLOT_SHIFT) & OGS_EDGE_RSLOT_MASK;
}

// Per-unit view of one topology's CSR: row offsets index `edg` directly;
// `eBase` converts them to topology-local edge ids (0 when staged in LDS).
struct UnitCsr {
  const uint32_t* rowp;
  const uint64_t* edg;
  uint32_t eBase;
  // exact reverse slots by topology-local edge id where the 9-bit field
  // saturates (rows of 511+ edges, ogs_graph.rslot_ext), or nullptr
  const uint32_t* rext;
};

// Index of edge e's reverse inside its neighbour's row (any row length).
__device__ __forceinline__ uint32_t csr_rslot(const UnitCsr& c, uint32_t e, uint32_t lo) {
  const uint32_t r = edge_rslot(lo);
  return (r == OGS_EDGE_RSLOT_MASK && c.rext) ? c.rext[e - c.eBase] : r;
}

// Topology-local id of the link behind directed edge e (v -> u): the smaller
// of the two directed edge ids. Used to test linksToIgnore masks.
__device__ __forceinline__ uint32_t link_id(const UnitCsr& c, uint32_t e,
                                            uint32_t lo) {
  const uint32_t rev = c.rowp[edge_dst(lo)] + csr_rslot(c, e, lo);
  return (e < rev ? e : rev) - c.eBase;
}

template <typename D, int W, int UT, bool WITH_NH, bool MASKED>
__device__ void spf_fixpoint(uint32_t N, uint32_t s, int lane,
                             const UnitCsr& c, bool hop, D* dist, uint32_t* nh,
                             const uint32_t* __restrict__ ignore) {
  using Scope = UnitScope<UT>;
  constexpr D kInf = DistInf<D>::value;
  for (uint32_t v = lane; v < N; v += UT) {
    dist[v] = (v == s) ? D(0) : kInf;
    if constexpr (WITH_NH) {
#pragma unroll
      for (int w = 0; w < W; ++w) nh[v * W + w] = 0u;
    }
  }
  Scope::sync();
  for (;;) {
    bool changed = false;
    for (uint32_t v = lane; v < N; v += UT) {
      if (v == s) continue;
      D best = kInf;
      uint32_t m[W];
#pragma unroll
      for (int w = 0; w < W; ++w) m[w] = 0u;
      const uint32_t eb = c.rowp[v], ee = c.rowp[v + 1];
      for (uint32_t e = eb; e < ee; ++e) {
        const uint64_t ed = c.edg[e];
        const uint32_t lo = static_cast<uint32_t>(ed);
        if (lo & OGS_EDGE_DOWN) continue;
        const uint32_t u = edge_dst(lo);
        const bool fromSrc = (u == s);
        if ((lo & OGS_EDGE_DST_OVERLOADED) && !fromSrc) continue;
        if constexpr (MASKED) {
          const uint32_t l = link_id(c, e, lo);
          if ((ignore[l >> 5] >> (l & 31u)) & 1u) continue;
        }
        const D du = dist[u];
        if (du == kInf) continue;
        const D cand = du + (hop ? D(1) : static_cast<D>(ed >> 32));
        if (cand > best) continue;
        if constexpr (WITH_NH) {
          uint32_t cw[W];
          if (fromSrc) {
            const uint32_t slot = edge_rslot(lo);
#pragma unroll
            for (int w = 0; w < W; ++w) {
              cw[w] = (int(slot >> 5) == w) ? (1u << (slot & 31u)) : 0u;
            }
          } else {
#pragma unroll
            for (int w = 0; w < W; ++w) cw[w] = nh[u * W + w];
          }
          if (cand < best) {
#pragma unroll
            for (int w = 0; w < W; ++w) m[w] = cw[w];
          } else {
#pragma unroll
            for (int w = 0; w < W; ++w) m[w] |= cw[w];
          }
        }
        best = cand;
      }
      bool diff = best != dist[v];
      if constexpr (WITH_NH) {
#pragma unroll
        for (int w = 0; w < W; ++w) diff |= (m[w] != nh[v * W + w]);
      }
      if (diff) {
        dist[v] = best;
        if constexpr (WITH_NH) {
#pragma unroll
          for (int w = 0; w < W; ++w) nh[v * W + w] = m[w];
        }
        changed = true;
      }
    }
    if (!Scope::any(changed)) break;
  }
}

// LDS carve-out helper (16-byte aligned pieces).
__host__ __device__ inline uint32_t align16(uint64_t x) {
  return static_cast<uint32_t>((x + 15u) & ~uint64_t(15));
}

}  // namespace ogs
