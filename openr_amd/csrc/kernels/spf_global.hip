// spf_global.hip — SPF + RouteDb for topologies past the LDS budget (SURVEY
// §8 row g1 "global frontier": WAN areas of tens of thousands of nodes, the
// reference's 99x99 GridTopology.StressTest, SpfSolverTest.cpp:2858-2873).
//
// Same fixpoint as spf_core.h / spf_frontier.hip (reference: LinkState::runSpf,
// LinkState.cpp:720-820; distances are the least solution of dist(v) = min
// over usable u of dist(u) + w(u, v), next-hop sets the least solution of
// NH(v) = U over tight u of (u == src ? {slot} : NH(u)), u relaxing iff u is
// the source or not hard-drained, 741-752). What differs is where the unit's
// state lives: dist / next-hop sets / push stamps / the two frontier lists
// are in HBM (the caller's output rows or the workspace), so there is no
// size limit but the 21-bit node ids of the edge encoding. One workgroup of
// 1024 threads per unit walks the frontier list of the round; relaxations
// are L2 atomics (atomicMin / atomicOr). A unit's workgroup runs on ONE CU,
// so its state never leaves that XCD's L2 until the kernel ends: a round
// ends with every wave's stores drained (s_waitcnt vmcnt(0)) and a workgroup
// barrier, and every read of state written in this launch is an L2-served
// `sc1` load (L1 bypassed: MI355X_MICROARCH.md, inter-workgroup visibility
// table) -- no L2 write-back / L1 invalidate per round. (The first form
// used agent-scope release + acquire fences per round, ~3.5 us of cache
// maintenance each: option "spf_global_sync" 0 keeps it for A/B.) Every
// round touches only the rows of the nodes changed in the previous round.
//
// Routes: route_global.h, one thread per (unit, prefix) against the unit's
// state in HBM. u32 or u64 distances (OGS_F_WIDE_METRIC).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "route_core.h"
#include "route_global.h"
#include "spf_core.h"
#include "engine.h"

namespace ogs {

constexpr int kGBlock = 1024;
constexpr int kGRow = 4;  // row edges per step of a frontier node

// L2SYNC: stores drained + barrier (state read back through sc1 loads);
// else agent-scope release / acquire fences around the barrier.
template <bool L2SYNC>
__device__ __forceinline__ void round_sync() {
  if constexpr (L2SYNC) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

// Read of state written earlier in this launch: an sc1 (L2-served) load
// under L2SYNC, a plain load after the agent acquire otherwise.
template <bool L2SYNC, typename T>
__device__ __forceinline__ T ld_state(const T* p) {
  if constexpr (L2SYNC) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    return *p;
  }
}

template <typename D>
__device__ __forceinline__ D atomic_min_d(D* p, D v) {
  return atomicMin(p, v);
}

// One unit's SPF into HBM. dist[v] (D), nh[w * Sn + v], stamp/q0/q1 scratch
// rows of this unit (>= N entries each).
template <typename D, int W, bool L2SYNC>
__global__ __launch_bounds__(kGBlock) void spf_global_kernel(
    ogs_graph g, const ogs_unit* __restrict__ units, uint32_t flags,
    D* __restrict__ oDist, uint32_t* __restrict__ oNh, uint32_t* __restrict__ scratch) {
  constexpr D kInf = DistInf<D>::value;
  const int tid = threadIdx.x;
  const uint32_t u0 = blockIdx.x;
  const ogs_unit unit = units[u0];
  const uint32_t s = unit.src;
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const size_t Sn = size_t(g.max_nodes);
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint64_t* __restrict__ edges = g.edges + e0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0;
  D* dist = oDist + u0 * Sn;
  uint32_t* nh = oNh + u0 * W * Sn;
  uint32_t* stamp = scratch + u0 * 3 * Sn;
  uint32_t* q0 = stamp + Sn;
  uint32_t* q1 = q0 + Sn;
  __shared__ uint32_t qcnt[3];

  for (uint32_t v = tid; v < N; v += kGBlock) {
    dist[v] = (v == s) ? D(0) : kInf;
    stamp[v] = 0u;
#pragma unroll
    for (int w = 0; w < W; ++w) nh[w * Sn + v] = 0u;
  }
  if (tid == 0) {
    q1[0] = s;  // round 1's list: buffer r & 1, count slot r % 3
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  round_sync<L2SYNC>();
  // t's first push of round r + 1 (stamp claimed): append to that list
  auto push = [&](uint32_t t, uint32_t r) {
    const uint32_t at = atomicAdd(&qcnt[(r + 1) % 3], 1u);
    ((r + 1) & 1 ? q1 : q0)[at] = t;
  };
  auto append = [&](uint32_t t, uint32_t r) {
    if (atomicMax(&stamp[t], r + 1) < r + 1) push(t, r);
  };
  auto weight = [&](uint64_t x) -> D {
    return hop ? D(1) : D(static_cast<uint32_t>(x >> 32));
  };

  // ---- dist phase: rows of the nodes whose distance dropped last round ----
  uint32_t r = 1, n = 1;
  for (; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = ld_state<L2SYNC>(cur + i);
      if (v != s && (nflags[v] & OGS_NODE_OVERLOADED)) continue;  // 741-752
      const D dv = ld_state<L2SYNC>(dist + v);
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      // kGRow edges at a time, each step's memory operations independent
      // (edge words, then the targets' dist, then the atomicMins, then the
      // stamps): one L2 round trip per step instead of one per edge and step
      for (uint32_t j0 = 0; j0 < m; j0 += kGRow) {
        uint32_t t[kGRow];
        D c[kGRow], seen[kGRow];
        bool ok[kGRow];
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          const uint64_t x = j0 + k < m ? edges[b + j0 + k] : uint64_t(OGS_EDGE_DOWN);
          const uint32_t lo = static_cast<uint32_t>(x);
          ok[k] = !(lo & OGS_EDGE_DOWN);
          t[k] = edge_dst(lo);
          c[k] = dv + weight(x);
        }
#pragma unroll
        for (int k = 0; k < kGRow; ++k) seen[k] = ok[k] ? ld_state<L2SYNC>(dist + t[k]) : D(0);
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          ok[k] = ok[k] && c[k] < seen[k];
          seen[k] = ok[k] ? atomic_min_d(&dist[t[k]], c[k]) : D(0);
        }
        uint32_t st[kGRow];
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          ok[k] = ok[k] && c[k] < seen[k];
          st[k] = ok[k] ? atomicMax(&stamp[t[k]], r + 1) : r + 1;
        }
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          if (ok[k] && st[k] < r + 1) push(t[k], r);
        }
      }
    }
    round_sync<L2SYNC>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();  // every thread has read the count before it is reset
  }

  // ---- next-hop phase: the source's row seeds link slots, tight pushes ----
  const uint32_t r0 = r;
  if (tid == 0) qcnt[0] = qcnt[1] = qcnt[2] = 0u;
  round_sync<L2SYNC>();
  {
    const uint32_t b = gRow[s] - e0, m = gRow[s + 1] - e0 - b;
    for (uint32_t j = tid; j < m && j < 32u * W; j += kGBlock) {
      const uint64_t x = edges[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      if (lo & OGS_EDGE_DOWN) continue;
      const uint32_t t = edge_dst(lo);
      if (weight(x) == ld_state<L2SYNC>(dist + t)) {
        atomicOr(&nh[(j >> 5) * Sn + t], 1u << (j & 31u));
        append(t, r0);
      }
    }
  }
  round_sync<L2SYNC>();
  n = qcnt[(r0 + 1) % 3];
  __syncthreads();
  for (r = r0 + 1; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = ld_state<L2SYNC>(cur + i);
      if (v == s || (nflags[v] & OGS_NODE_OVERLOADED)) continue;
      const D dv = ld_state<L2SYNC>(dist + v);
      uint32_t nv[W];
#pragma unroll
      for (int w = 0; w < W; ++w) nv[w] = ld_state<L2SYNC>(nh + w * Sn + v);
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      constexpr int kB = W <= 4 ? kGRow : 2;  // edges per step (as above)
      for (uint32_t j0 = 0; j0 < m; j0 += kB) {
        uint32_t t[kB];
        bool ok[kB];
        D c[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          const uint64_t x = j0 + k < m ? edges[b + j0 + k] : uint64_t(OGS_EDGE_DOWN);
          const uint32_t lo = static_cast<uint32_t>(x);
          ok[k] = !(lo & OGS_EDGE_DOWN);
          t[k] = edge_dst(lo);
          c[k] = dv + weight(x);
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          ok[k] = ok[k] && c[k] == ld_state<L2SYNC>(dist + t[k]);  // tight
        }
        uint32_t a[kB][W];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
#pragma unroll
          for (int w = 0; w < W; ++w) {
            a[k][w] = ok[k] ? nv[w] & ~ld_state<L2SYNC>(nh + w * Sn + t[k]) : 0u;
          }
        }
        bool add[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          add[k] = false;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            if (a[k][w] && (a[k][w] & ~atomicOr(&nh[w * Sn + t[k]], a[k][w]))) add[k] = true;
          }
        }
        uint32_t st[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) st[k] = add[k] ? atomicMax(&stamp[t[k]], r + 1) : r + 1;
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          if (add[k] && st[k] < r + 1) push(t[k], r);
        }
      }
    }
    round_sync<L2SYNC>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();
  }
}

// ---- next-hop sets of any width (sources of more than 512 links): the
// all-HBM form with a runtime word count; rslot is never read (push-style
// relaxation, link slots from the source's own row) ---------------------
template <typename D>
__global__ __launch_bounds__(kGBlock) void spf_global_wide_kernel(
    ogs_graph g, const ogs_unit* __restrict__ units, uint32_t flags, int W,
    D* __restrict__ oDist, uint32_t* __restrict__ oNh, uint32_t* __restrict__ scratch) {
  constexpr D kInf = DistInf<D>::value;
  const int tid = threadIdx.x;
  const uint32_t u0 = blockIdx.x;
  const ogs_unit unit = units[u0];
  const uint32_t s = unit.src;
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const size_t Sn = size_t(g.max_nodes);
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint64_t* __restrict__ edges = g.edges + e0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0;
  D* dist = oDist + u0 * Sn;
  uint32_t* nh = oNh + u0 * size_t(W) * Sn;
  uint32_t* stamp = scratch + u0 * 3 * Sn;
  uint32_t* q0 = stamp + Sn;
  uint32_t* q1 = q0 + Sn;
  __shared__ uint32_t qcnt[3];

  for (uint32_t v = tid; v < N; v += kGBlock) {
    dist[v] = (v == s) ? D(0) : kInf;
    stamp[v] = 0u;
    for (int w = 0; w < W; ++w) nh[w * Sn + v] = 0u;
  }
  if (tid == 0) {
    q1[0] = s;
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  round_sync<true>();
  auto push = [&](uint32_t t, uint32_t r) {
    const uint32_t at = atomicAdd(&qcnt[(r + 1) % 3], 1u);
    ((r + 1) & 1 ? q1 : q0)[at] = t;
  };
  auto append = [&](uint32_t t, uint32_t r) {
    if (atomicMax(&stamp[t], r + 1) < r + 1) push(t, r);
  };
  auto weight = [&](uint64_t x) -> D {
    return hop ? D(1) : D(static_cast<uint32_t>(x >> 32));
  };
  // ---- dist phase ----------------------------------------------------------
  uint32_t r = 1, n = 1;
  for (; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = ld_state<true>(cur + i);
      if (v != s && (nflags[v] & OGS_NODE_OVERLOADED)) continue;  // 741-752
      const D dv = ld_state<true>(dist + v);
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      for (uint32_t j = 0; j < m; ++j) {
        const uint64_t x = edges[b + j];
        const uint32_t lo = static_cast<uint32_t>(x);
        if (lo & OGS_EDGE_DOWN) continue;
        const uint32_t t = edge_dst(lo);
        const D c = dv + weight(x);
        if (c < ld_state<true>(dist + t) && c < atomic_min_d(&dist[t], c)) append(t, r);
      }
    }
    round_sync<true>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();
  }
  // ---- next-hop phase ------------------------------------------------------
  const uint32_t r0 = r;
  if (tid == 0) qcnt[0] = qcnt[1] = qcnt[2] = 0u;
  round_sync<true>();
  {
    const uint32_t b = gRow[s] - e0, m = gRow[s + 1] - e0 - b;
    for (uint32_t j = tid; j < m && j < 32u * uint32_t(W); j += kGBlock) {
      const uint64_t x = edges[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      if (lo & OGS_EDGE_DOWN) continue;
      const uint32_t t = edge_dst(lo);
      if (weight(x) == ld_state<true>(dist + t)) {
        atomicOr(&nh[(j >> 5) * Sn + t], 1u << (j & 31u));
        append(t, r0);
      }
    }
  }
  round_sync<true>();
  n = qcnt[(r0 + 1) % 3];
  __syncthreads();
  for (r = r0 + 1; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = ld_state<true>(cur + i);
      if (v == s || (nflags[v] & OGS_NODE_OVERLOADED)) continue;
      const D dv = ld_state<true>(dist + v);
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      for (uint32_t j = 0; j < m; ++j) {
        const uint64_t x = edges[b + j];
        const uint32_t lo = static_cast<uint32_t>(x);
        if (lo & OGS_EDGE_DOWN) continue;
        const uint32_t t = edge_dst(lo);
        if (dv + weight(x) != ld_state<true>(dist + t)) continue;  // not tight
        bool add = false;
        for (int w = 0; w < W; ++w) {
          const uint32_t a = ld_state<true>(nh + w * Sn + v) & ~ld_state<true>(nh + w * Sn + t);
          if (a && (a & ~atomicOr(&nh[w * Sn + t], a))) add = true;
        }
        if (add) append(t, r);
      }
    }
    round_sync<true>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();
  }
}

// SPF (+ RouteDb) with next-hop sets wider than 16 words.
hipError_t workspace(size_t bytes, hipStream_t stream, void** out);

template <typename D>
hipError_t launch_global_wide(const ogs_graph& g, const ogs_prefix_table* pt,
                              const ogs_unit* units, int nUnits, uint32_t flags, int W,
                              const ogs_spf_out& out, hipStream_t stream) {
  const size_t Sn = size_t(g.max_nodes), U = size_t(nUnits);
  auto r256 = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t distBytes = out.dist ? 0 : r256(U * Sn * sizeof(D));
  const size_t nhBytes = out.nh ? 0 : r256(U * W * Sn * 4);
  const size_t scratchBytes = r256(U * 3 * Sn * 4);
  void* ws = nullptr;
  hipError_t e = workspace(distBytes + nhBytes + scratchBytes, stream, &ws);
  if (e != hipSuccess) return e;
  char* base = static_cast<char*>(ws);
  D* dist = out.dist ? static_cast<D*>(out.dist) : reinterpret_cast<D*>(base);
  uint32_t* nh = out.nh ? out.nh : reinterpret_cast<uint32_t*>(base + distBytes);
  uint32_t* scratch = reinterpret_cast<uint32_t*>(base + distBytes + nhBytes);
  hipLaunchKernelGGL((spf_global_wide_kernel<D>), dim3(nUnits), dim3(kGBlock), 0, stream, g,
                     units, flags, W, dist, nh, scratch);
  e = hipGetLastError();
  if (e != hipSuccess || !pt || pt->max_prefixes == 0) return e;
  return launch_route_global_wide<D>(g, *pt, units, nUnits, flags, W, dist, nh, out, stream);
}

hipError_t launch_spf_routes_global_wide(const ogs_graph& g, const ogs_prefix_table* pt,
                                         const ogs_unit* units, int nUnits, uint32_t flags,
                                         int W, const ogs_spf_out& out, hipStream_t stream) {
  if (flags & OGS_F_WIDE_METRIC) {
    return launch_global_wide<uint64_t>(g, pt, units, nUnits, flags, W, out, stream);
  }
  return launch_global_wide<uint32_t>(g, pt, units, nUnits, flags, W, out, stream);
}

// ---- dist in LDS (units whose distances fit: N * sizeof(D) + two list
// bitsets <= 160 kB, e.g. 20k nodes at u32) ----------------------------------
// The same rounds with the unit's distances in LDS: a dist round's chain is
// then frontier entry -> row -> edge words (L2) with LDS atomics for the
// relaxations, instead of dist loads and atomics whose lines the atomics
// drop from L2. List membership is a bitset per round parity in LDS (bit set
// on the first push of a round, cleared when the entry is consumed). The
// next-hop words stay in HBM; the final distances are copied to the caller's
// row for the route kernel.
uint32_t global_lds_bytes(uint32_t Sn, uint32_t dsize) {
  return ((Sn * dsize + 15u) & ~15u) + 2u * 4u * ((Sn + 31u) / 32u);
}

template <typename D, int W>
__global__ __launch_bounds__(kGBlock) void spf_global_lds_kernel(
    ogs_graph g, const ogs_unit* __restrict__ units, uint32_t flags,
    D* __restrict__ oDist, uint32_t* __restrict__ oNh, uint32_t* __restrict__ scratch) {
  constexpr D kInf = DistInf<D>::value;
  const int tid = threadIdx.x;
  const uint32_t u0 = blockIdx.x;
  const ogs_unit unit = units[u0];
  const uint32_t s = unit.src;
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const size_t Sn = size_t(g.max_nodes);
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint64_t* __restrict__ edges = g.edges + e0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0;
  uint32_t* nh = oNh + u0 * W * Sn;
  uint32_t* q0 = scratch + u0 * 3 * Sn + Sn;  // the HBM form's list rows
  uint32_t* q1 = q0 + Sn;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  D* dist = reinterpret_cast<D*>(smem);
  const uint32_t mw = (uint32_t(Sn) + 31u) / 32u;
  uint32_t* mark = reinterpret_cast<uint32_t*>(smem + ((Sn * sizeof(D) + 15u) & ~size_t(15)));
  __shared__ uint32_t qcnt[3];

  for (uint32_t v = tid; v < N; v += kGBlock) {
    dist[v] = (v == s) ? D(0) : kInf;
#pragma unroll
    for (int w = 0; w < W; ++w) nh[w * Sn + v] = 0u;
  }
  for (uint32_t i = tid; i < 2 * mw; i += kGBlock) mark[i] = 0u;
  if (tid == 0) {
    q1[0] = s;
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  round_sync<true>();
  auto weight = [&](uint64_t x) -> D {
    return hop ? D(1) : D(static_cast<uint32_t>(x >> 32));
  };
  // first push of t into round r + 1's list
  auto append = [&](uint32_t t, uint32_t r) {
    const uint32_t bit = 1u << (t & 31u);
    if (!(atomicOr(&mark[((r + 1) & 1) * mw + (t >> 5)], bit) & bit)) {
      const uint32_t at = atomicAdd(&qcnt[(r + 1) % 3], 1u);
      ((r + 1) & 1 ? q1 : q0)[at] = t;
    }
  };
  auto consume = [&](uint32_t v, uint32_t r) {  // v leaves round r's list
    atomicAnd(&mark[(r & 1) * mw + (v >> 5)], ~(1u << (v & 31u)));
  };

  // ---- dist phase ----------------------------------------------------------
  uint32_t r = 1, n = 1;
  for (; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = ld_state<true>(cur + i);
      if (r > 1) consume(v, r);
      if (v != s && (nflags[v] & OGS_NODE_OVERLOADED)) continue;  // 741-752
      const D dv = dist[v];
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      for (uint32_t j0 = 0; j0 < m; j0 += kGRow) {
        uint64_t x[kGRow];
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          x[k] = j0 + k < m ? edges[b + j0 + k] : uint64_t(OGS_EDGE_DOWN);
        }
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          const uint32_t lo = static_cast<uint32_t>(x[k]);
          if (lo & OGS_EDGE_DOWN) continue;
          const uint32_t t = edge_dst(lo);
          const D c = dv + weight(x[k]);
          if (c < dist[t] && c < atomicMin(&dist[t], c)) append(t, r);
        }
      }
    }
    round_sync<true>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();
  }
  // the last round consumed nothing: clear both parities for the next phase
  for (uint32_t i = tid; i < 2 * mw; i += kGBlock) mark[i] = 0u;
  D* oD = oDist + u0 * Sn;
  for (uint32_t v = tid; v < N; v += kGBlock) oD[v] = dist[v];

  // ---- next-hop phase (words in HBM, L2 atomics) ---------------------------
  const uint32_t r0 = r;
  if (tid == 0) qcnt[0] = qcnt[1] = qcnt[2] = 0u;
  round_sync<true>();
  {
    const uint32_t b = gRow[s] - e0, m = gRow[s + 1] - e0 - b;
    for (uint32_t j = tid; j < m && j < 32u * W; j += kGBlock) {
      const uint64_t x = edges[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      if (lo & OGS_EDGE_DOWN) continue;
      const uint32_t t = edge_dst(lo);
      if (weight(x) == dist[t]) {
        atomicOr(&nh[(j >> 5) * Sn + t], 1u << (j & 31u));
        append(t, r0);
      }
    }
  }
  round_sync<true>();
  n = qcnt[(r0 + 1) % 3];
  __syncthreads();
  for (r = r0 + 1; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = ld_state<true>(cur + i);
      consume(v, r);
      if (v == s || (nflags[v] & OGS_NODE_OVERLOADED)) continue;
      const D dv = dist[v];
      uint32_t nv[W];
#pragma unroll
      for (int w = 0; w < W; ++w) nv[w] = ld_state<true>(nh + w * Sn + v);
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      constexpr int kB = W <= 4 ? kGRow : 2;
      for (uint32_t j0 = 0; j0 < m; j0 += kB) {
        uint32_t t[kB];
        bool ok[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          const uint64_t x = j0 + k < m ? edges[b + j0 + k] : uint64_t(OGS_EDGE_DOWN);
          const uint32_t lo = static_cast<uint32_t>(x);
          t[k] = edge_dst(lo);
          ok[k] = !(lo & OGS_EDGE_DOWN) && dv + weight(x) == dist[t[k]];  // tight
        }
        uint32_t a[kB][W];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
#pragma unroll
          for (int w = 0; w < W; ++w) {
            a[k][w] = ok[k] ? nv[w] & ~ld_state<true>(nh + w * Sn + t[k]) : 0u;
          }
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          bool add = false;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            if (a[k][w] && (a[k][w] & ~atomicOr(&nh[w * Sn + t[k]], a[k][w]))) add = true;
          }
          if (add) append(t[k], r);
        }
      }
    }
    round_sync<true>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();
  }
}

// ---- dist AND next-hop words in LDS (N * (sizeof(D) + 4W) + one list bitset
// <= 160 kB, e.g. 20k nodes at u32, W = 1) ----------------------------------
// Both phases relax with LDS atomics; only the frontier lists (HBM rows) and
// the CSR are read from L2. List membership is ONE bitset ("already in the
// next list"), cleared in bulk at the start of every round -- behind the
// same barrier that the round's first frontier loads are already in flight
// across. The final distances and next-hop words are copied to the caller's
// rows for the route kernel.
uint32_t global_lds2_bytes(uint32_t Sn, uint32_t dsize, int W) {
  return ((Sn * dsize + 15u) & ~15u) + ((Sn * 4u * uint32_t(W) + 15u) & ~15u) +
      4u * ((Sn + 31u) / 32u);
}

template <typename D, int W>
__global__ __launch_bounds__(kGBlock) void spf_global_lds2_kernel(
    ogs_graph g, const ogs_unit* __restrict__ units, uint32_t flags,
    D* __restrict__ oDist, uint32_t* __restrict__ oNh, uint32_t* __restrict__ scratch) {
  constexpr D kInf = DistInf<D>::value;
  const int tid = threadIdx.x;
  const uint32_t u0 = blockIdx.x;
  const ogs_unit unit = units[u0];
  const uint32_t s = unit.src;
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const size_t Sn = size_t(g.max_nodes);
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint64_t* __restrict__ edges = g.edges + e0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0;
  uint32_t* q0 = scratch + u0 * 3 * Sn + Sn;
  uint32_t* q1 = q0 + Sn;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  D* dist = reinterpret_cast<D*>(smem);
  uint32_t* nh = reinterpret_cast<uint32_t*>(smem + ((Sn * sizeof(D) + 15u) & ~size_t(15)));
  uint32_t* mark = nh + ((Sn * W + 3u) & ~size_t(3));
  const uint32_t mw = (uint32_t(Sn) + 31u) / 32u;
  __shared__ uint32_t qcnt[3];

  for (uint32_t v = tid; v < N; v += kGBlock) {
    dist[v] = (v == s) ? D(0) : kInf;
#pragma unroll
    for (int w = 0; w < W; ++w) nh[w * Sn + v] = 0u;
  }
  if (tid == 0) {
    q1[0] = s;
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  round_sync<true>();
  auto weight = [&](uint64_t x) -> D {
    return hop ? D(1) : D(static_cast<uint32_t>(x >> 32));
  };
  auto append = [&](uint32_t t, uint32_t r) {  // first push of t this round
    const uint32_t bit = 1u << (t & 31u);
    if (!(atomicOr(&mark[t >> 5], bit) & bit)) {
      const uint32_t at = atomicAdd(&qcnt[(r + 1) % 3], 1u);
      ((r + 1) & 1 ? q1 : q0)[at] = t;
    }
  };
  // round r's first frontier entry per thread is loaded, then the bitset is
  // cleared behind one barrier (the load's latency overlaps it)
  auto begin_round = [&](const uint32_t* cur, uint32_t n) {
    const uint32_t v0 = uint32_t(tid) < n ? ld_state<true>(cur + tid) : 0u;
    for (uint32_t i = tid; i < mw; i += kGBlock) mark[i] = 0u;
    __syncthreads();
    return v0;
  };

  // ---- dist phase ----------------------------------------------------------
  uint32_t r = 1, n = 1;
  for (; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    const uint32_t v0 = begin_round(cur, n);
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = i == uint32_t(tid) ? v0 : ld_state<true>(cur + i);
      if (v != s && (nflags[v] & OGS_NODE_OVERLOADED)) continue;  // 741-752
      const D dv = dist[v];
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      for (uint32_t j0 = 0; j0 < m; j0 += kGRow) {
        uint64_t x[kGRow];
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          x[k] = j0 + k < m ? edges[b + j0 + k] : uint64_t(OGS_EDGE_DOWN);
        }
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          const uint32_t lo = static_cast<uint32_t>(x[k]);
          if (lo & OGS_EDGE_DOWN) continue;
          const uint32_t t = edge_dst(lo);
          const D c = dv + weight(x[k]);
          if (c < dist[t] && c < atomicMin(&dist[t], c)) append(t, r);
        }
      }
    }
    round_sync<true>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();
  }

  // ---- next-hop phase ------------------------------------------------------
  const uint32_t r0 = r;
  if (tid == 0) qcnt[0] = qcnt[1] = qcnt[2] = 0u;
  for (uint32_t i = tid; i < mw; i += kGBlock) mark[i] = 0u;
  __syncthreads();
  {
    const uint32_t b = gRow[s] - e0, m = gRow[s + 1] - e0 - b;
    for (uint32_t j = tid; j < m && j < 32u * W; j += kGBlock) {
      const uint64_t x = edges[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      if (lo & OGS_EDGE_DOWN) continue;
      const uint32_t t = edge_dst(lo);
      if (weight(x) == dist[t]) {
        atomicOr(&nh[(j >> 5) * Sn + t], 1u << (j & 31u));
        append(t, r0);
      }
    }
  }
  round_sync<true>();
  n = qcnt[(r0 + 1) % 3];
  __syncthreads();
  for (r = r0 + 1; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    const uint32_t v0 = begin_round(cur, n);
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = i == uint32_t(tid) ? v0 : ld_state<true>(cur + i);
      if (v == s || (nflags[v] & OGS_NODE_OVERLOADED)) continue;
      const D dv = dist[v];
      uint32_t nv[W];
#pragma unroll
      for (int w = 0; w < W; ++w) nv[w] = nh[w * Sn + v];
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      for (uint32_t j0 = 0; j0 < m; j0 += kGRow) {
        uint64_t x[kGRow];
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          x[k] = j0 + k < m ? edges[b + j0 + k] : uint64_t(OGS_EDGE_DOWN);
        }
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          const uint32_t lo = static_cast<uint32_t>(x[k]);
          if (lo & OGS_EDGE_DOWN) continue;
          const uint32_t t = edge_dst(lo);
          if (dv + weight(x[k]) != dist[t]) continue;  // not tight
          bool add = false;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const uint32_t a = nv[w] & ~nh[w * Sn + t];
            if (a && (a & ~atomicOr(&nh[w * Sn + t], a))) add = true;
          }
          if (add) append(t, r);
        }
      }
    }
    round_sync<true>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();
  }
  D* oD = oDist + u0 * Sn;
  uint32_t* oN = oNh + u0 * W * Sn;
  for (uint32_t v = tid; v < N; v += kGBlock) {
    oD[v] = dist[v];
#pragma unroll
    for (int w = 0; w < W; ++w) oN[w * Sn + v] = nh[w * Sn + v];
  }
}

// ---- one phase, packed {dist, next-hop word} in LDS (W = 1, u32 distances;
// N * 8 + one list bitset <= 160 kB, e.g. 20k nodes) -------------------------
// As the frontier kernel's packed form (packed_rounds): each relaxation is a
// 64-bit LDS compare-and-swap of {dist, nh}; a strictly shorter candidate
// replaces the word, an equal one ORs its next hops in, and either change
// pushes the target. Distances and next-hop sets converge in the same rounds
// (the two-phase forms run the next-hop propagation as a second sequence of
// rounds); the least fixpoint is the same (spf_core.h).
uint32_t global_lds3_bytes(uint32_t Sn) { return Sn * 8u + 4u * ((Sn + 31u) / 32u); }

// With a prefix table (pt.max_prefixes > 0) the unit's RouteDb is written by
// the same workgroup after its last round (route_one against the packed LDS
// words, one thread per prefix, coalesced record stores), as
// route_global_kernel would from the HBM rows: the launch no longer reads
// its own dist / next-hop rows back (G1: 64 x 20k x 8 B of the 44 MB the PMC
// counted per launch pair, profiles/r05_pmc_g1.json).
__global__ __launch_bounds__(kGBlock) void spf_global_lds3_kernel(
    ogs_graph g, const ogs_unit* __restrict__ units, uint32_t flags,
    uint32_t* __restrict__ oDist, uint32_t* __restrict__ oNh, uint32_t* __restrict__ scratch,
    ogs_prefix_table pt, ogs_spf_out out) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  const uint32_t u0 = blockIdx.x;
  const ogs_unit unit = units[u0];
  const uint32_t s = unit.src;
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const size_t Sn = size_t(g.max_nodes);
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint64_t* __restrict__ edges = g.edges + e0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0;
  uint32_t* q0 = scratch + u0 * 3 * Sn + Sn;
  uint32_t* q1 = q0 + Sn;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* dn = reinterpret_cast<uint64_t*>(smem);              // [N] {dist, nh}
  uint32_t* mark = reinterpret_cast<uint32_t*>(dn + Sn);        // [ceil(N/32)]
  const uint32_t mw = (uint32_t(Sn) + 31u) / 32u;
  __shared__ uint32_t qcnt[3];

  for (uint32_t v = tid; v < N; v += kGBlock) dn[v] = (v == s) ? 0ull : uint64_t(kInf);
  if (tid == 0) {
    q1[0] = s;
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  round_sync<true>();
  const uint32_t sb = gRow[s] - e0;  // the source's row: its link slots
  uint32_t r = 1, n = 1;
  for (; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    uint32_t* nxt = (r & 1) ? q0 : q1;
    const uint32_t v0 = uint32_t(tid) < n ? ld_state<true>(cur + tid) : 0u;
    for (uint32_t i = tid; i < mw; i += kGBlock) mark[i] = 0u;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kGBlock) {
      const uint32_t v = i == uint32_t(tid) ? v0 : ld_state<true>(cur + i);
      if (v != s && (nflags[v] & OGS_NODE_OVERLOADED)) continue;  // 741-752
      const uint64_t xv = dn[v];
      const uint32_t dv = static_cast<uint32_t>(xv), nv = static_cast<uint32_t>(xv >> 32);
      const uint32_t b = gRow[v] - e0, m = gRow[v + 1] - e0 - b;
      for (uint32_t j0 = 0; j0 < m; j0 += kGRow) {
        uint64_t x[kGRow];
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          x[k] = j0 + k < m ? edges[b + j0 + k] : uint64_t(OGS_EDGE_DOWN);
        }
#pragma unroll
        for (int k = 0; k < kGRow; ++k) {
          const uint32_t lo = static_cast<uint32_t>(x[k]);
          if (lo & OGS_EDGE_DOWN) continue;
          const uint32_t t = edge_dst(lo);
          const uint32_t c = dv + (hop ? 1u : static_cast<uint32_t>(x[k] >> 32));
          // the source contributes its link slot, every other node NH(v)
          // (a source slot past bit 31 is not in a one-word set: dropped, as
          // the two-phase forms drop slots >= 32 W)
          const uint32_t slot = b + j0 + k - sb;
          const uint32_t bits = (v == s) ? (slot < 32u ? 1u << slot : 0u) : nv;
          uint64_t old = dn[t];
          bool changed = false;
          for (;;) {
            const uint32_t dt = static_cast<uint32_t>(old), nt = static_cast<uint32_t>(old >> 32);
            if (c > dt || (c == dt && !(bits & ~nt))) break;
            const uint64_t nw = c < dt ? (uint64_t(c) | (uint64_t(bits) << 32))
                                       : (uint64_t(dt) | (uint64_t(nt | bits) << 32));
            const uint64_t seen = atomicCAS(reinterpret_cast<unsigned long long*>(&dn[t]),
                                            static_cast<unsigned long long>(old),
                                            static_cast<unsigned long long>(nw));
            if (seen == old) {
              changed = true;
              break;
            }
            old = seen;
          }
          if (changed) {
            const uint32_t bit = 1u << (t & 31u);
            if (!(atomicOr(&mark[t >> 5], bit) & bit)) {
              nxt[atomicAdd(&qcnt[(r + 1) % 3], 1u)] = t;
            }
          }
        }
      }
    }
    round_sync<true>();
    n = qcnt[(r + 1) % 3];
    __syncthreads();
  }
  uint32_t* oD = oDist + u0 * Sn;
  uint32_t* oN = oNh + u0 * Sn;
  for (uint32_t v = tid; v < N; v += kGBlock) {
    const uint64_t x = dn[v];
    oD[v] = static_cast<uint32_t>(x);
    oN[v] = static_cast<uint32_t>(x >> 32);
  }
  // ---- the unit's RouteDb from the final LDS words (every thread left the
  // last round through its barrier: dn is final) --------------------------
  const uint32_t Sp = uint32_t(pt.max_prefixes);
  if (Sp == 0u) return;
  const uint32_t p0 = pt.pfx_base[unit.topo];
  const uint32_t P = pt.pfx_base[unit.topo + 1] - p0;
  const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0, (flags & OGS_F_V4_OVER_V6) != 0,
                     (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
  const PackedView sv{dn};
  for (uint32_t p = tid; p < Sp; p += kGBlock) {
    const size_t rec = size_t(u0) * Sp + p;
    uint32_t meta = 0, metric = kInf, selBits = 0, mask[1] = {0u};
    if (p < P) route_one<uint32_t, 1>(pt, p0 + p, s, nflags, sv, cfg, meta, metric, mask, selBits);
    if (out.meta) out.meta[rec] = meta;
    if (out.metric) static_cast<uint32_t*>(out.metric)[rec] = metric;
    if (out.sel) out.sel[rec] = selBits;
    if (out.mask) out.mask[rec] = mask[0];
  }
}

hipError_t workspace(size_t bytes, hipStream_t stream, void** out);

// "spf_global" option: 0 (default) the global path only where the LDS paths
// cannot hold a unit, 1 every ogs_spf_routes call (A/B, parity tests).
// EngineOptions::spfGlobal (engine.h), default 0
// "spf_global_sync": 1 (default) rounds end with drained stores + barrier
// and state is read through sc1 loads; 0 agent-scope fences per round (A/B)
// EngineOptions::spfGlobalSync (engine.h), default 1
// "spf_global_lds": 1 (default) the best LDS form that fits -- one-phase
// packed {dist, nh} words (spf_global_lds3_kernel, W = 1, u32), else
// distances and next-hop words in two phases (spf_global_lds2_kernel), else
// distances only (spf_global_lds_kernel); 3 the two-phase form, 2 distances
// only, 0 always the all-HBM form (A/B)
// EngineOptions::spfGlobalLds (engine.h), default 1

// Does the LDS-resident workgroup path fit a unit of this graph? (the last
// fallback of spf_route.hip: dist + next-hop words, CSR read from L2)
bool lds_unit_fits(const ogs_graph& g, int W, uint32_t flags) {
  const uint64_t d = (flags & OGS_F_WIDE_METRIC) ? 8 : 4;
  const uint64_t b = ((uint64_t(g.max_nodes) * d + 15) & ~15ull) +
      ((uint64_t(g.max_nodes) * W * 4 + 15) & ~15ull);
  return b <= 160u * 1024u;
}

uint32_t frontier_lds_bytes(uint32_t Sn, int W, bool queue, bool ninfo, bool stamp8);

bool use_global(const ogs_graph& g, int W, uint32_t flags) {
  if (opts().spfGlobal == 1 || !lds_unit_fits(g, W, flags)) return true;
  // past the frontier kernel's LDS budget the remaining LDS paths sweep
  // every edge every round; on such graphs (large sparse / deep: WAN areas
  // of 16k+ nodes) the HBM frontier wins -- G1, 20,000-node WAN x 64
  // sources: 12.4 ms vs 35.0 ms for the multi-source sweep
  return g.max_nodes > 256 && !(flags & OGS_F_WIDE_METRIC) &&
      frontier_lds_bytes(uint32_t(g.max_nodes), W, false, true, false) > 160u * 1024u;
}

template <typename D, int W>
hipError_t launch_global_w(const ogs_graph& g, const ogs_prefix_table* pt,
                           const ogs_unit* units, int nUnits, uint32_t flags,
                           const ogs_spf_out& out, hipStream_t stream) {
  const size_t Sn = size_t(g.max_nodes);
  const size_t U = size_t(nUnits);
  auto r256 = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t distBytes = out.dist ? 0 : r256(U * Sn * sizeof(D));
  const size_t nhBytes = out.nh ? 0 : r256(U * W * Sn * 4);
  const size_t scratchBytes = r256(U * 3 * Sn * 4);
  void* ws = nullptr;
  hipError_t e = workspace(distBytes + nhBytes + scratchBytes, stream, &ws);
  if (e != hipSuccess) return e;
  char* base = static_cast<char*>(ws);
  D* dist = out.dist ? static_cast<D*>(out.dist) : reinterpret_cast<D*>(base);
  uint32_t* nh = out.nh ? out.nh : reinterpret_cast<uint32_t*>(base + distBytes);
  uint32_t* scratch = reinterpret_cast<uint32_t*>(base + distBytes + nhBytes);
  const uint32_t lds = global_lds_bytes(uint32_t(Sn), sizeof(D));
  const uint32_t lds2 = global_lds2_bytes(uint32_t(Sn), sizeof(D), W);
  const uint32_t lds3 = global_lds3_bytes(uint32_t(Sn));
  if constexpr (W == 1 && sizeof(D) == 4) {
    if (opts().spfGlobalLds == 1 && opts().spfGlobalSync && lds3 <= 160u * 1024u) {
      auto k = spf_global_lds3_kernel;
      if (lds3 > 64u * 1024u) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(lds3));
        if (e != hipSuccess) return e;
      }
      // the route pass runs inside the launch (no separate route kernel)
      const ogs_prefix_table ptv = pt ? *pt : ogs_prefix_table{};
      hipLaunchKernelGGL(k, dim3(nUnits), dim3(kGBlock), lds3, stream, g, units, flags,
                         reinterpret_cast<uint32_t*>(dist), nh, scratch, ptv, out);
      return hipGetLastError();
    }
  }
  if ((opts().spfGlobalLds == 1 || opts().spfGlobalLds == 3) && opts().spfGlobalSync && lds2 <= 160u * 1024u) {
    auto k = spf_global_lds2_kernel<D, W>;
    if (lds2 > 64u * 1024u) {
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(lds2));
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, dim3(nUnits), dim3(kGBlock), lds2, stream, g, units, flags, dist, nh,
                       scratch);
  } else if ((opts().spfGlobalLds == 1 || opts().spfGlobalLds == 2) && opts().spfGlobalSync &&
             lds <= 160u * 1024u) {
    auto k = spf_global_lds_kernel<D, W>;
    if (lds > 64u * 1024u) {
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, dim3(nUnits), dim3(kGBlock), lds, stream, g, units, flags, dist, nh,
                       scratch);
  } else if (opts().spfGlobalSync) {
    hipLaunchKernelGGL((spf_global_kernel<D, W, true>), dim3(nUnits), dim3(kGBlock), 0, stream,
                       g, units, flags, dist, nh, scratch);
  } else {
    hipLaunchKernelGGL((spf_global_kernel<D, W, false>), dim3(nUnits), dim3(kGBlock), 0, stream,
                       g, units, flags, dist, nh, scratch);
  }
  e = hipGetLastError();
  if (e != hipSuccess || !pt || pt->max_prefixes == 0) return e;
  return launch_route_global<D, W>(g, *pt, units, nUnits, flags, dist, nh, out, stream);
}

template <typename D>
hipError_t launch_global_d(const ogs_graph& g, const ogs_prefix_table* pt,
                           const ogs_unit* units, int nUnits, uint32_t flags, int W,
                           const ogs_spf_out& out, hipStream_t stream) {
  switch (W) {
    case 1: return launch_global_w<D, 1>(g, pt, units, nUnits, flags, out, stream);
    case 2: return launch_global_w<D, 2>(g, pt, units, nUnits, flags, out, stream);
    case 4: return launch_global_w<D, 4>(g, pt, units, nUnits, flags, out, stream);
    case 8: return launch_global_w<D, 8>(g, pt, units, nUnits, flags, out, stream);
    case 16: return launch_global_w<D, 16>(g, pt, units, nUnits, flags, out, stream);
    default: return launch_global_wide<D>(g, pt, units, nUnits, flags, W, out, stream);
  }
}

// SPF (+ RouteDb when pt is non-NULL) of every unit through the global path.
hipError_t launch_spf_routes_global(const ogs_graph& g, const ogs_prefix_table* pt,
                                    const ogs_unit* units, int nUnits, uint32_t flags,
                                    int W, const ogs_spf_out& out, hipStream_t stream) {
  if (flags & OGS_F_WIDE_METRIC) {
    return launch_global_d<uint64_t>(g, pt, units, nUnits, flags, W, out, stream);
  }
  return launch_global_d<uint32_t>(g, pt, units, nUnits, flags, W, out, stream);
}

// ogs_routes_from_spf: route_global_kernel over caller-held SPF state.
hipError_t launch_routes_from_spf(const ogs_graph& g, const ogs_prefix_table& pt,
                                  const ogs_unit* units, int n, const void* dist,
                                  const uint32_t* nh, const uint32_t* reach, uint32_t flags,
                                  int W, const ogs_spf_out& out, hipStream_t stream) {
  const bool wide = (flags & OGS_F_WIDE_METRIC) != 0;
#define OGS_RFS(W_)                                                                         \
  return wide ? launch_route_global<uint64_t, W_>(g, pt, units, n, flags,                   \
                                                  static_cast<const uint64_t*>(dist), nh,   \
                                                  out, stream, reach)                       \
              : launch_route_global<uint32_t, W_>(g, pt, units, n, flags,                   \
                                                  static_cast<const uint32_t*>(dist), nh,   \
                                                  out, stream, reach);
  switch (W) {
    case 1: OGS_RFS(1)
    case 2: OGS_RFS(2)
    case 4: OGS_RFS(4)
    case 8: OGS_RFS(8)
    case 16: OGS_RFS(16)
    default:  // sources of more than 512 links
      return wide ? launch_route_global_wide<uint64_t>(g, pt, units, n, flags, W,
                                                       static_cast<const uint64_t*>(dist), nh,
                                                       out, stream, reach)
                  : launch_route_global_wide<uint32_t>(g, pt, units, n, flags, W,
                                                       static_cast<const uint32_t*>(dist), nh,
                                                       out, stream, reach);
  }
#undef OGS_RFS
}

}  // namespace ogs
