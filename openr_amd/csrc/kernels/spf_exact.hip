// spf_exact.hip — SPF in the reference's own extraction order, for the
// topologies where that order decides the result: zero link metrics and
// negative i32 metrics (LinkStateMetric is uint64_t, LinkState.h:16; the
// thrift i32 is sign-extended, LinkState.cpp:77-78, and sums wrap).
//
// LinkState::runSpf (LinkState.cpp:720-820) settles nodes in DijkstraQ order
// -- smallest (metric, node name), LinkState.h:618-626 -- and a node's
// next-hop set is built while its neighbours are settled: on a relaxation
// with metric >= the node's current one it unions the relaxing node's set
// (or, from the source, its own name), on > it first resets. With metrics
// >= 1 that equals the order-free fixpoint the other kernels solve; with a
// zero metric the union depends on which of two equal-distance nodes is
// settled first, and with wrapping sums the "shortest" distances themselves
// depend on the order. So this kernel replays the algorithm:
//  * one wavefront per unit, state in HBM (key u64, status, next-hop slot
//    sets in the ogs_spf_out layout, the open list);
//  * each step extracts the open node with the smallest (key, id) -- node
//    ids are name ranks, so id order is the reference's name tie-break --
//    by a 64-lane scan of the open list and a wave min-reduction;
//  * the settled node's row is relaxed lane-parallel; parallel links to one
//    neighbour collapse to their minimum first (the sequential loop reaches
//    the same state: reset on the smaller metric, union on ties), so a
//    neighbour is updated by exactly one lane;
//  * next hops are link-slot sets: the source's relaxation of t gives t's
//    name = every slot of the source's row leading to t; at the end each set
//    is filtered by getNextHopsThrift's link test (link up, max metric ==
//    dist(neighbour), SpfSolver.cpp:705-743), which is what every other
//    kernel's sets already hold.
// O(N) sequential steps: used only for units whose topology needs it.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "route_core.h"
#include "route_global.h"
#include "spf_core.h"

namespace ogs {

constexpr int kExactRow = 512;  // rows staged in LDS (longer: spf_exact_wide_kernel)

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// LinkStateMetric of an edge: the stored low 32 bits sign-extended (a u64
// from an i32 is exactly that), 1 for hop counts.
__device__ __forceinline__ uint64_t exact_weight(uint64_t x, bool hop) {
  return hop ? 1ull
             : static_cast<uint64_t>(static_cast<int64_t>(static_cast<int32_t>(
                   static_cast<uint32_t>(x >> 32))));
}

template <int W>
__global__ __launch_bounds__(64) void spf_exact_kernel(
    ogs_graph g, const ogs_unit* __restrict__ units, uint32_t flags,
    uint64_t* __restrict__ oDist, uint32_t* __restrict__ oNh,
    uint32_t* __restrict__ scratch, uint32_t* __restrict__ oReach) {
  constexpr uint64_t kInf = ~0ull;
  constexpr uint32_t kOpen = 1, kDone = 2;
  const int lane = threadIdx.x;
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
  uint64_t* key = oDist + u0 * Sn;
  uint32_t* nh = oNh + u0 * W * Sn;
  uint32_t* st = scratch + u0 * 2 * Sn;
  uint32_t* open = st + Sn;

  __shared__ uint32_t srcNbr[kExactRow];  // neighbour of each source slot
  __shared__ uint32_t rowT[kExactRow];
  __shared__ uint64_t rowC[kExactRow];
  __shared__ uint8_t rowV[kExactRow];

  const uint32_t sb = gRow[s] - e0, sdeg = gRow[s + 1] - e0 - sb;
  for (uint32_t j = lane; j < sdeg; j += 64) {
    srcNbr[j] = edge_dst(static_cast<uint32_t>(edges[sb + j]));
  }
  for (uint32_t v = lane; v < N; v += 64) {
    key[v] = kInf;
    st[v] = 0u;
#pragma unroll
    for (int w = 0; w < W; ++w) nh[w * Sn + v] = 0u;
  }
  wave_sync();
  if (lane == 0) {
    key[s] = 0;
    st[s] = kOpen;
    open[0] = s;
  }
  wave_sync();
  uint32_t nOpen = 1;

  while (nOpen) {
    // ---- extractMin: smallest (key, id) over the open list --------------
    uint64_t bk = kInf;
    uint32_t bv = 0xFFFFFFFFu, bi = 0;
    for (uint32_t i = lane; i < nOpen; i += 64) {
      const uint32_t v = open[i];
      const uint64_t k = key[v];
      if (k < bk || (k == bk && v < bv)) {
        bk = k;
        bv = v;
        bi = i;
      }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      const uint64_t ok = __shfl_xor(bk, d, 64);
      const uint32_t ov = __shfl_xor(bv, d, 64);
      const uint32_t oi = __shfl_xor(bi, d, 64);
      if (ok < bk || (ok == bk && ov < bv)) {
        bk = ok;
        bv = ov;
        bi = oi;
      }
    }
    const uint32_t u = bv;
    const uint64_t du = bk;
    wave_sync();
    if (lane == 0) {
      open[bi] = open[nOpen - 1];
      st[u] = kDone;
    }
    --nOpen;
    wave_sync();
    if (u != s && (nflags[u] & OGS_NODE_OVERLOADED)) continue;  // 741-752

    // ---- relax u's row -----------------------------------------------------
    const uint32_t b = gRow[u] - e0, m = gRow[u + 1] - e0 - b;
    for (uint32_t j = lane; j < m; j += 64) {
      const uint64_t x = edges[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      const uint32_t t = edge_dst(lo);
      rowT[j] = t;
      rowC[j] = du + exact_weight(x, hop);  // wraps like the reference's u64
      rowV[j] = !(lo & OGS_EDGE_DOWN) && st[t] != kDone;
    }
    wave_sync();
    uint32_t nu[W];
#pragma unroll
    for (int w = 0; w < W; ++w) nu[w] = (u == s) ? 0u : nh[w * Sn + u];
    for (uint32_t j0 = 0; j0 < m; j0 += 64) {  // wave-uniform trip count
      const uint32_t j = j0 + lane;
      bool append = false;
      uint32_t t = 0;
      if (j < m && rowV[j]) {
        t = rowT[j];
        uint64_t c = rowC[j];
        bool rep = true;  // lowest valid slot of u's row leading to t
        for (uint32_t k = 0; k < m; ++k) {
          if (k == j || !rowV[k] || rowT[k] != t) continue;
          if (k < j) rep = false;
          if (rowC[k] < c) c = rowC[k];
        }
        if (rep) {
          uint32_t add[W];
#pragma unroll
          for (int w = 0; w < W; ++w) add[w] = nu[w];
          if (u == s) {  // "directly connected": the neighbour's own name
            for (uint32_t k = 0; k < sdeg && k < 32u * W; ++k) {
              if (srcNbr[k] == t) add[k >> 5] |= 1u << (k & 31u);
            }
          }
          const uint32_t stt = st[t];
          const uint64_t kt = key[t];
          if (stt == 0u) {  // insertNode(t, c), then the >= branch
            key[t] = c;
            st[t] = kOpen;
#pragma unroll
            for (int w = 0; w < W; ++w) nh[w * Sn + t] = add[w];
            append = true;
          } else if (kt > c) {  // strictly better: reset, then union
            key[t] = c;
#pragma unroll
            for (int w = 0; w < W; ++w) nh[w * Sn + t] = add[w];
          } else if (kt == c) {
#pragma unroll
            for (int w = 0; w < W; ++w) nh[w * Sn + t] |= add[w];
          }
        }
      }
      // one representative lane per distinct neighbour: appends are disjoint
      const uint64_t ball = __ballot(append);
      if (append) {
        const uint32_t at = nOpen + __builtin_amdgcn_mbcnt_hi(
            uint32_t(ball >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(ball), 0u));
        open[at] = t;
      }
      nOpen += __popcll(ball);
    }
    wave_sync();
  }

  // ---- outputs: unreachable = all ones, plus the settled bitset (a reached
  // node's wrapped distance can itself be all ones); getNextHopsThrift's
  // link filter ------------------------------------------------------------
  for (uint32_t v = lane; v < N; v += 64) {
    const bool done = st[v] == kDone;
    if (!done) key[v] = kInf;
  }
  uint32_t* reach = oReach + size_t(u0) * ((Sn + 31) / 32);
  for (uint32_t i = lane; i < (uint32_t(Sn) + 31u) / 32u; i += 64) {
    uint32_t word = 0u;
    for (uint32_t b = 0; b < 32u; ++b) {
      const uint32_t v = 32u * i + b;
      if (v < N && st[v] == kDone) word |= 1u << b;
    }
    reach[i] = word;
  }
  wave_sync();
  uint32_t f[W];
#pragma unroll
  for (int w = 0; w < W; ++w) f[w] = 0u;
  for (uint32_t k = 0; k < sdeg && k < 32u * W; ++k) {
    const uint64_t x = edges[sb + k];
    const uint32_t lo = static_cast<uint32_t>(x);
    const uint32_t t = edge_dst(lo);
    if (!(lo & OGS_EDGE_DOWN) && st[t] == kDone && exact_weight(x, hop) == key[t]) {
      f[k >> 5] |= 1u << (k & 31u);
    }
  }
  for (uint32_t v = lane; v < N; v += 64) {
#pragma unroll
    for (int w = 0; w < W; ++w) nh[w * Sn + v] &= f[w];
  }
}

// The same replay for rows of any length and next-hop sets of any width
// (nodes of 512+ links; runtime W): rows are read from HBM instead of staged
// in LDS, next-hop words are read and written in place.
__global__ __launch_bounds__(64) void spf_exact_wide_kernel(
    ogs_graph g, const ogs_unit* __restrict__ units, uint32_t flags, int W,
    uint64_t* __restrict__ oDist, uint32_t* __restrict__ oNh,
    uint32_t* __restrict__ scratch, uint32_t* __restrict__ oReach) {
  constexpr uint64_t kInf = ~0ull;
  constexpr uint32_t kOpen = 1, kDone = 2;
  const int lane = threadIdx.x;
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
  uint64_t* key = oDist + u0 * Sn;
  uint32_t* nh = oNh + u0 * size_t(W) * Sn;
  uint32_t* st = scratch + u0 * 2 * Sn;
  uint32_t* open = st + Sn;
  const uint32_t sb = gRow[s] - e0, sdeg = gRow[s + 1] - e0 - sb;
  for (uint32_t v = lane; v < N; v += 64) {
    key[v] = kInf;
    st[v] = 0u;
    for (int w = 0; w < W; ++w) nh[w * Sn + v] = 0u;
  }
  wave_sync();
  if (lane == 0) {
    key[s] = 0;
    st[s] = kOpen;
    open[0] = s;
  }
  wave_sync();
  uint32_t nOpen = 1;
  while (nOpen) {
    uint64_t bk = kInf;
    uint32_t bv = 0xFFFFFFFFu, bi = 0;
    for (uint32_t i = lane; i < nOpen; i += 64) {
      const uint32_t v = open[i];
      const uint64_t k = key[v];
      if (k < bk || (k == bk && v < bv)) {
        bk = k;
        bv = v;
        bi = i;
      }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      const uint64_t ok = __shfl_xor(bk, d, 64);
      const uint32_t ov = __shfl_xor(bv, d, 64);
      const uint32_t oi = __shfl_xor(bi, d, 64);
      if (ok < bk || (ok == bk && ov < bv)) {
        bk = ok;
        bv = ov;
        bi = oi;
      }
    }
    const uint32_t u = bv;
    const uint64_t du = bk;
    wave_sync();
    if (lane == 0) {
      open[bi] = open[nOpen - 1];
      st[u] = kDone;
    }
    --nOpen;
    wave_sync();
    if (u != s && (nflags[u] & OGS_NODE_OVERLOADED)) continue;  // 741-752
    const uint32_t b = gRow[u] - e0, m = gRow[u + 1] - e0 - b;
    auto valid = [&](uint32_t k, uint32_t& t, uint64_t& c) {
      const uint64_t x = edges[b + k];
      const uint32_t lo = static_cast<uint32_t>(x);
      t = edge_dst(lo);
      c = du + exact_weight(x, hop);
      return !(lo & OGS_EDGE_DOWN) && st[t] != kDone;
    };
    for (uint32_t j0 = 0; j0 < m; j0 += 64) {  // wave-uniform trip count
      const uint32_t j = j0 + lane;
      bool append = false;
      uint32_t t = 0;
      uint64_t c = 0;
      if (j < m && valid(j, t, c)) {
        bool rep = true;  // lowest valid slot of u's row leading to t
        for (uint32_t k = 0; k < m; ++k) {
          uint32_t tk;
          uint64_t ck;
          if (k == j || !valid(k, tk, ck) || tk != t) continue;
          if (k < j) rep = false;
          if (ck < c) c = ck;
        }
        if (rep) {
          const uint32_t stt = st[t];
          const uint64_t kt = key[t];
          const int mode = stt == 0u ? 0 : (kt > c ? 1 : (kt == c ? 2 : 3));
          if (mode != 3) {
            if (mode != 2) key[t] = c;
            if (mode == 0) st[t] = kOpen;
            for (int w = 0; w < W; ++w) {
              uint32_t add = (u == s) ? 0u : nh[w * Sn + u];
              if (u == s) {  // "directly connected": the neighbour's own name
                for (uint32_t k = 32u * w; k < sdeg && k < 32u * (w + 1); ++k) {
                  if (edge_dst(static_cast<uint32_t>(edges[sb + k])) == t) {
                    add |= 1u << (k & 31u);
                  }
                }
              }
              nh[w * Sn + t] = mode == 2 ? (nh[w * Sn + t] | add) : add;
            }
            append = mode == 0;
          }
        }
      }
      const uint64_t ball = __ballot(append);
      if (append) {
        const uint32_t at = nOpen + __builtin_amdgcn_mbcnt_hi(
            uint32_t(ball >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(ball), 0u));
        open[at] = t;
      }
      nOpen += __popcll(ball);
    }
    wave_sync();
  }
  for (uint32_t v = lane; v < N; v += 64) {
    if (st[v] != kDone) key[v] = kInf;
  }
  uint32_t* reach = oReach + size_t(u0) * ((Sn + 31) / 32);
  for (uint32_t i = lane; i < (uint32_t(Sn) + 31u) / 32u; i += 64) {
    uint32_t word = 0u;
    for (uint32_t bb = 0; bb < 32u; ++bb) {
      const uint32_t v = 32u * i + bb;
      if (v < N && st[v] == kDone) word |= 1u << bb;
    }
    reach[i] = word;
  }
  wave_sync();
  // getNextHopsThrift's link filter, one word at a time
  for (int w = 0; w < W; ++w) {
    uint32_t f = 0u;
    for (uint32_t k = 32u * w; k < sdeg && k < 32u * (w + 1); ++k) {
      const uint64_t x = edges[sb + k];
      const uint32_t lo = static_cast<uint32_t>(x);
      const uint32_t t = edge_dst(lo);
      if (!(lo & OGS_EDGE_DOWN) && st[t] == kDone && exact_weight(x, hop) == key[t]) {
        f |= 1u << (k & 31u);
      }
    }
    for (uint32_t v = lane; v < N; v += 64) nh[w * Sn + v] &= f;
  }
}

hipError_t workspace(size_t bytes, hipStream_t stream, void** out);

hipError_t launch_exact_wide(const ogs_graph& g, const ogs_prefix_table* pt,
                             const ogs_unit* units, int nUnits, uint32_t flags, int W,
                             const ogs_spf_out& out, hipStream_t stream) {
  const size_t Sn = size_t(g.max_nodes), U = size_t(nUnits);
  auto r256 = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t distBytes = out.dist ? 0 : r256(U * Sn * 8);
  const size_t nhBytes = out.nh ? 0 : r256(U * W * Sn * 4);
  const size_t scratchBytes = r256(U * 2 * Sn * 4);
  const size_t reachBytes = out.reached ? 0 : r256(U * ((Sn + 31) / 32) * 4);
  void* ws = nullptr;
  hipError_t e = workspace(distBytes + nhBytes + scratchBytes + reachBytes, stream, &ws);
  if (e != hipSuccess) return e;
  char* base = static_cast<char*>(ws);
  uint64_t* dist = out.dist ? static_cast<uint64_t*>(out.dist) : reinterpret_cast<uint64_t*>(base);
  uint32_t* nh = out.nh ? out.nh : reinterpret_cast<uint32_t*>(base + distBytes);
  uint32_t* scratch = reinterpret_cast<uint32_t*>(base + distBytes + nhBytes);
  uint32_t* reach = out.reached ? out.reached
                                : reinterpret_cast<uint32_t*>(base + distBytes + nhBytes +
                                                              scratchBytes);
  hipLaunchKernelGGL(spf_exact_wide_kernel, dim3(nUnits), dim3(64), 0, stream, g, units, flags,
                     W, dist, nh, scratch, reach);
  e = hipGetLastError();
  if (e != hipSuccess || !pt || pt->max_prefixes == 0) return e;
  if (W <= 16) {
    switch (W) {
      case 1: return launch_route_global<uint64_t, 1>(g, *pt, units, nUnits, flags, dist, nh, out, stream, reach);
      case 2: return launch_route_global<uint64_t, 2>(g, *pt, units, nUnits, flags, dist, nh, out, stream, reach);
      case 4: return launch_route_global<uint64_t, 4>(g, *pt, units, nUnits, flags, dist, nh, out, stream, reach);
      case 8: return launch_route_global<uint64_t, 8>(g, *pt, units, nUnits, flags, dist, nh, out, stream, reach);
      default: return launch_route_global<uint64_t, 16>(g, *pt, units, nUnits, flags, dist, nh, out, stream, reach);
    }
  }
  return launch_route_global_wide<uint64_t>(g, *pt, units, nUnits, flags, W, dist, nh, out,
                                            stream, reach);
}

template <int W>
hipError_t launch_exact_w(const ogs_graph& g, const ogs_prefix_table* pt,
                          const ogs_unit* units, int nUnits, uint32_t flags,
                          const ogs_spf_out& out, hipStream_t stream) {
  const size_t Sn = size_t(g.max_nodes), U = size_t(nUnits);
  auto r256 = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t distBytes = out.dist ? 0 : r256(U * Sn * 8);
  const size_t nhBytes = out.nh ? 0 : r256(U * W * Sn * 4);
  const size_t scratchBytes = r256(U * 2 * Sn * 4);
  const size_t reachBytes = out.reached ? 0 : r256(U * ((Sn + 31) / 32) * 4);
  void* ws = nullptr;
  hipError_t e = workspace(distBytes + nhBytes + scratchBytes + reachBytes, stream, &ws);
  if (e != hipSuccess) return e;
  char* base = static_cast<char*>(ws);
  uint64_t* dist = out.dist ? static_cast<uint64_t*>(out.dist) : reinterpret_cast<uint64_t*>(base);
  uint32_t* nh = out.nh ? out.nh : reinterpret_cast<uint32_t*>(base + distBytes);
  uint32_t* scratch = reinterpret_cast<uint32_t*>(base + distBytes + nhBytes);
  uint32_t* reach = out.reached ? out.reached
                                : reinterpret_cast<uint32_t*>(base + distBytes + nhBytes +
                                                              scratchBytes);
  hipLaunchKernelGGL((spf_exact_kernel<W>), dim3(nUnits), dim3(64), 0, stream, g, units,
                     flags, dist, nh, scratch, reach);
  e = hipGetLastError();
  if (e != hipSuccess || !pt || pt->max_prefixes == 0) return e;
  return launch_route_global<uint64_t, W>(g, *pt, units, nUnits, flags, dist, nh, out, stream,
                                          reach);
}

// OGS_F_EXACT_ORDER: SPF (+ RouteDb) in the reference's extraction order.
// 64-bit distances (OGS_F_WIDE_METRIC layout); any degree.
hipError_t launch_spf_routes_exact(const ogs_graph& g, const ogs_prefix_table* pt,
                                   const ogs_unit* units, int nUnits, uint32_t flags,
                                   int W, const ogs_spf_out& out, hipStream_t stream) {
  if (!(flags & OGS_F_WIDE_METRIC)) return hipErrorInvalidValue;
  // rows past the LDS row stage or sets past 16 words: rows read from HBM
  if (g.max_degree > kExactRow || W > 16 || (W & (W - 1))) {
    return launch_exact_wide(g, pt, units, nUnits, flags, W, out, stream);
  }
  switch (W) {
    case 1: return launch_exact_w<1>(g, pt, units, nUnits, flags, out, stream);
    case 2: return launch_exact_w<2>(g, pt, units, nUnits, flags, out, stream);
    case 4: return launch_exact_w<4>(g, pt, units, nUnits, flags, out, stream);
    case 8: return launch_exact_w<8>(g, pt, units, nUnits, flags, out, stream);
    case 16: return launch_exact_w<16>(g, pt, units, nUnits, flags, out, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace ogs
