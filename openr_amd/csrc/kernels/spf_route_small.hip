// spf_route_small.hip — latency-optimised fused SPF + RouteDb for small
// topologies (<= 256 nodes, degree <= 8): the C1/C2 batch path.
//
// Same algorithm and outputs as spf_route.hip (see its header for the
// reference mapping); what changes is how one unit's work is laid onto the
// CDNA4 machine. A C2 launch is 4096 independent units, i.e. 16 units per CU,
// all resident at once, so kernel time == one unit's latency. This variant
// attacks that latency:
//  * staging: every global array the unit needs (CSR row offsets + edges,
//    node flags, the topology's prefix table) is loaded in ONE batch of
//    independent loads per lane and only then written to LDS, so the unit
//    pays ~one HBM latency instead of one per array / per element;
//  * relaxation: each lane owns NPL nodes and keeps their edges (<= MAXD)
//    and current (dist, next-hop) values in registers. A round issues all
//    dist[u] / nh[u] LDS reads of a node back to back and folds them with
//    selects (no data-dependent branches), so a round costs ~2 LDS latencies
//    per owned node instead of 3 dependent round trips per edge;
//  * unit width UT in {64, 128, 256}: 64 = one wavefront per unit, no
//    barriers; 128/256 = one workgroup per unit (1-2 nodes per lane, one
//    s_barrier per round), trading a barrier for half the serial work.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "route_core.h"
#include "spf_core.h"

namespace ogs {

template <int UT>
struct SmallScope;
template <>
struct SmallScope<64> : UnitScope<64> {};
template <int UT>
struct SmallScope {  // one workgroup (UT threads) per unit
  static __device__ __forceinline__ void sync() { __syncthreads(); }
  static __device__ __forceinline__ bool any(bool x) {
    return __syncthreads_or(x) != 0;
  }
};

// LDS image of one unit. Offsets are computed identically on host and device.
struct SmallLayout {
  uint32_t dist, nh, row, edges, flags, advOff, advNode, advMetrics, advMinNh,
      pfxFlags, total;
  __host__ __device__ static SmallLayout make(uint32_t N, uint32_t E,
                                              uint32_t P, uint32_t A, int W,
                                              int distBytes) {
    SmallLayout L;
    uint32_t o = 0;
    L.dist = o;
    o += align16(uint64_t(N) * distBytes);
    L.nh = o;
    o += align16(uint64_t(N) * W * 4);
    L.row = o;
    o += align16(uint64_t(N + 1) * 4);
    L.edges = o;
    o += align16(uint64_t(E) * 8);
    L.flags = o;
    o += align16(N);
    L.advOff = o;
    o += align16(uint64_t(P + 1) * 4);
    L.advNode = o;
    o += align16(uint64_t(A) * 4);
    L.advMetrics = o;
    o += align16(uint64_t(A) * 16);
    L.advMinNh = o;
    o += align16(uint64_t(A) * 8);
    L.pfxFlags = o;
    o += align16(P);
    L.total = o;
    return L;
  }
};

// Batched global->LDS copy of up to K*UT elements per array: all loads of
// all arrays are issued before the first LDS write.
template <int UT, int K, typename T>
struct Stage {
  T v[K];
  __device__ __forceinline__ void load(const T* __restrict__ src, uint32_t n,
                                       int lane, uint32_t base) {
    if (n == 0) return;  // unit-uniform: never touch an empty array
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t i = base + uint32_t(k * UT + lane);
      v[k] = src[i < n ? i : (n ? n - 1 : 0)];  // clamp: no branch per load
    }
  }
  __device__ __forceinline__ void store(T* dst, uint32_t n, int lane,
                                        uint32_t base) const {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t i = base + uint32_t(k * UT + lane);
      if (i < n) dst[i] = v[k];
    }
  }
};

template <typename D, int W, int UT, int NPL, int MAXD>
__global__ __launch_bounds__(UT == 64 ? 256 : UT) void spf_route_small_kernel(
    ogs_graph g, ogs_prefix_table pt, int hasPrefixes,
    const ogs_unit* __restrict__ units, int nUnits, uint32_t flags,
    ogs_spf_out out, uint32_t ldsPerUnit, uint32_t maxA) {
  using Scope = SmallScope<UT>;
  constexpr D kInf = DistInf<D>::value;
  constexpr int kBlockThreads = UT == 64 ? 256 : UT;
  constexpr int kUnitsPerBlock = kBlockThreads / UT;
  const int uib = threadIdx.x / UT;
  const int lane = threadIdx.x % UT;
  const int uidx = blockIdx.x * kUnitsPerBlock + uib;
  if (uidx >= nUnits) return;
#ifdef OGS_STAMPS  // diagnostic build only: phase clocks into out.sel
  const uint64_t tStart = __builtin_amdgcn_s_memtime();
  uint64_t tStaged = 0, tSpf = 0;
  uint32_t rounds = 0;
#endif

  const ogs_unit unit = units[uidx];
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const uint32_t s = unit.src;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint32_t E = gRow[N] - e0;
  uint32_t p0 = 0, P = 0, a0 = 0, A = 0;
  if (hasPrefixes) {
    p0 = pt.pfx_base[unit.topo];
    P = pt.pfx_base[unit.topo + 1] - p0;
    a0 = pt.adv_off[p0];
    A = pt.adv_off[p0 + P] - a0;
  }
  const SmallLayout L =
      SmallLayout::make(g.max_nodes, g.max_edges, pt.max_prefixes, maxA, W,
                        sizeof(D));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* base = smem + uib * ldsPerUnit;
  D* dist = reinterpret_cast<D*>(base + L.dist);
  uint32_t* nh = reinterpret_cast<uint32_t*>(base + L.nh);
  uint32_t* lrow = reinterpret_cast<uint32_t*>(base + L.row);
  uint64_t* ledg = reinterpret_cast<uint64_t*>(base + L.edges);
  uint8_t* lflags = reinterpret_cast<uint8_t*>(base + L.flags);
  uint32_t* lAdvOff = reinterpret_cast<uint32_t*>(base + L.advOff);
  uint32_t* lAdvNode = reinterpret_cast<uint32_t*>(base + L.advNode);
  int4* lAdvMetrics = reinterpret_cast<int4*>(base + L.advMetrics);
  int64_t* lAdvMinNh = reinterpret_cast<int64_t*>(base + L.advMinNh);
  uint8_t* lPfxFlags = reinterpret_cast<uint8_t*>(base + L.pfxFlags);

  // ---- one batch of global loads, then LDS writes ------------------------
  {
    constexpr int KE = (MAXD * NPL + 1) / 2 + 1;  // edges per lane per pass
    Stage<UT, NPL + 1, uint32_t> sRow;
    Stage<UT, KE, uint64_t> sEdge;
    Stage<UT, NPL, uint8_t> sFlag;
    sRow.load(gRow, N + 1, lane, 0);
    sEdge.load(g.edges + e0, E, lane, 0);
    sFlag.load(g.node_flags + nb, N, lane, 0);
    Stage<UT, 2, uint32_t> sOff, sNode;
    Stage<UT, 2, int4> sMet;
    Stage<UT, 2, int64_t> sMin;
    Stage<UT, 2, uint8_t> sPf;
    if (hasPrefixes) {
      sOff.load(pt.adv_off + p0, P + 1, lane, 0);
      sNode.load(pt.adv_node + a0, A, lane, 0);
      sMet.load(reinterpret_cast<const int4*>(pt.adv_metrics) + a0, A, lane, 0);
      sMin.load(pt.adv_min_nh + a0, A, lane, 0);
      sPf.load(pt.pfx_flags + p0, P, lane, 0);
    }
    sRow.store(lrow, N + 1, lane, 0);
    sEdge.store(ledg, E, lane, 0);
    sFlag.store(lflags, N, lane, 0);
    for (uint32_t b = KE * UT; b < E; b += KE * UT) {  // rare: big rows
      sEdge.load(g.edges + e0, E, lane, b);
      sEdge.store(ledg, E, lane, b);
    }
    if (hasPrefixes) {
      sOff.store(lAdvOff, P + 1, lane, 0);
      sNode.store(lAdvNode, A, lane, 0);
      sMet.store(lAdvMetrics, A, lane, 0);
      sMin.store(lAdvMinNh, A, lane, 0);
      sPf.store(lPfxFlags, P, lane, 0);
      for (uint32_t b = 2 * UT; b < P + 1 || b < A; b += 2 * UT) {
        sOff.load(pt.adv_off + p0, P + 1, lane, b);
        sNode.load(pt.adv_node + a0, A, lane, b);
        sMet.load(reinterpret_cast<const int4*>(pt.adv_metrics) + a0, A, lane, b);
        sMin.load(pt.adv_min_nh + a0, A, lane, b);
        sPf.load(pt.pfx_flags + p0, P, lane, b);
        sOff.store(lAdvOff, P + 1, lane, b);
        sNode.store(lAdvNode, A, lane, b);
        sMet.store(lAdvMetrics, A, lane, b);
        sMin.store(lAdvMinNh, A, lane, b);
        sPf.store(lPfxFlags, P, lane, b);
      }
    }
    // prefix segment offsets become unit-local
    for (uint32_t i = lane; hasPrefixes && i <= P; i += UT) lAdvOff[i] -= a0;
  }
  Scope::sync();

#ifdef OGS_STAMPS
  tStaged = __builtin_amdgcn_s_memtime();
#endif
  // ---- register-resident node slots --------------------------------------
  const bool hop = flags & OGS_F_HOP_METRIC;
  uint64_t ed[NPL][MAXD];
  D dcur[NPL];
  uint32_t ncur[NPL][W];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const uint32_t v = lane + k * UT;
    const bool own = v < N;
    // staged row offsets are global; the staged edges start at e0
    const uint32_t eb = own ? lrow[v] - e0 : 0u;
    const uint32_t deg = own ? lrow[v + 1] - lrow[v] : 0u;
#pragma unroll
    for (int j = 0; j < MAXD; ++j) {
      ed[k][j] = (uint32_t(j) < deg) ? ledg[eb + j] : uint64_t(OGS_EDGE_DOWN);
    }
    dcur[k] = (v == s) ? D(0) : kInf;
#pragma unroll
    for (int w = 0; w < W; ++w) ncur[k][w] = 0u;
    if (own) {
      dist[v] = dcur[k];
#pragma unroll
      for (int w = 0; w < W; ++w) nh[v * W + w] = 0u;
    }
  }
  Scope::sync();

  // ---- SPF: branch-free pull rounds to the fixpoint -----------------------
  for (;;) {
    bool changed = false;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const uint32_t v = lane + k * UT;
      D du[MAXD];
      uint32_t uu[MAXD];
      bool ok[MAXD];
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        const uint32_t lo = static_cast<uint32_t>(ed[k][j]);
        const uint32_t u = edge_dst(lo);
        ok[j] = !(lo & OGS_EDGE_DOWN) &&
            !((lo & OGS_EDGE_DST_OVERLOADED) && u != s);
        uu[j] = ok[j] ? u : 0u;
      }
#pragma unroll
      for (int j = 0; j < MAXD; ++j) du[j] = dist[uu[j]];
      D best = kInf;
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        const D w = hop ? D(1) : static_cast<D>(ed[k][j] >> 32);
        const D cand = (ok[j] && du[j] != kInf) ? du[j] + w : kInf;
        best = cand < best ? cand : best;
      }
      uint32_t m[W];
#pragma unroll
      for (int w = 0; w < W; ++w) m[w] = 0u;
      if (best != kInf) {
#pragma unroll
        for (int j = 0; j < MAXD; ++j) {
          const uint32_t lo = static_cast<uint32_t>(ed[k][j]);
          const D w8 = hop ? D(1) : static_cast<D>(ed[k][j] >> 32);
          const bool tight = ok[j] && du[j] != kInf && du[j] + w8 == best;
          const bool fromSrc = uu[j] == s;
          const uint32_t slot = edge_rslot(lo);
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const uint32_t c = fromSrc
                ? ((int(slot >> 5) == w) ? (1u << (slot & 31u)) : 0u)
                : nh[uu[j] * W + w];
            m[w] |= tight ? c : 0u;
          }
        }
      }
      bool diff = (best != dcur[k]);
#pragma unroll
      for (int w = 0; w < W; ++w) diff |= (m[w] != ncur[k][w]);
      if (v < N && v != s && diff) {
        dcur[k] = best;
        dist[v] = best;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          ncur[k][w] = m[w];
          nh[v * W + w] = m[w];
        }
        changed = true;
      }
    }
#ifdef OGS_STAMPS
    ++rounds;
#endif
    if (!Scope::any(changed)) break;
  }
#ifdef OGS_STAMPS
  tSpf = __builtin_amdgcn_s_memtime();
#endif

  // ---- SPF outputs ---------------------------------------------------------
  const uint32_t Sn = g.max_nodes;
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const uint32_t v = lane + k * UT;
    if (v >= N) continue;
    if (out.dist) reinterpret_cast<D*>(out.dist)[size_t(uidx) * Sn + v] = dcur[k];
    if (out.nh) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        out.nh[(size_t(uidx) * W + w) * Sn + v] = ncur[k][w];
      }
    }
  }
  if (!hasPrefixes) return;

  // ---- fused RouteDb from LDS ---------------------------------------------
  ogs_prefix_table lp{};
  lp.max_prefixes = pt.max_prefixes;
  lp.adv_off = lAdvOff;
  lp.adv_node = lAdvNode;
  lp.adv_metrics = reinterpret_cast<const int32_t*>(lAdvMetrics);
  lp.adv_min_nh = lAdvMinNh;
  lp.pfx_flags = lPfxFlags;
  const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0,
                     (flags & OGS_F_V4_OVER_V6) != 0,
                     (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
  const uint32_t Sp = pt.max_prefixes;
  for (uint32_t p = lane; p < P; p += UT) {
    uint32_t meta, selBits;
    D metric;
    uint32_t mask[W];
    route_one<D, W>(lp, p, s, lflags, SplitView<D, W>{dist, nh}, cfg, meta,
                    metric, mask, selBits);
    const size_t o = size_t(uidx) * Sp + p;
    if (out.meta) out.meta[o] = meta;
    if (out.metric) reinterpret_cast<D*>(out.metric)[o] = metric;
    if (out.sel) out.sel[o] = selBits;
    if (out.mask) {
#pragma unroll
      for (int w = 0; w < W; ++w) out.mask[(size_t(uidx) * W + w) * Sp + p] = mask[w];
    }
  }
#ifdef OGS_STAMPS
  Scope::sync();
  if (lane == 0 && out.sel) {
    const uint64_t tEnd = __builtin_amdgcn_s_memtime();
    uint32_t* d = out.sel + size_t(uidx) * Sp;
    d[0] = uint32_t(tStaged - tStart);
    d[1] = uint32_t(tSpf - tStaged);
    d[2] = uint32_t(tEnd - tSpf);
    d[3] = rounds;
  }
#endif
}

template <typename D, int W, int UT, int NPL, int MAXD>
hipError_t launch_small(const ogs_graph& g, const ogs_prefix_table& pt,
                        int hasPrefixes, const ogs_unit* units, int nUnits,
                        uint32_t flags, const ogs_spf_out& out, uint32_t lds,
                        uint32_t maxA, hipStream_t stream) {
  constexpr int threads = UT == 64 ? 256 : UT;
  constexpr int upb = threads / UT;
  const int grid = (nUnits + upb - 1) / upb;
  const size_t bytes = size_t(lds) * upb;
  auto k = spf_route_small_kernel<D, W, UT, NPL, MAXD>;
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(k),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(threads), bytes, stream, g, pt,
                     hasPrefixes, units, nUnits, flags, out, lds, maxA);
  return hipGetLastError();
}

// Returns true (and launches) when the small path applies.
template <typename D, int W>
bool try_small(const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes,
               const ogs_unit* units, int nUnits, uint32_t flags,
               const ogs_spf_out& out, int maxDegree, uint32_t maxA,
               int unitWidth, hipStream_t stream, hipError_t* err) {
  if (g.max_nodes > 256 || maxDegree > 8 || maxDegree < 0) return false;
  const uint32_t P = hasPrefixes ? pt.max_prefixes : 0;
  const uint32_t A = hasPrefixes ? maxA : 0;
  const uint32_t lds = SmallLayout::make(g.max_nodes, g.max_edges, P, A, W,
                                         sizeof(D)).total;
  const int N = g.max_nodes;
  const int ut = unitWidth ? unitWidth : (N <= 128 ? 128 : 256);
  const bool d4 = maxDegree <= 4;
  // unit width x nodes per lane x register edges
#define OGS_SMALL(UT_, NPL_, MAXD_)                                           \
  *err = launch_small<D, W, UT_, NPL_, MAXD_>(g, pt, hasPrefixes, units,      \
                                              nUnits, flags, out, lds, A,     \
                                              stream);                        \
  return true;
  if (ut == 64 && uint64_t(lds) * 4 <= 160 * 1024) {
    if (N <= 64) { if (d4) { OGS_SMALL(64, 1, 4) } OGS_SMALL(64, 1, 8) }
    if (N <= 128) { if (d4) { OGS_SMALL(64, 2, 4) } OGS_SMALL(64, 2, 8) }
    if (d4) { OGS_SMALL(64, 4, 4) }
    OGS_SMALL(64, 4, 8)
  }
  if (lds > 160 * 1024) return false;
  if (ut <= 128 && N <= 128) { if (d4) { OGS_SMALL(128, 1, 4) } OGS_SMALL(128, 1, 8) }
  if (d4) { OGS_SMALL(256, 1, 4) }
  OGS_SMALL(256, 1, 8)
#undef OGS_SMALL
}

#define OGS_INST(D_, W_)                                                      \
  template bool try_small<D_, W_>(const ogs_graph&, const ogs_prefix_table&,  \
                                  int, const ogs_unit*, int, uint32_t,        \
                                  const ogs_spf_out&, int, uint32_t, int,     \
                                  hipStream_t, hipError_t*);
OGS_INST(uint32_t, 1)
OGS_INST(uint64_t, 1)
#undef OGS_INST

}  // namespace ogs
