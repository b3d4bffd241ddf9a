// ksp.hip — edge-disjoint k-th shortest paths (KSP2) for gfx950.
//
// Replaces LinkState::getKthPaths + traceOnePath (LinkState.cpp:226-247,
// 674-703). One work unit = (topology, source, destination, ignore-mask):
//   1. SPF over the links NOT in the unit's linksToIgnore mask (the masked
//      second pass; empty mask = the k = 1 SPF), wave/workgroup-parallel in
//      LDS (spf_core.h);
//   2. the reference's greedy trace, run by lane 0: repeatedly walk from the
//      destination back to the source over NodeSpfResult::pathLinks in the
//      reference order, marking every link visited (never unmarked), until
//      no path remains. pathLinks(v) = tight links from relaxing
//      predecessors in settlement order; with metrics >= 1 settlement order
//      is (dist, name) (LinkState.h:618-626) = (dist, id), and a
//      predecessor's parallel links follow its CSR row (canonical link
//      order; the reference uses folly-hash order there, parity unpinned,
//      see DESIGN.md). The recursion is an explicit stack in LDS; each frame
//      resumes its scan from the last (dist, pred, slot) key it tried.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "openr_gpu.h"
#include "spf_core.h"
#include "engine.h"

namespace ogs {

constexpr uint32_t kExactRowK = 512;  // exact-order rows staged in LDS (longer: HBM)

// 8 B per recursion level: the last edge (node -> pred) chosen at this frame
// is both the path edge once the recursion below it succeeds and the resume
// key (dist[pred], pred, rslot) of the next choice; ~0u = nothing chosen yet
struct Frame {
  uint32_t node;
  uint32_t edge;
};

template <typename D>
__device__ bool key_less(D da, uint32_t ua, uint32_t sa, D db, uint32_t ub,
                         uint32_t sb) {
  if (da != db) return da < db;
  if (ua != ub) return ua < ub;
  return sa < sb;
}

// Every edge-disjoint path of one getKthPaths(src, dest, k) call (lane 0):
// traceOnePath repeated with one visited-link set until it fails. Writes the
// paths of output row `row`; also sets each emitted path's links in
// `pathMask` (the next k's linksToIgnore) when non-NULL. Returns the
// path_count word (bit 31 = output capacity exceeded).
template <typename D, bool MASKED>
__device__ uint32_t trace_paths(const UnitCsr& csr, const D* dist, uint32_t s,
                                uint32_t t, uint32_t* visited, Frame* stack,
                                const uint32_t* ignore, const ogs_path_out& out,
                                size_t row, uint32_t* pathMask) {
  constexpr D kInf = DistInf<D>::value;
  uint32_t* pathLen = out.path_len + row * out.max_paths;
  uint32_t* pathEdges = out.path_edges + row * out.max_edges;
  uint32_t nPaths = 0, nEdges = 0, status = 0;
  const bool reachable = (s != t) && dist[t] != kInf;
  while (reachable) {
    // one traceOnePath(src, dest) call
    int sp = 0;
    stack[0] = Frame{t, 0xFFFFFFFFu};
    bool found = false;
    while (sp >= 0) {
      Frame& f = stack[sp];
      const uint32_t v = f.node;
      const D dv = dist[v];
      // next unvisited pathLink of v after the resume key
      D bd = kInf;
      uint32_t bu = 0xFFFFFFFFu, bs = 0xFFFFFFFFu, be = 0xFFFFFFFFu;
      const bool fresh = f.edge == 0xFFFFFFFFu;
      uint32_t lastU = 0u, lastSlot = 0u;
      if (!fresh) {
        const uint32_t llo = static_cast<uint32_t>(csr.edg[f.edge]);
        lastU = edge_dst(llo);
        lastSlot = csr_rslot(csr, f.edge, llo);
      }
      const D ld = fresh ? D(0) : dist[lastU];
      // the row's edges 8 at a time: the loads of a batch are independent
      // (HBM/L2 latency once per batch, not once per edge)
      const uint32_t rEnd = csr.rowp[v + 1];
      for (uint32_t eb = csr.rowp[v]; eb < rEnd; eb += 8) {
        uint64_t xs[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
          xs[k] = eb + k < rEnd ? csr.edg[eb + k] : uint64_t(OGS_EDGE_DOWN);
        }
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
          const uint32_t e = eb + k;
          const uint64_t ed = xs[k];
          const uint32_t lo = static_cast<uint32_t>(ed);
          if (lo & OGS_EDGE_DOWN) continue;
          const uint32_t u = edge_dst(lo);
          if ((lo & OGS_EDGE_DST_OVERLOADED) && u != s) continue;
          if constexpr (MASKED) {
            const uint32_t l = link_id(csr, e, lo);
            if ((ignore[l >> 5] >> (l & 31u)) & 1u) continue;
          }
          const D du = dist[u];
          if (du == kInf || du + static_cast<D>(ed >> 32) != dv) continue;
          const uint32_t slot = csr_rslot(csr, e, lo);
          if (!fresh && !key_less<D>(ld, lastU, lastSlot, du, u, slot)) continue;
          if (key_less<D>(du, u, slot, bd, bu, bs)) {
            bd = du;
            bu = u;
            bs = slot;
            be = e;
          }
        }
      }
      if (be == 0xFFFFFFFFu) {  // exhausted: this recursion level fails
        --sp;
        continue;
      }
      f.edge = be;  // resume key (and the path edge if the recursion succeeds)
      const uint32_t l = link_id(csr, be, static_cast<uint32_t>(csr.edg[be]));
      if ((visited[l >> 5] >> (l & 31u)) & 1u) continue;  // already used
      visited[l >> 5] |= 1u << (l & 31u);
      if (bu == s) {
        found = true;
        break;
      }
      ++sp;
      stack[sp] = Frame{bu, 0xFFFFFFFFu};
    }
    if (!found) break;
    // path src -> dest = chosen edges from the top frame down to frame 0
    if (nPaths >= out.max_paths || nEdges + uint32_t(sp + 1) > out.max_edges) {
      status = 1;  // output capacity exceeded
      break;
    }
    for (int i = sp; i >= 0; --i) {
      const uint32_t e = stack[i].edge;
      pathEdges[nEdges++] = e - csr.eBase;
      if (pathMask) {
        const uint32_t l = link_id(csr, e, static_cast<uint32_t>(csr.edg[e]));
        pathMask[l >> 5] |= 1u << (l & 31u);
      }
    }
    pathLen[nPaths++] = uint32_t(sp + 1);
  }
  return nPaths | (status << 31);
}

// trace_paths by one whole wavefront (32-bit distances): the same greedy
// DFS with the same choices, but each step's scan of the node's row is
// spread over the lanes (lane j tests edge j of a 64-edge window) and the
// next pathLink is a wave-wide min of the packed key (dist, pred, slot) --
// one LDS round trip and a 6-step reduction per step instead of a serial
// walk of the row by lane 0. Every lane runs the uniform control flow and
// holds the same frame state; LDS state (stack, visited, masks, outputs) is
// written by lane 0 and made visible to the wave before it is read.
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor(static_cast<uint32_t>(x), o);
    const uint32_t hi = __shfl_xor(static_cast<uint32_t>(x >> 32), o);
    const uint64_t y = (uint64_t(hi) << 32) | lo;
    x = y < x ? y : x;
  }
  return x;
}

__device__ __forceinline__ void lane_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool MASKED>
__device__ uint32_t trace_paths_wave(const UnitCsr& csr, const uint32_t* dist, uint32_t s,
                                     uint32_t t, uint32_t* visited, Frame* stack,
                                     const uint32_t* ignore, const ogs_path_out& out,
                                     size_t row, uint32_t* pathMask, int lane) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  constexpr uint64_t kNone = ~0ull;
  // packed key: dist | reverse edge index (rowp[pred] + slot: rows are
  // contiguous in pred order, so this is the lexicographic (dist, pred,
  // slot) order of key_less for rows of any length)
  auto pack = [&](uint32_t d, uint32_t u, uint32_t slot) {
    return (uint64_t(d) << 32) | (csr.rowp[u] + slot);
  };
  uint32_t* pathLen = out.path_len + row * out.max_paths;
  uint32_t* pathEdges = out.path_edges + row * out.max_edges;
  uint32_t nPaths = 0, nEdges = 0, status = 0;
  const bool reachable = (s != t) && dist[t] != kInf;
  while (reachable) {
    int sp = 0;
    if (lane == 0) stack[0] = Frame{t, 0xFFFFFFFFu};
    lane_sync();
    bool found = false;
    while (sp >= 0) {
      const Frame f = stack[sp];
      const uint32_t v = f.node;
      const uint32_t dv = dist[v];
      const bool fresh = f.edge == 0xFFFFFFFFu;
      uint64_t lastKey = 0;
      if (!fresh) {
        const uint32_t llo = static_cast<uint32_t>(csr.edg[f.edge]);
        lastKey = pack(dist[edge_dst(llo)], edge_dst(llo), csr_rslot(csr, f.edge, llo));
      }
      uint64_t best = kNone;
      uint32_t be = 0xFFFFFFFFu, blo = 0u;
      const uint32_t rEnd = csr.rowp[v + 1];
      for (uint32_t eb = csr.rowp[v]; eb < rEnd; eb += 64) {
        const uint32_t e = eb + uint32_t(lane);
        uint64_t key = kNone;
        uint32_t lo = 0u;
        if (e < rEnd) {
          const uint64_t ed = csr.edg[e];
          lo = static_cast<uint32_t>(ed);
          const uint32_t u = edge_dst(lo);
          bool ok = !(lo & OGS_EDGE_DOWN) && !((lo & OGS_EDGE_DST_OVERLOADED) && u != s);
          if constexpr (MASKED) {
            if (ok) {
              const uint32_t l = link_id(csr, e, lo);
              ok = !((ignore[l >> 5] >> (l & 31u)) & 1u);
            }
          }
          if (ok) {
            const uint32_t du = dist[u];
            if (du != kInf && du + static_cast<uint32_t>(ed >> 32) == dv) {
              const uint64_t k = pack(du, u, csr_rslot(csr, e, lo));
              if (fresh || k > lastKey) key = k;
            }
          }
        }
        // the window's best candidate: with one candidate lane (a unique
        // tight predecessor, the common case) its key directly, else the
        // wave-wide min; the winner's edge word comes back through
        // v_readlane (uniform lane), not a reload of the CSR
        const uint64_t cand = __ballot(key != kNone);
        if (cand == 0ull) continue;  // uniform
        int wl;
        uint64_t m;
        if ((cand & (cand - 1ull)) == 0ull) {
          wl = int(__builtin_ctzll(cand));
          m = (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(key >> 32), wl))) << 32) |
              uint32_t(__builtin_amdgcn_readlane(int(uint32_t(key)), wl));
        } else {
          m = wave_min_u64(key);
          wl = int(__builtin_ctzll(__ballot(key == m)));
        }
        if (m < best) {
          best = m;
          be = uint32_t(__builtin_amdgcn_readlane(int(e), wl));
          blo = uint32_t(__builtin_amdgcn_readlane(int(lo), wl));
        }
      }
      if (best == kNone) {  // exhausted: this recursion level fails
        --sp;
        continue;
      }
      const uint32_t bu = edge_dst(blo);  // the chosen pred
      if (lane == 0) stack[sp].edge = be;  // resume key (+ path edge on success)
      const uint32_t l = link_id(csr, be, blo);
      const bool seen = (visited[l >> 5] >> (l & 31u)) & 1u;
      lane_sync();
      if (seen) continue;  // already used
      if (lane == 0) visited[l >> 5] |= 1u << (l & 31u);
      if (bu == s) {
        lane_sync();
        found = true;
        break;
      }
      ++sp;
      if (lane == 0) stack[sp] = Frame{bu, 0xFFFFFFFFu};
      lane_sync();
    }
    if (!found) break;
    // path src -> dest = chosen edges from the top frame down to frame 0
    if (nPaths >= out.max_paths || nEdges + uint32_t(sp + 1) > out.max_edges) {
      status = 1;  // output capacity exceeded
      break;
    }
    for (int i = sp; i >= 0; --i) {
      const uint32_t e = stack[i].edge;
      if (lane == 0) {
        pathEdges[nEdges] = e - csr.eBase;
        if (pathMask) {
          const uint32_t l = link_id(csr, e, static_cast<uint32_t>(csr.edg[e]));
          pathMask[l >> 5] |= 1u << (l & 31u);
        }
      }
      ++nEdges;
    }
    if (lane == 0) pathLen[nPaths] = uint32_t(sp + 1);
    ++nPaths;
    lane_sync();
  }
  return nPaths | (status << 31);
}

// "ksp_wave_trace" option: 1 (default) the traces of 32-bit-distance units
// run on a whole wavefront (trace_paths_wave), 0 on lane 0 (A/B)
// EngineOptions::kspWaveTrace (engine.h), default 1
// (An early stop of the k = 2 SPF once every distance lowered in a round
// exceeds the destination's saved nothing on C5 -- 0.49 vs 0.49 ms of KSP2
// kernels per job, profiles/r03_c5_ksp_stop_ab.log: the launch lasts as
// long as its farthest destinations -- and was removed in round 4.)

template <typename D, int UT, bool STAGE, bool MASKED>
__global__ __launch_bounds__(kBlock) void ksp_kernel(
    ogs_graph g, const ogs_path_unit* __restrict__ units, int nUnits,
    const uint32_t* __restrict__ masks, uint32_t maskWords,
    ogs_path_out out, uint32_t ldsPerUnit, int waveTrace) {
  constexpr int kUnitsPerBlock = kBlock / UT;
  const int uib = threadIdx.x / UT;
  const int lane = threadIdx.x % UT;
  const int uidx = blockIdx.x * kUnitsPerBlock + uib;
  if (uidx >= nUnits) return;

  const ogs_path_unit unit = units[uidx];
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const uint32_t s = unit.src, t = unit.dest;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint32_t E = gRow[N] - e0;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* base = smem + uib * ldsPerUnit;
  D* dist = reinterpret_cast<D*>(base);
  uint32_t off = align16(uint64_t(N) * sizeof(D));
  uint32_t* visited = reinterpret_cast<uint32_t*>(base + off);
  off += align16(uint64_t((E + 31) / 32) * 4);
  Frame* stack = reinterpret_cast<Frame*>(base + off);
  off += align16(uint64_t(N) * sizeof(Frame));
  UnitCsr csr;
  if constexpr (STAGE) {
    uint32_t* lrow = reinterpret_cast<uint32_t*>(base + off);
    off += align16(uint64_t(N + 1) * 4);
    uint64_t* ledg = reinterpret_cast<uint64_t*>(base + off);
    for (uint32_t i = lane; i <= N; i += UT) lrow[i] = gRow[i] - e0;
    for (uint32_t i = lane; i < E; i += UT) ledg[i] = g.edges[e0 + i];
    csr = UnitCsr{lrow, ledg, 0u, g.rslot_ext ? g.rslot_ext + e0 : nullptr};
  } else {
    csr = UnitCsr{gRow, g.edges, e0, g.rslot_ext ? g.rslot_ext + e0 : nullptr};
  }
  for (uint32_t i = lane; i < (E + 31) / 32; i += UT) visited[i] = 0u;
  const uint32_t* ignore =
      MASKED ? masks + size_t(uidx) * maskWords : nullptr;
  spf_fixpoint<D, 1, UT, false, MASKED>(N, s, lane, csr, false, dist, nullptr,
                                        ignore);

  if constexpr (sizeof(D) == 4) {
    if (waveTrace) {
      if (lane >= 64) return;  // wave 0 of a workgroup unit traces
      const uint32_t c = trace_paths_wave<MASKED>(csr, dist, s, t, visited, stack, ignore,
                                                  out, uidx, nullptr, lane);
      if (lane == 0) out.path_count[uidx] = c;
      return;
    }
  }
  if (lane != 0) return;
  out.path_count[uidx] = trace_paths<D, MASKED>(
      csr, dist, s, t, visited, stack, ignore, out, uidx, nullptr);
}

template <typename D, int UT, bool STAGE, bool MASKED>
hipError_t ksp_launch(const ogs_graph& g, const ogs_path_unit* units,
                      int nUnits, const uint32_t* masks, uint32_t maskWords,
                      const ogs_path_out& out, uint32_t lds,
                      hipStream_t stream) {
  constexpr int upb = kBlock / UT;
  const int grid = (nUnits + upb - 1) / upb;
  const size_t bytes = size_t(lds) * upb;
  auto k = ksp_kernel<D, UT, STAGE, MASKED>;
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(k),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), bytes, stream, g, units,
                     nUnits, masks, maskWords, out, lds, opts().kspWaveTrace);
  return hipGetLastError();
}

// ---- HBM-state KSP: units past the LDS budget, and the exact order -------
// The LDS paths above hold a unit's distances, link bitsets and trace stack
// in LDS (<= 160 kB per unit). Past that -- areas of tens of thousands of
// nodes (LinkState::getKthPaths has no size bound) -- and
// for zero / negative link metrics, where the reference's settle order
// decides pathLinks, the unit's state lives in HBM scratch:
//  * fixpoint domain (metrics >= 1): one 1024-thread workgroup per unit,
//    frontier rounds as in spf_global.hip (atomics in L2, agent-scope
//    fences between rounds); pathLinks(v) order = (dist, id) of the
//    predecessor, then its CSR row;
//  * exact domain (OGS_F_EXACT_ORDER): one wavefront per unit replays the
//    DijkstraQ extraction order (as spf_exact.hip) and records each node's
//    settle rank. runSpf (LinkState.cpp:720-820) appends link (u, v) to
//    pathLinks(v) when u is settled before v, relaxes and u's metric + w <=
//    v's current metric, and clears the list on a strict improvement; the
//    entries that survive are exactly the links with rank(u) < rank(v), u
//    relaxing and d(u) + w == d(v) in wrapping u64 arithmetic (an entry
//    added before the last improvement has d(u) + w > d(v)), in (rank(u),
//    u's row) order.
// Both trace on one wavefront with a two-word key (trace_paths_wave's scan).
constexpr int kKspHbmBlock = 1024;
constexpr uint32_t kRankNew = 0xFFFFFFFFu;   // never inserted
constexpr uint32_t kRankOpen = 0xFFFFFFFEu;  // in the open list
// EngineOptions::kspHbm (engine.h), default 0  // "ksp_hbm" option: 1 = every KSP unit on the HBM path

hipError_t workspace(size_t bytes, hipStream_t stream, void** out);

// A unit's workgroup runs on one CU: its HBM state stays in that XCD's L2
// for the whole launch. Rounds end with every wave's stores drained and a
// barrier; state written in this launch is read back through sc1 (L2-served,
// L1-bypassing) loads -- the L1 may hold lines that L2 atomics have since
// changed (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ void hbm_block_sync() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

template <typename T>
__device__ __forceinline__ T ld_l2(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void hbm_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// LinkStateMetric of an edge in the exact domain: the stored i32 sign-
// extended to u64 (LinkState.cpp:77-78); sums wrap like the reference's.
__device__ __forceinline__ uint64_t ksp_exact_weight(uint64_t x) {
  return static_cast<uint64_t>(static_cast<int64_t>(static_cast<int32_t>(
      static_cast<uint32_t>(x >> 32))));
}

// Fixpoint-domain distances with the unit's state in HBM (whole workgroup).
template <typename D, bool MASKED>
__device__ void frontier_dist_hbm(uint32_t N, uint32_t s, const UnitCsr& c,
                                  const uint8_t* __restrict__ nflags, D* dist,
                                  uint32_t* stamp, uint32_t* q0, uint32_t* q1,
                                  uint32_t* qcnt, const uint32_t* ignore) {
  constexpr D kInf = DistInf<D>::value;
  const int tid = threadIdx.x;
  for (uint32_t v = tid; v < N; v += kKspHbmBlock) {
    dist[v] = (v == s) ? D(0) : kInf;
    stamp[v] = 0u;
  }
  if (tid == 0) {
    q1[0] = s;  // round r's list: buffer r & 1, count slot r % 3
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  hbm_block_sync();
  uint32_t n = 1;
  for (uint32_t r = 1; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint32_t* cur = (r & 1) ? q1 : q0;
    uint32_t* nxt = (r & 1) ? q0 : q1;
    for (uint32_t i = tid; i < n; i += kKspHbmBlock) {
      const uint32_t v = ld_l2(cur + i);
      if (v != s && (nflags[v] & OGS_NODE_OVERLOADED)) continue;  // 741-752
      const D dv = ld_l2(dist + v);
      const uint32_t rEnd = c.rowp[v + 1];
      for (uint32_t e = c.rowp[v]; e < rEnd; ++e) {
        const uint64_t ed = c.edg[e];
        const uint32_t lo = static_cast<uint32_t>(ed);
        if (lo & OGS_EDGE_DOWN) continue;
        if constexpr (MASKED) {
          const uint32_t l = link_id(c, e, lo);
          if ((ignore[l >> 5] >> (l & 31u)) & 1u) continue;
        }
        const uint32_t t = edge_dst(lo);
        const D cand = dv + static_cast<D>(static_cast<uint32_t>(ed >> 32));
        if (cand < ld_l2(dist + t) && cand < atomicMin(&dist[t], cand)) {
          if (atomicMax(&stamp[t], r + 1) < r + 1) {
            nxt[atomicAdd(&qcnt[(r + 1) % 3], 1u)] = t;
          }
        }
      }
    }
    hbm_block_sync();
    n = qcnt[(r + 1) % 3];
    __syncthreads();  // every thread has read the count before it is reset
  }
}

// Exact-domain distances + settle ranks (one wavefront; HBM state). The
// unit's rows are staged in LDS one settled node at a time (degree <=
// OGS_MAX_DEGREE); parallel links to one neighbour collapse to their minimum
// first (the sequential loop reaches the same key).
template <bool MASKED>
__device__ void exact_dist_hbm(uint32_t N, uint32_t s, const UnitCsr& c,
                               const uint8_t* __restrict__ nflags, uint64_t* key,
                               uint32_t* rank, uint32_t* open, const uint32_t* ignore,
                               uint32_t* rowT, uint64_t* rowC, uint8_t* rowV, int lane) {
  constexpr uint64_t kInf = ~0ull;
  for (uint32_t v = lane; v < N; v += 64) {
    key[v] = kInf;
    rank[v] = kRankNew;
  }
  hbm_wave_sync();
  if (lane == 0) {
    key[s] = 0;
    rank[s] = kRankOpen;
    open[0] = s;
  }
  hbm_wave_sync();
  uint32_t nOpen = 1, step = 0;
  while (nOpen) {
    // extractMin: smallest (key, id) over the open list (LinkState.h:618-626)
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
    hbm_wave_sync();
    if (lane == 0) {
      open[bi] = open[nOpen - 1];
      rank[u] = step;
    }
    --nOpen;
    ++step;
    hbm_wave_sync();
    if (u != s && (nflags[u] & OGS_NODE_OVERLOADED)) continue;  // 741-752
    const uint32_t b = c.rowp[u], m = c.rowp[u + 1] - b;
    for (uint32_t j = lane; j < m; j += 64) {
      const uint64_t x = c.edg[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      const uint32_t t = edge_dst(lo);
      bool ok = !(lo & OGS_EDGE_DOWN) && rank[t] >= kRankOpen;  // 762-763
      if constexpr (MASKED) {
        if (ok) {
          const uint32_t l = link_id(c, b + j, lo);
          ok = !((ignore[l >> 5] >> (l & 31u)) & 1u);
        }
      }
      rowT[j] = t;
      rowC[j] = du + ksp_exact_weight(x);  // wraps like the reference's u64
      rowV[j] = ok;
    }
    hbm_wave_sync();
    for (uint32_t j0 = 0; j0 < m; j0 += 64) {  // wave-uniform trip count
      const uint32_t j = j0 + lane;
      bool append = false;
      uint32_t t = 0;
      if (j < m && rowV[j]) {
        t = rowT[j];
        uint64_t cc = rowC[j];
        bool rep = true;  // lowest valid slot of u's row leading to t
        for (uint32_t k = 0; k < m; ++k) {
          if (k == j || !rowV[k] || rowT[k] != t) continue;
          if (k < j) rep = false;
          if (rowC[k] < cc) cc = rowC[k];
        }
        if (rep) {
          if (rank[t] == kRankNew) {  // insertNode(t, c)
            key[t] = cc;
            rank[t] = kRankOpen;
            append = true;
          } else if (key[t] > cc) {  // strictly better (791-795)
            key[t] = cc;
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
    hbm_wave_sync();
  }
}

// The greedy trace (trace_paths_wave) over HBM state with a two-word key:
// fixpoint (dist(u), rowp[u] + slot), exact (rank(u), slot).
template <typename D, bool EXACT, bool MASKED>
__device__ uint32_t trace_paths_hbm(const UnitCsr& csr, const D* dist, const uint32_t* rank,
                                    uint32_t s, uint32_t t, uint32_t* visited, Frame* stack,
                                    const uint32_t* ignore, const ogs_path_out& out,
                                    size_t row, uint32_t* pathMask, int lane) {
  constexpr D kInf = DistInf<D>::value;
  constexpr uint64_t kNoneHi = ~0ull;
  constexpr uint32_t kNoneLo = 0xFFFFFFFFu;
  auto less = [](uint64_t ah, uint32_t al, uint64_t bh, uint32_t bl) {
    return ah < bh || (ah == bh && al < bl);
  };
  auto keyOf = [&](uint32_t u, uint32_t slot, uint64_t& hi, uint32_t& lo) {
    if constexpr (EXACT) {
      hi = rank[u];
      lo = slot;
    } else {
      hi = static_cast<uint64_t>(ld_l2(dist + u));
      lo = csr.rowp[u] + slot;  // (u, slot) order for rows of any length
    }
  };
  uint32_t* pathLen = out.path_len + row * out.max_paths;
  uint32_t* pathEdges = out.path_edges + row * out.max_edges;
  uint32_t nPaths = 0, nEdges = 0, status = 0;
  const bool reachable = (s != t) && (EXACT ? rank[t] < kRankOpen : ld_l2(dist + t) != kInf);
  while (reachable) {
    int sp = 0;
    if (lane == 0) stack[0] = Frame{t, 0xFFFFFFFFu};
    hbm_wave_sync();
    bool found = false;
    while (sp >= 0) {
      const Frame f = stack[sp];
      const uint32_t v = f.node;
      const D dv = ld_l2(dist + v);
      const uint32_t rv = EXACT ? rank[v] : 0u;
      const bool fresh = f.edge == 0xFFFFFFFFu;
      uint64_t lastHi = 0;
      uint32_t lastLo = 0;
      if (!fresh) {
        const uint32_t llo = static_cast<uint32_t>(csr.edg[f.edge]);
        keyOf(edge_dst(llo), csr_rslot(csr, f.edge, llo), lastHi, lastLo);
      }
      uint64_t bHi = kNoneHi;
      uint32_t bLo = kNoneLo, be = 0xFFFFFFFFu;
      const uint32_t rEnd = csr.rowp[v + 1];
      for (uint32_t eb = csr.rowp[v]; eb < rEnd; eb += 64) {
        const uint32_t e = eb + uint32_t(lane);
        uint64_t kh = kNoneHi;
        uint32_t kl = kNoneLo;
        if (e < rEnd) {
          const uint64_t ed = csr.edg[e];
          const uint32_t lo = static_cast<uint32_t>(ed);
          const uint32_t u = edge_dst(lo);
          bool ok = !(lo & OGS_EDGE_DOWN) && !((lo & OGS_EDGE_DST_OVERLOADED) && u != s);
          if constexpr (MASKED) {
            if (ok) {
              const uint32_t l = link_id(csr, e, lo);
              ok = !((ignore[l >> 5] >> (l & 31u)) & 1u);
            }
          }
          if (ok) {
            const D du = ld_l2(dist + u);
            bool tight;
            if constexpr (EXACT) {
              tight = rank[u] < rv && du + ksp_exact_weight(ed) == dv;
            } else {
              tight = du != kInf && du + static_cast<D>(static_cast<uint32_t>(ed >> 32)) == dv;
            }
            if (tight) {
              uint64_t h;
              uint32_t l;
              keyOf(u, csr_rslot(csr, e, lo), h, l);
              if (fresh || less(lastHi, lastLo, h, l)) {
                kh = h;
                kl = l;
              }
            }
          }
        }
        uint64_t mh = kh;
        uint32_t ml = kl;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const uint32_t a = __shfl_xor(static_cast<uint32_t>(mh), o);
          const uint32_t b = __shfl_xor(static_cast<uint32_t>(mh >> 32), o);
          const uint32_t c = __shfl_xor(ml, o);
          const uint64_t oh = (uint64_t(b) << 32) | a;
          if (less(oh, c, mh, ml)) {
            mh = oh;
            ml = c;
          }
        }
        if (less(mh, ml, bHi, bLo)) {
          const uint64_t who = __ballot(kh == mh && kl == ml);
          bHi = mh;
          bLo = ml;
          be = __shfl(e, int(__builtin_ctzll(who)));
        }
      }
      if (be == 0xFFFFFFFFu) {  // exhausted: this recursion level fails
        --sp;
        continue;
      }
      const uint32_t blo = static_cast<uint32_t>(csr.edg[be]);
      const uint32_t bu = edge_dst(blo);
      if (lane == 0) stack[sp].edge = be;  // resume key (+ path edge on success)
      const uint32_t l = link_id(csr, be, blo);
      const bool seen = (visited[l >> 5] >> (l & 31u)) & 1u;
      hbm_wave_sync();
      if (seen) continue;  // already used
      if (lane == 0) visited[l >> 5] |= 1u << (l & 31u);
      if (bu == s) {
        hbm_wave_sync();
        found = true;
        break;
      }
      ++sp;
      if (lane == 0) stack[sp] = Frame{bu, 0xFFFFFFFFu};
      hbm_wave_sync();
    }
    if (!found) break;
    if (nPaths >= out.max_paths || nEdges + uint32_t(sp + 1) > out.max_edges) {
      status = 1;  // output capacity exceeded
      break;
    }
    for (int i = sp; i >= 0; --i) {
      const uint32_t e = stack[i].edge;
      if (lane == 0) {
        pathEdges[nEdges] = e - csr.eBase;
        if (pathMask) {
          const uint32_t l = link_id(csr, e, static_cast<uint32_t>(csr.edg[e]));
          pathMask[l >> 5] |= 1u << (l & 31u);
        }
      }
      ++nEdges;
    }
    if (lane == 0) pathLen[nPaths] = uint32_t(sp + 1);
    ++nPaths;
    hbm_wave_sync();
  }
  return nPaths | (status << 31);
}

// Per-unit HBM scratch: dist | stamp or rank | list 0 (open list) | list 1 |
// visited | mask | stack, each 256-B aligned.
struct KspHbmLayout {
  size_t dist, aux, q0, q1, visited, mask, stack, rowT, rowC, rowV, total;
  // rowDeg: rows staged in HBM for the exact replay (rows past kExactRowK)
  __host__ __device__ static KspHbmLayout make(uint64_t N, uint64_t E, uint64_t dsize,
                                               uint64_t rowDeg = 0) {
    auto r = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
    const uint64_t lw = (E + 31) / 32 + 1;
    KspHbmLayout L;
    size_t o = 0;
    L.dist = o;
    o += r(N * dsize);
    L.aux = o;
    o += r(N * 4);
    L.q0 = o;
    o += r(N * 4);
    L.q1 = o;
    o += r(N * 4);
    L.visited = o;
    o += r(lw * 4);
    L.mask = o;
    o += r(lw * 4);
    L.stack = o;
    o += r(N * sizeof(Frame));
    L.rowT = o;
    o += r(rowDeg * 4);
    L.rowC = o;
    o += r(rowDeg * 8);
    L.rowV = o;
    o += r(rowDeg);
    L.total = o;
    return L;
  }
};

// TWO: the KSP2 batch (k = 1 into o1, k = 2 with the k = 1 links ignored
// into o2; units carry their source index as in ksp2_kernel). Otherwise one
// getKthPaths call per unit (masks = its linksToIgnore when MASKED) into o1.
template <typename D, bool EXACT, bool TWO, bool MASKED>
__global__ __launch_bounds__(EXACT ? 64 : kKspHbmBlock) void ksp_hbm_kernel(
    ogs_graph g, const ogs_unit* __restrict__ sources, int nSources,
    const ogs_path_unit* __restrict__ units, uint32_t uBase,
    const uint32_t* __restrict__ masks, uint32_t maskWords, ogs_path_out o1,
    ogs_path_out o2, char* __restrict__ scratch) {
  static_assert(!EXACT || sizeof(D) == 8, "exact order: 64-bit distances");
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t uidx = uBase + blockIdx.x;
  const ogs_path_unit unit = units[uidx];
  if constexpr (TWO) {
    const uint32_t slot = unit.reserved;
    if (slot >= uint32_t(nSources) || sources[slot].topo != unit.topo ||
        sources[slot].src != unit.src) {
      if (tid == 0) {  // malformed unit: reported, never traced
        o1.path_count[uidx] = 0xC0000000u;
        o2.path_count[uidx] = 0xC0000000u;
      }
      return;
    }
  }
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint32_t E = gRow[N] - e0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const UnitCsr csr{gRow, g.edges, e0, g.rslot_ext ? g.rslot_ext + e0 : nullptr};
  const uint32_t s = unit.src, t = unit.dest;
  const bool hbmRows = EXACT && uint32_t(g.max_degree) > kExactRowK;
  const KspHbmLayout L = KspHbmLayout::make(uint32_t(g.max_nodes), uint32_t(g.max_edges),
                                            sizeof(D), hbmRows ? uint32_t(g.max_degree) : 0u);
  char* base = scratch + size_t(blockIdx.x) * L.total;
  D* dist = reinterpret_cast<D*>(base + L.dist);
  uint32_t* aux = reinterpret_cast<uint32_t*>(base + L.aux);
  uint32_t* q0 = reinterpret_cast<uint32_t*>(base + L.q0);
  uint32_t* q1 = reinterpret_cast<uint32_t*>(base + L.q1);
  uint32_t* visited = reinterpret_cast<uint32_t*>(base + L.visited);
  uint32_t* mask = reinterpret_cast<uint32_t*>(base + L.mask);
  Frame* stack = reinterpret_cast<Frame*>(base + L.stack);
  __shared__ uint32_t qcnt[3];
  __shared__ uint32_t bcast;
  __shared__ uint32_t rowT[EXACT ? kExactRowK : 1];
  __shared__ uint64_t rowC[EXACT ? kExactRowK : 1];
  __shared__ uint8_t rowV[EXACT ? kExactRowK : 1];
  const uint32_t linkWords = (E + 31) / 32;
  const int nt = EXACT ? 64 : kKspHbmBlock;
  for (uint32_t i = tid; i < linkWords; i += nt) {
    visited[i] = 0u;
    if (TWO) mask[i] = 0u;
  }
  const uint32_t* ign = MASKED ? masks + size_t(uidx) * maskWords : nullptr;
  auto spf = [&](const uint32_t* ignore, auto maskedTag) {
    constexpr bool M = decltype(maskedTag)::value;
    if constexpr (EXACT) {
      // rows of 512+ edges are staged in the unit's HBM scratch
      exact_dist_hbm<M>(N, s, csr, nflags, reinterpret_cast<uint64_t*>(dist), aux, q0, ignore,
                        hbmRows ? reinterpret_cast<uint32_t*>(base + L.rowT) : rowT,
                        hbmRows ? reinterpret_cast<uint64_t*>(base + L.rowC) : rowC,
                        hbmRows ? reinterpret_cast<uint8_t*>(base + L.rowV) : rowV, lane);
    } else {
      frontier_dist_hbm<D, M>(N, s, csr, nflags, dist, aux, q0, q1, qcnt, ignore);
    }
    hbm_block_sync();
  };
  spf(ign, std::integral_constant<bool, MASKED>{});
  uint32_t c1 = 0;
  if (tid < 64) {
    c1 = trace_paths_hbm<D, EXACT, MASKED>(csr, dist, aux, s, t, visited, stack, ign, o1,
                                           uidx, TWO ? mask : nullptr, lane);
    if (lane == 0) o1.path_count[uidx] = c1;
  }
  if constexpr (TWO) {
    if (tid == 0) bcast = c1;
    hbm_block_sync();
    c1 = bcast;
    // k = 1 found nothing: linksToIgnore is empty, k = 2 finds nothing
    // either; a k = 1 overflow leaves the mask incomplete (reported)
    if (c1 == 0u || (c1 >> 31)) {
      if (tid == 0) o2.path_count[uidx] = c1 & 0x80000000u;
      return;
    }
    for (uint32_t i = tid; i < linkWords; i += nt) visited[i] = 0u;
    hbm_block_sync();
    spf(mask, std::integral_constant<bool, true>{});
    if (tid < 64) {
      const uint32_t c2 = trace_paths_hbm<D, EXACT, true>(csr, dist, aux, s, t, visited, stack,
                                                          mask, o2, uidx, nullptr, lane);
      if (lane == 0) o2.path_count[uidx] = c2;
    }
  }
}

// Launches the HBM-state path over n units in chunks whose scratch stays
// below kKspHbmScratch.
template <typename D, bool EXACT, bool TWO, bool MASKED>
hipError_t launch_ksp_hbm(const ogs_graph& g, const ogs_unit* sources, int nSources,
                          const ogs_path_unit* units, int nUnits, const uint32_t* masks,
                          uint32_t maskWords, const ogs_path_out& o1, const ogs_path_out& o2,
                          hipStream_t stream) {
  constexpr size_t kKspHbmScratch = size_t(4) << 30;
  const bool hbmRows = EXACT && uint32_t(g.max_degree) > kExactRowK;
  const size_t per = KspHbmLayout::make(uint32_t(g.max_nodes), uint32_t(g.max_edges),
                                        sizeof(D), hbmRows ? uint32_t(g.max_degree) : 0u)
                         .total;
  size_t chunk = kKspHbmScratch / per;
  if (chunk < 1) chunk = 1;
  if (chunk > size_t(nUnits)) chunk = size_t(nUnits);
  void* ws = nullptr;
  hipError_t e = workspace(chunk * per, stream, &ws);
  if (e != hipSuccess) return e;
  for (size_t u0 = 0; u0 < size_t(nUnits); u0 += chunk) {
    const size_t n = std::min(chunk, size_t(nUnits) - u0);
    hipLaunchKernelGGL((ksp_hbm_kernel<D, EXACT, TWO, MASKED>), dim3(uint32_t(n)),
                       dim3(EXACT ? 64 : kKspHbmBlock), 0, stream, g, sources, nSources, units,
                       uint32_t(u0), masks, maskWords, o1, o2, static_cast<char*>(ws));
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <typename D, bool MASKED>
hipError_t ksp_dispatch(const ogs_graph& g, const ogs_path_unit* units,
                        int nUnits, const uint32_t* masks, uint32_t maskWords,
                        const ogs_path_out& out, hipStream_t stream,
                        int* unsupported) {
  const uint64_t N = g.max_nodes, E = g.max_edges;
  if (opts().kspHbm) {
    return launch_ksp_hbm<D, false, false, MASKED>(g, nullptr, 0, units, nUnits, masks,
                                                   maskWords, out, out, stream);
  }
  const uint64_t core = align16(N * sizeof(D)) + align16((E + 31) / 32 * 4) +
      align16(N * sizeof(Frame));
  const uint64_t staged = core + align16((N + 1) * 4) + align16(E * 8);
  constexpr uint64_t kBudget = 160 * 1024;
  if (N <= 256 && staged * 4 <= kBudget / 2) {
    return ksp_launch<D, 64, true, MASKED>(g, units, nUnits, masks, maskWords,
                                           out, uint32_t(staged), stream);
  }
  if (staged <= kBudget / 2) {
    return ksp_launch<D, kBlock, true, MASKED>(g, units, nUnits, masks,
                                               maskWords, out, uint32_t(staged),
                                               stream);
  }
  if (core <= kBudget) {
    return ksp_launch<D, kBlock, false, MASKED>(g, units, nUnits, masks,
                                                maskWords, out, uint32_t(core),
                                                stream);
  }
  (void)unsupported;  // past LDS: state in HBM
  return launch_ksp_hbm<D, false, false, MASKED>(g, nullptr, 0, units, nUnits, masks,
                                                 maskWords, out, out, stream);
}

hipError_t launch_ksp(const ogs_graph& g, const ogs_path_unit* units,
                      int nUnits, const uint32_t* masks, uint32_t maskWords,
                      uint32_t flags, const ogs_path_out& out,
                      hipStream_t stream, int* unsupported) {
  const bool wide = flags & OGS_F_WIDE_METRIC;
  if (flags & OGS_F_EXACT_ORDER) {
    if (!wide) {
      *unsupported = 1;
      return hipSuccess;
    }
    return masks ? launch_ksp_hbm<uint64_t, true, false, true>(g, nullptr, 0, units, nUnits,
                                                               masks, maskWords, out, out, stream)
                 : launch_ksp_hbm<uint64_t, true, false, false>(g, nullptr, 0, units, nUnits,
                                                                nullptr, 0, out, out, stream);
  }
  if (masks) {
    return wide ? ksp_dispatch<uint64_t, true>(g, units, nUnits, masks,
                                               maskWords, out, stream,
                                               unsupported)
                : ksp_dispatch<uint32_t, true>(g, units, nUnits, masks,
                                               maskWords, out, stream,
                                               unsupported);
  }
  return wide ? ksp_dispatch<uint64_t, false>(g, units, nUnits, nullptr, 0,
                                              out, stream, unsupported)
              : ksp_dispatch<uint32_t, false>(g, units, nUnits, nullptr, 0, out,
                                              stream, unsupported);
}

// ---- KSP2 batch: getKthPaths(src, d, 1) and (src, d, 2) for many d -------
// Launch 1 (ksp_base_kernel): one unmasked SPF per distinct (topology,
// source) -- the reference's memoised getSpfResult(src) -- into HBM.
// Launch 2 (ksp2_kernel): per unit, the source's distances are copied into
// LDS, lane 0 traces the k = 1 paths and marks their links in an LDS mask,
// the unit reruns SPF with those links ignored (runSpf(src, true,
// linksToIgnore), LinkState.cpp:691-693) and lane 0 traces the k = 2 paths.

// Dist-only SPF with LDS node lists (the queue form of spf_frontier.hip's
// queue_spf, workgroup units only): round r walks the nodes changed in round
// r - 1 and pushes dist + w over their usable, unmasked links; one barrier
// per round. Same least fixpoint as spf_fixpoint (spf_core.h).
//
// prune (the masked rerun of ksp2_kernel: the k = 2 trace of destination
// `prune` only reads distances below dist(prune)): a push whose candidate is
// not below the current dist(prune) is dropped. Link metrics are >= 1 on
// this path (zero / negative metrics take the exact-order HBM form), so a
// node u with d(u) >= d(t) is never a predecessor on a shortest path to t
// (d(u) + w > d(t) >= d(v) for every v the trace visits), and every node
// with d(u) < d(t) keeps its exact distance: each relaxation along its
// shortest path has a candidate < d(t) <= dist(prune) at all times. Nodes at
// or past d(t) may keep larger (or no) distances; the trace's tight test
// rejects them either way. OGS_NODE_NONE: no pruning (the base SPF).
template <typename D, bool MASKED>
__device__ void queue_dist(uint32_t N, uint32_t s, const UnitCsr& c,
                           const uint8_t* __restrict__ nflags, D* dist,
                           uint32_t* stamp, uint16_t* q0, uint16_t* q1,
                           uint32_t* qcnt, const uint32_t* ignore,
                           uint32_t prune = OGS_NODE_NONE) {
  constexpr D kInf = DistInf<D>::value;
  const int tid = threadIdx.x;
  for (uint32_t v = tid; v < N; v += kBlock) {
    dist[v] = (v == s) ? D(0) : kInf;
    stamp[v] = 0u;
  }
  if (tid == 0) {
    q1[0] = uint16_t(s);  // round 1's list: buffer 1 & 1, count slot 1 % 3
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  __syncthreads();
  uint32_t n = 1;
  for (uint32_t r = 1; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint16_t* cur = (r & 1) ? q1 : q0;
    uint16_t* nxt = (r & 1) ? q0 : q1;
    for (uint32_t i = tid; i < n; i += kBlock) {
      const uint32_t v = cur[i];
      if (v != s && (nflags[v] & OGS_NODE_OVERLOADED)) continue;
      const D dv = dist[v];
      const D ub = prune != OGS_NODE_NONE ? dist[prune] : kInf;
      if (dv >= ub) continue;  // every push of v would be pruned
      const uint32_t rEnd = c.rowp[v + 1];
      for (uint32_t eb = c.rowp[v]; eb < rEnd; eb += 8) {
        uint64_t xs[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
          xs[k] = eb + k < rEnd ? c.edg[eb + k] : uint64_t(OGS_EDGE_DOWN);
        }
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
          const uint64_t ed = xs[k];
          const uint32_t lo = static_cast<uint32_t>(ed);
          if (lo & OGS_EDGE_DOWN) continue;
          if constexpr (MASKED) {
            const uint32_t l = link_id(c, eb + k, lo);
            if ((ignore[l >> 5] >> (l & 31u)) & 1u) continue;
          }
          const uint32_t t = edge_dst(lo);
          const D cand = dv + static_cast<D>(ed >> 32);
          if (cand < ub && cand < dist[t] && cand < atomicMin(&dist[t], cand)) {
            if (atomicMax(&stamp[t], r + 1) < r + 1) {
              nxt[atomicAdd(&qcnt[(r + 1) % 3], 1u)] = uint16_t(t);
            }
          }
        }
      }
    }
    __syncthreads();
    n = qcnt[(r + 1) % 3];
  }
}

// Per-unit LDS carve-up of both launches: dist, visited + mask link bitsets,
// trace stack, the queue form's stamps / lists / counters, optionally the
// staged CSR.
template <typename D>
struct KspLds {
  D* dist;
  uint32_t* visited;
  uint32_t* mask;
  Frame* stack;
  uint32_t* stamp;
  uint16_t *q0, *q1;
  uint32_t* qcnt;
  const uint8_t* nflags;
  UnitCsr csr;
  uint32_t N, linkWords;
};

// stage: 0 CSR read from HBM/L2, 1 row offsets in LDS, 2 rows + edges.
// The trace stack and the queue form's stamps / lists share one region: a
// unit traces (k = 1), then runs its SPF, then traces again (k = 2), never
// both at once -- 8 B per node less, more units per CU.
template <typename D>
__host__ __device__ inline uint64_t ksp_work_bytes(uint64_t N, bool queue) {
  const uint64_t st = align16(N * sizeof(Frame));
  const uint64_t q = queue ? align16(N * 4) + 2 * align16(N * 2) + 16 : 0;
  return st > q ? st : q;
}

template <typename D>
__host__ __device__ inline uint64_t ksp2_lds_bytes(uint64_t N, uint64_t E,
                                                   int stage, bool queue) {
  uint64_t b = align16(N * sizeof(D)) + 2 * align16((E + 31) / 32 * 4) +
      ksp_work_bytes<D>(N, queue);
  if (stage >= 1) b += align16((N + 1) * 4);
  if (stage >= 2) b += align16(E * 8);
  return b;
}

template <typename D, int STAGE, bool QUEUE, int UT>
__device__ KspLds<D> ksp_lds(char* base, const ogs_graph& g, uint32_t topo,
                             int lane) {
  const uint32_t nb = g.node_base[topo];
  const uint32_t N = g.node_base[topo + 1] - nb;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint32_t E = gRow[N] - e0;
  KspLds<D> l;
  l.N = N;
  l.linkWords = (E + 31) / 32;
  l.nflags = g.node_flags + nb;
  l.dist = reinterpret_cast<D*>(base);
  uint32_t off = align16(uint64_t(N) * sizeof(D));
  l.visited = reinterpret_cast<uint32_t*>(base + off);
  off += align16(uint64_t(l.linkWords) * 4);
  l.mask = reinterpret_cast<uint32_t*>(base + off);
  off += align16(uint64_t(l.linkWords) * 4);
  l.stack = reinterpret_cast<Frame*>(base + off);  // shared with the queue's
  if constexpr (QUEUE) {
    uint32_t q = off;
    l.stamp = reinterpret_cast<uint32_t*>(base + q);
    q += align16(uint64_t(N) * 4);
    l.q0 = reinterpret_cast<uint16_t*>(base + q);
    q += align16(uint64_t(N) * 2);
    l.q1 = reinterpret_cast<uint16_t*>(base + q);
    q += align16(uint64_t(N) * 2);
    l.qcnt = reinterpret_cast<uint32_t*>(base + q);
  }
  off += uint32_t(ksp_work_bytes<D>(N, QUEUE));
  if constexpr (STAGE >= 1) {
    uint32_t* lrow = reinterpret_cast<uint32_t*>(base + off);
    off += align16(uint64_t(N + 1) * 4);
    for (uint32_t i = lane; i <= N; i += UT) lrow[i] = gRow[i] - e0;
    if constexpr (STAGE >= 2) {
      uint64_t* ledg = reinterpret_cast<uint64_t*>(base + off);
      for (uint32_t i = lane; i < E; i += UT) ledg[i] = g.edges[e0 + i];
      l.csr = UnitCsr{lrow, ledg, 0u, g.rslot_ext ? g.rslot_ext + e0 : nullptr};
    } else {
      l.csr = UnitCsr{lrow, g.edges + e0, 0u, g.rslot_ext ? g.rslot_ext + e0 : nullptr};
    }
  } else {
    l.csr = UnitCsr{gRow, g.edges, e0, g.rslot_ext ? g.rslot_ext + e0 : nullptr};
  }
  for (uint32_t i = lane; i < l.linkWords; i += UT) {
    l.visited[i] = 0u;
    l.mask[i] = 0u;
  }
  return l;
}

// Lane 0's value to every lane of the unit.
template <int UT>
__device__ __forceinline__ uint32_t unit_bcast(uint32_t x) {
  if constexpr (UT == 64) {
    return __shfl(x, 0, 64);
  } else {
    __shared__ uint32_t b;
    __syncthreads();
    if (threadIdx.x == 0) b = x;
    __syncthreads();
    return b;
  }
}

// The unit's SPF into l.dist: queue form (workgroup units) or the pull
// fixpoint (spf_core.h).
template <typename D, int UT, bool QUEUE, bool MASKED>
__device__ __forceinline__ void ksp_spf(const KspLds<D>& l, uint32_t s, int lane,
                                        uint32_t prune = OGS_NODE_NONE) {
  if constexpr (QUEUE) {
    static_assert(UT == kBlock, "queue form: one workgroup per unit");
    queue_dist<D, MASKED>(l.N, s, l.csr, l.nflags, l.dist, l.stamp, l.q0, l.q1,
                          l.qcnt, l.mask, prune);
  } else {
    spf_fixpoint<D, 1, UT, false, MASKED>(l.N, s, lane, l.csr, false, l.dist,
                                          nullptr, MASKED ? l.mask : nullptr);
  }
}

template <typename D, int UT, int STAGE, bool QUEUE>
__global__ __launch_bounds__(kBlock) void ksp_base_kernel(
    ogs_graph g, const ogs_unit* __restrict__ sources, int nSources,
    D* __restrict__ srcDist, uint32_t ldsPerUnit) {
  constexpr int kUnitsPerBlock = kBlock / UT;
  const int uib = threadIdx.x / UT;
  const int lane = threadIdx.x % UT;
  const int sidx = blockIdx.x * kUnitsPerBlock + uib;
  if (sidx >= nSources) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ogs_unit src = sources[sidx];
  auto l = ksp_lds<D, STAGE, QUEUE, UT>(smem + uib * ldsPerUnit, g, src.topo, lane);
  ksp_spf<D, UT, QUEUE, false>(l, src.src, lane);
  D* row = srcDist + size_t(sidx) * uint32_t(g.max_nodes);
  for (uint32_t v = lane; v < l.N; v += UT) row[v] = l.dist[v];
}

template <typename D, int UT, int STAGE, bool QUEUE>
__global__ __launch_bounds__(kBlock) void ksp2_kernel(
    ogs_graph g, const ogs_unit* __restrict__ sources, int nSources,
    const D* __restrict__ srcDist, const ogs_path_unit* __restrict__ units,
    int nUnits, ogs_path_out o1, ogs_path_out o2, uint32_t ldsPerUnit, int waveTrace) {
  constexpr int kUnitsPerBlock = kBlock / UT;
  using Scope = UnitScope<UT>;
  const int uib = threadIdx.x / UT;
  const int lane = threadIdx.x % UT;
  const int uidx = blockIdx.x * kUnitsPerBlock + uib;
  // whole-block early exit only: the workgroup-scope path has barriers
  if (blockIdx.x * kUnitsPerBlock >= nUnits) return;
  const bool live = uidx < nUnits;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (!live) return;  // UT == 64 only: a wave of its own, no block barrier
  const ogs_path_unit unit = units[uidx];
  const uint32_t slot = unit.reserved;
  if (slot >= uint32_t(nSources) || sources[slot].topo != unit.topo ||
      sources[slot].src != unit.src) {
    if (lane == 0) {  // malformed unit: reported, never traced
      o1.path_count[uidx] = 0xC0000000u;
      o2.path_count[uidx] = 0xC0000000u;
    }
    return;
  }
  auto l = ksp_lds<D, STAGE, QUEUE, UT>(smem + uib * ldsPerUnit, g, unit.topo, lane);
  const D* row = srcDist + size_t(slot) * uint32_t(g.max_nodes);
  for (uint32_t v = lane; v < l.N; v += UT) l.dist[v] = row[v];
  Scope::sync();
  const uint32_t s = unit.src, t = unit.dest;
  uint32_t c1 = 0;
  const bool prune = (waveTrace & 2) != 0;  // "ksp_prune"
  const bool wt = sizeof(D) == 4 && (waveTrace & 1);
  if (wt && lane < 64) {
    if constexpr (sizeof(D) == 4) {
      c1 = trace_paths_wave<false>(l.csr, l.dist, s, t, l.visited, l.stack, nullptr, o1,
                                   uidx, l.mask, lane);
    }
    if (lane == 0) o1.path_count[uidx] = c1;
  } else if (!wt && lane == 0) {
    c1 = trace_paths<D, false>(l.csr, l.dist, s, t, l.visited, l.stack, nullptr,
                               o1, uidx, l.mask);
    o1.path_count[uidx] = c1;
  }
  c1 = unit_bcast<UT>(c1);
  // k = 1 found no path (src == dest or unreachable): linksToIgnore is empty,
  // so k = 2 re-traces the same SPF and finds none either. A k = 1 overflow
  // leaves the mask incomplete: reported for k = 2 as well.
  if (c1 == 0u || (c1 >> 31)) {
    if (lane == 0) o2.path_count[uidx] = c1 & 0x80000000u;
    return;
  }
  for (uint32_t i = lane; i < l.linkWords; i += UT) l.visited[i] = 0u;
  // the masked rerun only needs the distances below d(t) ("ksp_prune")
  ksp_spf<D, UT, QUEUE, true>(l, s, lane, prune ? t : OGS_NODE_NONE);
  if constexpr (sizeof(D) == 4) {
    if (wt) {
      if (lane >= 64) return;
      const uint32_t c2 = trace_paths_wave<true>(l.csr, l.dist, s, t, l.visited, l.stack,
                                                 l.mask, o2, uidx, nullptr, lane);
      if (lane == 0) o2.path_count[uidx] = c2;
      return;
    }
  }
  if (lane != 0) return;
  o2.path_count[uidx] = trace_paths<D, true>(l.csr, l.dist, s, t, l.visited,
                                             l.stack, l.mask, o2, uidx, nullptr);
}

template <typename D, int UT, int STAGE, bool QUEUE>
hipError_t ksp2_launch(const ogs_graph& g, const ogs_unit* sources,
                       int nSources, D* srcDist, const ogs_path_unit* units,
                       int nUnits, const ogs_path_out& o1,
                       const ogs_path_out& o2, uint32_t lds,
                       hipStream_t stream) {
  constexpr int upb = kBlock / UT;
  const size_t bytes = size_t(lds) * upb;
  auto kb = ksp_base_kernel<D, UT, STAGE, QUEUE>;
  auto k2 = ksp2_kernel<D, UT, STAGE, QUEUE>;
  if (bytes > 64 * 1024) {
    for (const void* f : {reinterpret_cast<const void*>(kb),
                          reinterpret_cast<const void*>(k2)}) {
      hipError_t e = hipFuncSetAttribute(
          f, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
      if (e != hipSuccess) return e;
    }
  }
  hipLaunchKernelGGL(kb, dim3((nSources + upb - 1) / upb), dim3(kBlock), bytes,
                     stream, g, sources, nSources, srcDist, lds);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k2, dim3((nUnits + upb - 1) / upb), dim3(kBlock), bytes,
                     stream, g, sources, nSources,
                     static_cast<const D*>(srcDist), units, nUnits, o1, o2, lds,
                     (opts().kspWaveTrace ? 1 : 0) | (opts().kspPrune ? 2 : 0));
  return hipGetLastError();
}

hipError_t workspace(size_t bytes, hipStream_t stream, void** out);

// "ksp_queue": 1 (default) workgroup units solve SPF with LDS node lists,
// 0 with the pull fixpoint. "ksp_stage": -1 (default) auto -- the edges in
// LDS only when three units still fit a CU, else the row offsets only --;
// 0 nothing staged, 1 row offsets, 2 rows + edges whenever they fit.
// EngineOptions::kspQueue (engine.h), default 1
// "ksp_prune": 1 (default) the masked rerun of the queue form drops pushes
// at or past the destination's current distance (queue_dist); 0 full SPF
// EngineOptions::kspPrune (engine.h), default 1
// EngineOptions::kspStage (engine.h), default -1

template <typename D>
hipError_t ksp2_dispatch(const ogs_graph& g, const ogs_unit* sources,
                         int nSources, const ogs_path_unit* units, int nUnits,
                         const ogs_path_out& o1, const ogs_path_out& o2,
                         hipStream_t stream, int* unsupported) {
  const uint64_t N = g.max_nodes, E = g.max_edges;
  constexpr uint64_t kBudget = 160 * 1024;
  if (opts().kspHbm) {
    return launch_ksp_hbm<D, false, true, false>(g, sources, nSources, units, nUnits,
                                                 nullptr, 0, o1, o2, stream);
  }
  void* ws = nullptr;
  hipError_t e = workspace(size_t(nSources) * size_t(N) * sizeof(D), stream, &ws);
  if (e != hipSuccess) return e;
  D* d = static_cast<D*>(ws);
  const uint64_t tiny = ksp2_lds_bytes<D>(N, E, 2, false);
  if (N <= 256 && tiny * 4 <= kBudget / 2) {
    return ksp2_launch<D, 64, 2, false>(g, sources, nSources, d, units, nUnits,
                                        o1, o2, uint32_t(tiny), stream);
  }
  const bool q = opts().kspQueue != 0 && N <= 65535;
  int st = opts().kspStage;
  if (st < 0) st = ksp2_lds_bytes<D>(N, E, 2, q) * 3 <= kBudget ? 2 : 1;
  while (st > 0 && ksp2_lds_bytes<D>(N, E, st, q) > kBudget) --st;
  const uint64_t b = ksp2_lds_bytes<D>(N, E, st, q);
  if (b > kBudget) {  // past LDS: state in HBM
    (void)unsupported;
    return launch_ksp_hbm<D, false, true, false>(g, sources, nSources, units, nUnits,
                                                 nullptr, 0, o1, o2, stream);
  }
#define OGS_KSP2(ST_, Q_)                                                      \
  return ksp2_launch<D, kBlock, ST_, Q_>(g, sources, nSources, d, units, nUnits, \
                                         o1, o2, uint32_t(b), stream);
  if (q) {
    if (st == 2) { OGS_KSP2(2, true) }
    if (st == 1) { OGS_KSP2(1, true) }
    OGS_KSP2(0, true)
  }
  if (st == 2) { OGS_KSP2(2, false) }
  if (st == 1) { OGS_KSP2(1, false) }
  OGS_KSP2(0, false)
#undef OGS_KSP2
}

hipError_t launch_ksp2(const ogs_graph& g, const ogs_unit* sources,
                       int nSources, const ogs_path_unit* units, int nUnits,
                       uint32_t flags, const ogs_path_out& o1,
                       const ogs_path_out& o2, hipStream_t stream,
                       int* unsupported) {
  if (flags & OGS_F_EXACT_ORDER) {
    if (!(flags & OGS_F_WIDE_METRIC)) {
      *unsupported = 1;
      return hipSuccess;
    }
    return launch_ksp_hbm<uint64_t, true, true, false>(g, sources, nSources, units, nUnits,
                                                       nullptr, 0, o1, o2, stream);
  }
  return (flags & OGS_F_WIDE_METRIC)
      ? ksp2_dispatch<uint64_t>(g, sources, nSources, units, nUnits, o1, o2,
                                stream, unsupported)
      : ksp2_dispatch<uint32_t>(g, sources, nSources, units, nUnits, o1, o2,
                                stream, unsupported);
}

}  // namespace ogs
