// spf_frontier.hip — frontier SPF for large topologies, one workgroup per
// (topology, source) unit: C3 fabric all-sources (N = 2,080, E = 43,008),
// C4 link-failure variants and C5 areas of WAN graphs.
//
// Same fixpoint as spf_core.h / spf_route_ms.hip (reference mapping there:
// LinkState::runSpf, LinkState.cpp:720-820): distances are the least
// solution of dist(v) = min over usable u of dist(u) + w(u, v), next-hop
// sets the least solution of NH(v) = U over tight u of (u == src ?
// {slot(src->v)} : NH(u)), where u relaxes iff u == src or u is not
// hard-drained (741-752). What differs is the work schedule: the pull
// sweeps of the other kernels touch every edge in every round; here only the
// rows of nodes that CHANGED in the previous round are pushed (Bellman-Ford
// with a frontier), so each phase costs about one pass over the edges:
//  * chunk_prep_kernel cuts every topology's rows into chunks of <= 8
//    directed edges, once per call, into a workspace list (u64: node | count
//    | hard-drained bit, local edge begin), so a round's work is balanced
//    over the workgroup however skewed the degrees (fabric: RSW 8, SSW 32,
//    FSW 84 links) and the list costs no LDS;
//  * stamp[v] = the round in which v must be pushed (set when its distance /
//    next-hop set changes; a node changed again mid-round is simply pushed
//    once more in the next round, which is exact for a monotone fixpoint);
//  * dist phase: push dist[v] + w into dist[u] with LDS atomicMin;
//    next-hop phase: the source's row seeds link-slot bits on tight edges,
//    then changed nodes push NH(v) into tight neighbours with atomicOr;
//  * edges and chunks stay in HBM/L2 (shared by every source of the batch);
//    LDS holds only dist / next-hop sets / stamps (10 B per node at W = 1),
//    so up to 7 units share a CU and hide each other's L2 latency.
// Outputs: dist[u*Sn + v], nh[(u*W + w)*Sn + v] (ogs_spf_out layout); the
// fused form then streams the unit's RouteDb (route_stream.h) from LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "openr_gpu.h"
#include "route_core.h"
#include "route_stream.h"
#include "spf_core.h"
#include "engine.h"

namespace ogs {

#ifndef OGS_CHUNK_EDGES  // edges per chunk record (A/B builds: -DOGS_CHUNK_EDGES=16)
#define OGS_CHUNK_EDGES 8
#endif
constexpr uint32_t kChunk = OGS_CHUNK_EDGES;
constexpr uint32_t kChunkCntShift = 21;  // bits 21..24: edge count - 1
constexpr uint32_t kChunkDrained = 1u << 25;
constexpr int kMaxDead = 8;  // ogs_unit_mods.dead_per_unit limit

// Exclusive prefix sum of x over the workgroup's current tile; returns the
// sum's base for this thread and adds the tile total to *base (LDS).
__device__ __forceinline__ uint32_t tile_scan(uint32_t x, uint32_t* wsum,
                                              uint32_t* base) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint32_t off = *base;
  for (int w = 0; w < wave; ++w) off += wsum[w];
  __syncthreads();
  if (threadIdx.x == kBlock - 1) *base = off + inc;
  return off + inc - x;
}

// Upper bound of sum_v ceil(deg(v)/8) over a topology.
__host__ __device__ inline uint32_t chunk_cap(const ogs_graph& g) {
  return uint32_t(g.max_edges) / kChunk + uint32_t(g.max_nodes);
}

// One workgroup per topology: chunks[t*cap + i], count nChunk[t].
__global__ __launch_bounds__(kBlock) void chunk_prep_kernel(
    ogs_graph g, uint32_t cap, uint64_t* __restrict__ chunks,
    uint32_t* __restrict__ nChunk) {
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ uint32_t base;
  const uint32_t t = blockIdx.x;
  const uint32_t nb = g.node_base[t];
  const uint32_t N = g.node_base[t + 1] - nb;
  const uint32_t* __restrict__ row = g.row_ptr + nb;
  const uint32_t e0 = row[0];
  uint64_t* out = chunks + size_t(t) * cap;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (uint32_t t0 = 0; t0 < N; t0 += kBlock) {
    const uint32_t v = t0 + threadIdx.x;
    uint32_t b = 0, deg = 0;
    if (v < N) {
      b = row[v] - e0;
      deg = row[v + 1] - e0 - b;
    }
    const uint32_t n = (deg + kChunk - 1) / kChunk;
    const uint32_t at = tile_scan(n, wsum, &base);
    const uint32_t drained =
        (v < N && (g.node_flags[nb + v] & OGS_NODE_OVERLOADED)) ? kChunkDrained : 0u;
    for (uint32_t k = 0; k < n; ++k) {
      const uint32_t cnt = min(kChunk, deg - k * kChunk);
      out[at + k] = uint64_t(v | ((cnt - 1) << kChunkCntShift) | drained) |
          (uint64_t(b + k * kChunk) << 32);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) nChunk[t] = base;
}

// Loads chunk ch's edges into registers: past the chunk's count an edge
// reads as DOWN (dst 0, never relaxes).
// Dead edges of a link-failure variant (ogs_unit_mods), unit-uniform.
struct DeadEdges {
  uint32_t e[kMaxDead];
  __device__ __forceinline__ bool has(uint32_t x) const {
    bool d = false;
#pragma unroll
    for (int k = 0; k < kMaxDead; ++k) d |= x == e[k];
    return d;
  }
};

template <bool MODS>
__device__ __forceinline__ void load_chunk(const uint64_t* __restrict__ edges,
                                           uint64_t ch, uint64_t (&x)[kChunk],
                                           const DeadEdges& dead) {
  const uint32_t b = uint32_t(ch >> 32);
  const uint32_t n = ((uint32_t(ch) >> kChunkCntShift) & 15u) + 1u;
#pragma unroll
  for (uint32_t i = 0; i < kChunk; ++i) {
    x[i] = i < n ? edges[b + i] : uint64_t(OGS_EDGE_DOWN);
    if constexpr (MODS) {
      if (dead.has(b + i)) x[i] |= uint64_t(OGS_EDGE_DOWN);
    }
  }
}

// chunk records loaded per scan step (independent L2 loads in flight)
constexpr int kScanBatch = 8;

// The chunk scan of one round over the thread's records c = tid, tid + B,
// ... < C, kScanBatch record loads in flight per step; relax(record, edges)
// runs for the records that pass active(record). Each lane walks only ITS
// active records (a lane-local bitmask, lowest first), so a wave runs as
// many relaxations per batch as its busiest lane has active records, not one
// per batch slot that any lane has active (a large frontier makes most slots
// active in some lane). PIPE: the next active record's edges are loaded
// before the current one is relaxed, two chunks of edges in registers (the
// few-units-per-CU geometries, B >= 512, where a round is a chain of
// dependent L2 round trips rather than a share of a busy CU).
template <int B, bool PIPE, bool MODS, typename Act, typename Relax>
__device__ __forceinline__ void scan_active(const uint64_t* __restrict__ chunks, uint32_t C,
                                            const uint64_t* __restrict__ edges,
                                            const DeadEdges& dead, bool slotWalk, Act active,
                                            Relax relax) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t c0 = tid; c0 < C; c0 += kScanBatch * B) {
    // eight records in named registers and record k by a select tree: an
    // indexed register array would be demoted to scratch memory
    static_assert(kScanBatch == 8, "eight records per scan step");
    auto rec = [&](int k) {
      const uint32_t c = c0 + uint32_t(k) * B;
      return c < C ? chunks[c] : ~0ull;
    };
    const uint64_t r0 = rec(0), r1 = rec(1), r2 = rec(2), r3 = rec(3);
    const uint64_t r4 = rec(4), r5 = rec(5), r6 = rec(6), r7 = rec(7);
    uint32_t m = 0;
    auto test = [&](int k, uint64_t ch) {
      if (c0 + uint32_t(k) * B < C && active(ch)) m |= 1u << k;
    };
    test(0, r0), test(1, r1), test(2, r2), test(3, r3);
    test(4, r4), test(5, r5), test(6, r6), test(7, r7);
    auto pick = [=](uint32_t k) {
      const uint64_t a01 = (k & 1u) ? r1 : r0, a23 = (k & 1u) ? r3 : r2;
      const uint64_t a45 = (k & 1u) ? r5 : r4, a67 = (k & 1u) ? r7 : r6;
      const uint64_t b0 = (k & 2u) ? a23 : a01, b1 = (k & 2u) ? a67 : a45;
      return (k & 4u) ? b1 : b0;
    };
    if (!PIPE && slotWalk) {  // A/B: one relaxation per slot any lane has active
      auto one = [&](int k, uint64_t ch) {
        if (!((m >> k) & 1u)) return;
        uint64_t x[kChunk];
        load_chunk<MODS>(edges, ch, x, dead);
        relax(ch, x);
      };
      one(0, r0), one(1, r1), one(2, r2), one(3, r3);
      one(4, r4), one(5, r5), one(6, r6), one(7, r7);
    } else if constexpr (!PIPE) {
      while (m) {
        const uint64_t ch = pick(uint32_t(__builtin_ctz(m)));
        m &= m - 1u;
        uint64_t x[kChunk];
        load_chunk<MODS>(edges, ch, x, dead);
        relax(ch, x);
      }
    } else {
      if (!m) continue;
      uint64_t ch = pick(uint32_t(__builtin_ctz(m)));
      m &= m - 1u;
      uint64_t x[kChunk];
      load_chunk<MODS>(edges, ch, x, dead);
      for (;;) {
        const bool more = m != 0u;
        uint64_t chn = 0, xn[kChunk];
        if (more) {
          chn = pick(uint32_t(__builtin_ctz(m)));
          m &= m - 1u;
          load_chunk<MODS>(edges, chn, xn, dead);
        }
        relax(ch, x);
        if (!more) break;
        ch = chn;
#pragma unroll
        for (uint32_t i = 0; i < kChunk; ++i) x[i] = xn[i];
      }
    }
  }
}

// One unit's SPF into LDS (dist[v], nh[v*W + w]); returns after the final
// workgroup barrier. stamp[] is scratch. B = threads per workgroup.
template <int W, bool MODS, int B = kBlock>
__device__ __forceinline__ void frontier_spf(
    uint32_t N, uint32_t s, const uint64_t* __restrict__ edges,
    const uint64_t* __restrict__ chunks, uint32_t C, bool hop,
    const uint32_t* __restrict__ gRow, uint32_t e0, uint32_t* dist,
    uint32_t* nh, uint16_t* stamp, uint64_t* tp, const DeadEdges& dead, bool seedRow,
    bool slotWalk) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  for (uint32_t v = tid; v < N; v += B) {
    dist[v] = (v == s) ? 0u : kInf;
    stamp[v] = (v == s) ? 1 : 0;
#pragma unroll
    for (int w = 0; w < W; ++w) nh[v * W + w] = 0u;
  }
  __syncthreads();
#ifdef OGS_STAMPS
  tp[0] = __builtin_amdgcn_s_memtime();
#endif

  // ---- dist phase: push dist(v) + w from the nodes changed last round ------
  // The round scans every chunk record for changed nodes: the thread's
  // records are loaded kScanBatch at a time (independent L2 loads in
  // flight) before their stamps are tested, instead of one dependent load
  // per record.
  // round 1 is the source's row alone: relaxed directly, one edge per thread
  // ("spf_seed_row"; off: round 1 scans like the others)
  if (seedRow) {
    const uint32_t b = gRow[s] - e0, n = gRow[s + 1] - e0 - b;
    for (uint32_t j = tid; j < n; j += B) {
      const uint64_t x = edges[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      if (lo & OGS_EDGE_DOWN) continue;
      if constexpr (MODS) {
        if (dead.has(b + j)) continue;
      }
      const uint32_t t = edge_dst(lo);
      const uint32_t c = hop ? 1u : static_cast<uint32_t>(x >> 32);
      if (c < dist[t]) {
        atomicMin(&dist[t], c);
        stamp[t] = 2;
      }
    }
    __syncthreads();
  }
  uint32_t r = seedRow ? 2 : 1;
  constexpr bool kPipe = B >= 512;
  for (;; ++r) {
    bool changed = false;
    auto active = [&](uint64_t ch) {
      const uint32_t v = uint32_t(ch) & OGS_EDGE_DST_MASK;
      return stamp[v] == r && (!(uint32_t(ch) & kChunkDrained) || v == s);
    };
    scan_active<B, kPipe, MODS>(chunks, C, edges, dead, slotWalk, active,
                                [&](uint64_t ch, const uint64_t (&x)[kChunk]) {
      const uint32_t v = uint32_t(ch) & OGS_EDGE_DST_MASK;
      const uint32_t dv = dist[v];
      uint32_t t[kChunk], cand[kChunk], dt[kChunk];
#pragma unroll
      for (uint32_t i = 0; i < kChunk; ++i) {
        const uint32_t lo = static_cast<uint32_t>(x[i]);
        t[i] = edge_dst(lo);
        cand[i] = (lo & OGS_EDGE_DOWN)
            ? kInf : dv + (hop ? 1u : static_cast<uint32_t>(x[i] >> 32));
      }
#pragma unroll
      for (uint32_t i = 0; i < kChunk; ++i) dt[i] = dist[t[i]];
#pragma unroll
      for (uint32_t i = 0; i < kChunk; ++i) {
        if (cand[i] < dt[i]) {
          atomicMin(&dist[t[i]], cand[i]);
          stamp[t[i]] = uint16_t(r + 1);
          changed = true;
        }
      }
    });
    if (!__syncthreads_or(changed)) break;
  }
#ifdef OGS_STAMPS
  tp[1] = __builtin_amdgcn_s_memtime();
  tp[3] = r;
#endif

  // ---- next-hop phase --------------------------------------------------------
  // seed: the source's own row (slot j = j-th edge of the source's row)
  const uint32_t r0 = r + 1;
  {
    const uint32_t b = gRow[s] - e0, n = gRow[s + 1] - e0 - b;
    for (uint32_t j = tid; j < n && j < 32u * W; j += B) {
      const uint64_t x = edges[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      if (lo & OGS_EDGE_DOWN) continue;
      if constexpr (MODS) {
        if (dead.has(b + j)) continue;
      }
      const uint32_t t = edge_dst(lo);
      const uint32_t w = hop ? 1u : static_cast<uint32_t>(x >> 32);
      if (w == dist[t]) {
        atomicOr(&nh[t * W + (j >> 5)], 1u << (j & 31u));
        stamp[t] = uint16_t(r0);
      }
    }
  }
  __syncthreads();
  // then changed nodes push NH(v) into tight neighbours
  for (r = r0;; ++r) {
    bool changed = false;
    auto active = [&](uint64_t ch) {
      const uint32_t v = uint32_t(ch) & OGS_EDGE_DST_MASK;
      return stamp[v] == r && v != s && !(uint32_t(ch) & kChunkDrained);
    };
    scan_active<B, kPipe, MODS>(chunks, C, edges, dead, slotWalk, active,
                                [&](uint64_t ch, const uint64_t (&x)[kChunk]) {
      const uint32_t v = uint32_t(ch) & OGS_EDGE_DST_MASK;
      const uint32_t dv = dist[v];
      uint32_t nv[W];
#pragma unroll
      for (int w = 0; w < W; ++w) nv[w] = nh[v * W + w];
      uint32_t t[kChunk], cand[kChunk], dt[kChunk];
#pragma unroll
      for (uint32_t i = 0; i < kChunk; ++i) {
        const uint32_t lo = static_cast<uint32_t>(x[i]);
        t[i] = edge_dst(lo);
        cand[i] = (lo & OGS_EDGE_DOWN)
            ? kInf : dv + (hop ? 1u : static_cast<uint32_t>(x[i] >> 32));
      }
#pragma unroll
      for (uint32_t i = 0; i < kChunk; ++i) dt[i] = dist[t[i]];
#pragma unroll
      for (uint32_t i = 0; i < kChunk; ++i) {
        if (cand[i] != dt[i]) continue;  // not a tight edge (or down)
        bool add = false;
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const uint32_t a = nv[k] & ~nh[t[i] * W + k];
          if (a) {
            atomicOr(&nh[t[i] * W + k], a);
            add = true;
          }
        }
        if (add) {
          stamp[t[i]] = uint16_t(r + 1);
          changed = true;
        }
      }
    });
    if (!__syncthreads_or(changed)) break;
  }
#ifdef OGS_STAMPS
  tp[2] = __builtin_amdgcn_s_memtime();
  tp[4] = r - r0 + 1;
#endif
}

// One-phase packed form of the chunk scan (W = 1): each node's LDS word is
// {dist, next-hop word}; a pushed edge replaces a longer word (64-bit LDS
// compare-and-swap) or ORs its next hops into an equal one, so distances and
// next-hop sets converge in the same rounds (the fabric: 5 rounds instead of
// 5 + 4 for the two phases above) -- the least fixpoint of spf_core.h, as
// queue_spf_packed. dn[v] is over dist + nh (8 B per node).
template <bool MODS, int B = kBlock>
__device__ __forceinline__ void frontier_spf_packed(
    uint32_t N, uint32_t s, const uint64_t* __restrict__ edges,
    const uint64_t* __restrict__ chunks, uint32_t C, bool hop,
    const uint32_t* __restrict__ gRow, uint32_t e0, uint64_t* dn, uint8_t* stamp,
    uint64_t* tp, const DeadEdges& dead, bool seedRow, bool slotWalk, bool preload) {
  // u8 round stamps (1 B per node, so 8 C3 units fit a CU): after 256
  // rounds a stale stamp can match again -- a reached node is pushed once
  // more with its current word, a no-op for the monotone fixpoint; an
  // unreached one (dist kInf, never stamped: stamp 0 == uint8_t(256)) is
  // skipped in relax, since kInf + w would wrap to a small candidate
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  for (uint32_t v = tid; v < N; v += B) {
    dn[v] = (v == s) ? 0ull : uint64_t(kInf);
    stamp[v] = (v == s) ? 1 : 0;
  }
  __syncthreads();
#ifdef OGS_STAMPS
  tp[0] = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t sb = gRow[s] - e0;  // the source's row: its link slots
  // round 1 is the source's row alone: its edges are relaxed directly (one
  // per thread) instead of a scan of every chunk record for one stamp
  // ("spf_seed_row" option; off: round 1 scans like the others)
  if (seedRow) {
    const uint32_t n = gRow[s + 1] - e0 - sb;
    for (uint32_t j = tid; j < n; j += B) {
      const uint64_t x = edges[sb + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      if (lo & OGS_EDGE_DOWN) continue;
      if constexpr (MODS) {
        if (dead.has(sb + j)) continue;
      }
      const uint32_t t = edge_dst(lo);
      const uint32_t c = hop ? 1u : static_cast<uint32_t>(x >> 32);
      const uint32_t bits = j < 32u ? 1u << j : 0u;
      uint64_t old = dn[t];
      for (;;) {
        const uint32_t dt = static_cast<uint32_t>(old), nt = static_cast<uint32_t>(old >> 32);
        if (c > dt || (c == dt && !(bits & ~nt))) break;
        const uint64_t nw = c < dt ? (uint64_t(c) | (uint64_t(bits) << 32))
                                   : (uint64_t(dt) | (uint64_t(nt | bits) << 32));
        const uint64_t seen = atomicCAS(reinterpret_cast<unsigned long long*>(&dn[t]),
                                        static_cast<unsigned long long>(old),
                                        static_cast<unsigned long long>(nw));
        if (seen == old) {
          stamp[t] = 2;
          break;
        }
        old = seen;
      }
    }
    __syncthreads();
  }
  uint32_t r = seedRow ? 2 : 1;
  const uint32_t* dn32 = reinterpret_cast<const uint32_t*>(dn);  // dist = low word
  for (;; ++r) {
    bool changed = false;
    auto active = [&](uint64_t ch) {
      const uint32_t v = uint32_t(ch) & OGS_EDGE_DST_MASK;
      return stamp[v] == uint8_t(r) && (!(uint32_t(ch) & kChunkDrained) || v == s);
    };
    auto relax = [&](uint64_t ch, const uint64_t (&x)[kChunk]) {
      const uint32_t v = uint32_t(ch) & OGS_EDGE_DST_MASK;
      const uint64_t xv = dn[v];
      const uint32_t dv = static_cast<uint32_t>(xv), nv = static_cast<uint32_t>(xv >> 32);
      if (dv == kInf) return;  // a stale stamp on an unreached node
      const uint32_t b = uint32_t(ch >> 32);
      // the targets' distances first (independent LDS reads): a longer
      // candidate -- most pushes of a dense frontier -- is dropped without
      // the dependent read + compare-and-swap chain below (distances only
      // fall, so a stale preload never drops a useful push)
      uint32_t dt[kChunk];
#pragma unroll
      for (uint32_t i = 0; i < kChunk; ++i) {
        dt[i] = preload ? dn32[2u * edge_dst(uint32_t(x[i]))] : 0xFFFFFFFFu;
      }
#pragma unroll
      for (uint32_t i = 0; i < kChunk; ++i) {
        const uint32_t lo = static_cast<uint32_t>(x[i]);
        if (lo & OGS_EDGE_DOWN) continue;
        const uint32_t t = edge_dst(lo);
        const uint32_t c = dv + (hop ? 1u : static_cast<uint32_t>(x[i] >> 32));
        if (c > dt[i]) continue;
        // the source contributes its link slot (W = 1: degree <= 32), every
        // other node NH(v) (LinkState.cpp:808-811)
        const uint32_t slot = b + i - sb;
        const uint32_t bits = (v == s) ? (slot < 32u ? 1u << slot : 0u) : nv;
        uint64_t old = dn[t];
        for (;;) {
          const uint32_t dt = static_cast<uint32_t>(old), nt = static_cast<uint32_t>(old >> 32);
          if (c > dt || (c == dt && !(bits & ~nt))) break;
          const uint64_t nw = c < dt ? (uint64_t(c) | (uint64_t(bits) << 32))
                                     : (uint64_t(dt) | (uint64_t(nt | bits) << 32));
          const uint64_t seen = atomicCAS(reinterpret_cast<unsigned long long*>(&dn[t]),
                                          static_cast<unsigned long long>(old),
                                          static_cast<unsigned long long>(nw));
          if (seen == old) {
            stamp[t] = uint8_t(r + 1);
            changed = true;
            break;
          }
          old = seen;
        }
      }
    };
    scan_active<B, (B >= 512), MODS>(chunks, C, edges, dead, slotWalk, active, relax);
    if (!__syncthreads_or(changed)) break;
  }
#ifdef OGS_STAMPS
  tp[1] = tp[2] = __builtin_amdgcn_s_memtime();
  tp[3] = r;
  tp[4] = 0;
#endif
}

// ---- queue form: sparse, deep topologies (C4 / C5 WAN areas) ---------------
// The chunk scan above reads every chunk record of the topology each round
// to find the changed nodes: cheap per round on the dense fabric (few,
// wide rounds), but a WAN needs ~70 narrow rounds per phase and the scan
// dominates. Here the nodes changed in round r are appended (once, stamp
// dedupe by LDS atomicMax) to an LDS list that round r + 1 walks; a round
// touches only the rows of those nodes and ends at ONE workgroup barrier
// (three rotating list counters, so the next count is reset while the
// current one is live). Same fixpoint, same outputs as frontier_spf.
// Edges of a row, 8 loads in flight at a time: fn(local edge id, edge).
template <typename Fn>
__device__ __forceinline__ void for_row(const uint64_t* __restrict__ edges,
                                        uint32_t b, uint32_t m, Fn fn) {
  for (uint32_t jb = 0; jb < m; jb += 8) {
    uint64_t xs[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      xs[k] = jb + k < m ? edges[b + jb + k] : uint64_t(OGS_EDGE_DOWN);
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      if (jb + k < m) fn(b + jb + k, xs[k]);
    }
  }
}

template <int W, bool MODS>
__device__ __forceinline__ void queue_spf(
    uint32_t N, uint32_t s, const uint64_t* __restrict__ edges,
    const uint32_t* __restrict__ gRow, uint32_t e0,
    const uint8_t* __restrict__ nflags, bool hop, uint32_t* dist, uint32_t* nh,
    uint32_t* stamp, uint16_t* q0, uint16_t* q1, uint32_t* qcnt, uint32_t* ninfo,
    uint64_t* tp, const DeadEdges& dead) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  constexpr uint32_t kDrained = 0x80000000u;
  const int tid = threadIdx.x;
  for (uint32_t v = tid; v < N; v += kBlock) {
    dist[v] = (v == s) ? 0u : kInf;
    stamp[v] = 0u;
#pragma unroll
    for (int w = 0; w < W; ++w) nh[v * W + w] = 0u;
  }
  // node info: local row begin | hard-drained bit (one LDS read per node)
  for (uint32_t v = tid; ninfo && v <= N; v += kBlock) {  // nullptr: CSR reads
    ninfo[v] = (gRow[v] - e0) |
        ((v < N && (nflags[v] & OGS_NODE_OVERLOADED)) ? kDrained : 0u);
  }
  if (tid == 0) {
    q1[0] = uint16_t(s);  // round 1's list: buffer 1 & 1, count slot 1 % 3
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  __syncthreads();
#ifdef OGS_STAMPS
  tp[0] = __builtin_amdgcn_s_memtime();
#endif
  // list of round r: buffer r & 1, count slot r % 3; appends go to round
  // r + 1's buffer / slot; slot (r + 2) % 3 is idle during round r
  auto append = [&](uint32_t t, uint32_t r) {
    if (atomicMax(&stamp[t], r + 1) < r + 1) {
      const uint32_t at = atomicAdd(&qcnt[(r + 1) % 3], 1u);
      ((r + 1) & 1 ? q1 : q0)[at] = uint16_t(t);
    }
  };
  uint32_t r = 1, n = 1;
  for (; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint16_t* cur = (r & 1) ? q1 : q0;
    for (uint32_t i = tid; i < n; i += kBlock) {
      const uint32_t v = cur[i];
      const uint32_t iv = ninfo ? ninfo[v]
                                : ((gRow[v] - e0) |
                                   ((nflags[v] & OGS_NODE_OVERLOADED) ? kDrained : 0u));
      const uint32_t b = iv & ~kDrained;
      const uint32_t rowEnd = ninfo ? (ninfo[v + 1] & ~kDrained) : gRow[v + 1] - e0;
      if (v != s && (iv & kDrained)) continue;  // LinkState.cpp:741-752
      const uint32_t dv = dist[v];
      for_row(edges, b, rowEnd - b, [&](uint32_t e, uint64_t x) {
        const uint32_t lo = static_cast<uint32_t>(x);
        if (lo & OGS_EDGE_DOWN) return;
        if constexpr (MODS) {
          if (dead.has(e)) return;
        }
        const uint32_t t = edge_dst(lo);
        const uint32_t c = dv + (hop ? 1u : static_cast<uint32_t>(x >> 32));
        if (c < dist[t] && c < atomicMin(&dist[t], c)) append(t, r);
      });
    }
    __syncthreads();
    n = qcnt[(r + 1) % 3];
  }
#ifdef OGS_STAMPS
  tp[1] = __builtin_amdgcn_s_memtime();
  tp[3] = r;
#endif
  // ---- next-hop phase: seeds from the source's row, then tight pushes -----
  const uint32_t r0 = r;
  __syncthreads();  // every thread has read the last (zero) count
  if (tid == 0) qcnt[0] = qcnt[1] = qcnt[2] = 0u;
  __syncthreads();
  {
    const uint32_t b = gRow[s] - e0, m = gRow[s + 1] - e0 - b;
    for (uint32_t j = tid; j < m && j < 32u * W; j += kBlock) {
      const uint64_t x = edges[b + j];
      const uint32_t lo = static_cast<uint32_t>(x);
      if (lo & OGS_EDGE_DOWN) continue;
      if constexpr (MODS) {
        if (dead.has(b + j)) continue;
      }
      const uint32_t t = edge_dst(lo);
      const uint32_t w = hop ? 1u : static_cast<uint32_t>(x >> 32);
      if (w == dist[t]) {
        atomicOr(&nh[t * W + (j >> 5)], 1u << (j & 31u));
        append(t, r0);
      }
    }
  }
  __syncthreads();
  n = qcnt[(r0 + 1) % 3];
  for (r = r0 + 1; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint16_t* cur = (r & 1) ? q1 : q0;
    for (uint32_t i = tid; i < n; i += kBlock) {
      const uint32_t v = cur[i];
      const uint32_t iv = ninfo ? ninfo[v]
                                : ((gRow[v] - e0) |
                                   ((nflags[v] & OGS_NODE_OVERLOADED) ? kDrained : 0u));
      const uint32_t b = iv & ~kDrained;
      const uint32_t rowEnd = ninfo ? (ninfo[v + 1] & ~kDrained) : gRow[v + 1] - e0;
      if (v == s || (iv & kDrained)) continue;
      const uint32_t dv = dist[v];
      uint32_t nv[W];
#pragma unroll
      for (int w = 0; w < W; ++w) nv[w] = nh[v * W + w];
      for_row(edges, b, rowEnd - b, [&](uint32_t e, uint64_t x) {
        const uint32_t lo = static_cast<uint32_t>(x);
        if (lo & OGS_EDGE_DOWN) return;
        if constexpr (MODS) {
          if (dead.has(e)) return;
        }
        const uint32_t t = edge_dst(lo);
        if (dv + (hop ? 1u : static_cast<uint32_t>(x >> 32)) != dist[t]) return;
        bool add = false;
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const uint32_t a = nv[k] & ~nh[t * W + k];
          if (a && (a & ~atomicOr(&nh[t * W + k], a))) add = true;
        }
        if (add) append(t, r);
      });
    }
    __syncthreads();
    n = qcnt[(r + 1) % 3];
  }
#ifdef OGS_STAMPS
  tp[2] = __builtin_amdgcn_s_memtime();
  tp[4] = r - r0;
#endif
}

// Queue form with ONE phase (next-hop sets of one word): dist and next-hop
// bits packed per node in a u64 LDS word {dist | nh << 32} updated by CAS,
// so a push carries both -- a strictly shorter candidate replaces the word,
// an equal one ORs its bits in -- and a node whose word changed is queued
// again. Converges to the same least fixpoint as the two-phase form in about
// half the rounds (a node's final push carries its final word; contributions
// of a pred survive only while it stays tight, since a strictly shorter path
// resets the word). (Push stamps folded into the words' top bits measured
// 8 % slower on C4 -- concurrent CASes on a node conflict more -- and were
// removed in round 4.)
// Rounds of the packed queue SPF from the current list state: round r's
// list is buffer r & 1 with count slot r % 3 holding n entries (stamps
// already claim them). Returns the round after the last non-empty one.
template <bool MODS>
__device__ __forceinline__ uint32_t packed_rounds(
    uint32_t s, const uint64_t* __restrict__ edges, const uint32_t* __restrict__ gRow,
    uint32_t e0, const uint8_t* __restrict__ nflags, bool hop, uint64_t* dn,
    uint32_t* stamp, uint16_t* q0, uint16_t* q1, uint32_t* qcnt, const uint32_t* ninfo,
    const DeadEdges& dead, uint32_t r, uint32_t n) {
  constexpr uint32_t kDrained = 0x80000000u;
  const int tid = threadIdx.x;
  for (; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint16_t* cur = (r & 1) ? q1 : q0;
    uint16_t* nxt = (r & 1) ? q0 : q1;
    for (uint32_t i = tid; i < n; i += kBlock) {
      const uint32_t v = cur[i];
      const uint32_t iv = ninfo ? ninfo[v]
                                : ((gRow[v] - e0) |
                                   ((nflags[v] & OGS_NODE_OVERLOADED) ? kDrained : 0u));
      const uint32_t b = iv & ~kDrained;
      const uint32_t rowEnd = ninfo ? (ninfo[v + 1] & ~kDrained) : gRow[v + 1] - e0;
      if (v != s && (iv & kDrained)) continue;  // LinkState.cpp:741-752
      const uint64_t xv = dn[v];
      const uint32_t dv = static_cast<uint32_t>(xv);
      const uint32_t nv = static_cast<uint32_t>(xv >> 32);
      for_row(edges, b, rowEnd - b, [&](uint32_t e, uint64_t x) {
        const uint32_t lo = static_cast<uint32_t>(x);
        if (lo & OGS_EDGE_DOWN) return;
        if constexpr (MODS) {
          if (dead.has(e)) return;
        }
        const uint32_t t = edge_dst(lo);
        const uint32_t c = dv + (hop ? 1u : static_cast<uint32_t>(x >> 32));
        // the source contributes the link slot (its row index), others NH(v)
        const uint32_t bits = (v == s) ? (1u << (e - b)) : nv;
        uint64_t old = dn[t];
        for (;;) {
          const uint32_t dt = static_cast<uint32_t>(old);
          const uint32_t nt = static_cast<uint32_t>(old >> 32);
          if (c > dt || (c == dt && !(bits & ~nt))) return;
          const uint64_t nw = c < dt ? (uint64_t(c) | (uint64_t(bits) << 32))
                                     : (uint64_t(dt) | (uint64_t(nt | bits) << 32));
          const uint64_t seen = atomicCAS(reinterpret_cast<unsigned long long*>(&dn[t]),
                                          static_cast<unsigned long long>(old),
                                          static_cast<unsigned long long>(nw));
          if (seen == old) break;
          old = seen;
        }
        if (atomicMax(&stamp[t], r + 1) < r + 1) nxt[atomicAdd(&qcnt[(r + 1) % 3], 1u)] = uint16_t(t);
      });
    }
    __syncthreads();
    n = qcnt[(r + 1) % 3];
  }
  return r;
}

template <bool MODS>
__device__ __forceinline__ void queue_spf_packed(
    uint32_t N, uint32_t s, const uint64_t* __restrict__ edges,
    const uint32_t* __restrict__ gRow, uint32_t e0,
    const uint8_t* __restrict__ nflags, bool hop, uint64_t* dn, uint32_t* stamp,
    uint16_t* q0, uint16_t* q1, uint32_t* qcnt, uint32_t* ninfo, uint64_t* tp,
    const DeadEdges& dead) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  constexpr uint32_t kDrained = 0x80000000u;
  const int tid = threadIdx.x;
  for (uint32_t v = tid; v < N; v += kBlock) {
    dn[v] = (v == s) ? 0ull : uint64_t(kInf);
    stamp[v] = 0u;
  }
  for (uint32_t v = tid; ninfo && v <= N; v += kBlock) {  // nullptr: CSR reads
    ninfo[v] = (gRow[v] - e0) |
        ((v < N && (nflags[v] & OGS_NODE_OVERLOADED)) ? kDrained : 0u);
  }
  if (tid == 0) {
    q1[0] = uint16_t(s);
    qcnt[0] = 0u;
    qcnt[1] = 1u;
    qcnt[2] = 0u;
  }
  __syncthreads();
#ifdef OGS_STAMPS
  tp[0] = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t r = packed_rounds<MODS>(s, edges, gRow, e0, nflags, hop, dn, stamp,
                                         q0, q1, qcnt, ninfo, dead, 1u, 1u);
#ifdef OGS_STAMPS
  tp[1] = tp[2] = __builtin_amdgcn_s_memtime();
  tp[3] = r;
  tp[4] = 0;
#else
  (void)r;
#endif
}

uint32_t frontier_lds_bytes(uint32_t Sn, int W, bool queue = false, bool ninfo = true,
                            bool stamp8 = false) {
  const uint32_t core = 4u * (((Sn + 3u) & ~3u) + ((Sn * W + 3u) & ~3u));
  if (!queue) return core + (stamp8 ? ((Sn + 3u) & ~3u) : 2u * ((Sn + 1u) & ~1u));
  // + u32 stamps + two u16 node lists (+ u32 node info [Sn + 1])
  return core + 4u * ((Sn + 3u) & ~3u) + 2u * 2u * ((Sn + 1u) & ~1u) +
      (ninfo ? 4u * ((Sn + 4u) & ~3u) : 0u);
}

// internal launch flag (above the public OGS_F_* bits): the queue forms read
// row bounds / drained bits from the CSR instead of an LDS node-info array
constexpr uint32_t kFlagNinfoGlobal = 1u << 30;
// round 1 of the chunk-scan forms scans the chunk records too (spf_seed_row 0)
constexpr uint32_t kFlagScanRound1 = 1u << 27;
// Chunk-scan walk: per slot ("spf_lane_walk" 0) or per lane (1); -1 (auto)
// walks lanes in the few-units-per-CU geometries (B >= 512) only: at 256
// threads and 7 units per CU the lane walk measured 3 % slower on C3
// (1.316 vs 1.277 ms, profiles/r04_scan_ab.log). "spf_preload" 0: no
// preloaded target distances in the packed relax (A/B).
constexpr uint32_t kFlagSlotWalk = 1u << 29;
constexpr uint32_t kFlagNoPreload = 1u << 26;
// EngineOptions::spfLaneWalk (engine.h), default -1
// EngineOptions::spfPreload (engine.h), default 1

#ifdef OGS_STAMPS
// diagnostic build (make stamps): 8 phase clocks per workgroup of the last
// frontier launch, read back with ogs_diag_stamps (tools/c3_stamps.py)
constexpr uint32_t kDiagWgs = 65536;
__device__ uint32_t g_diagStamps[kDiagWgs * 8];
#endif

// ROUTES = false: SPF only, dist / nh to HBM.
// ROUTES = true: SPF + the unit's RouteDb stream (route_stream.h) from LDS;
// dist / nh go to HBM only when requested.
// B threads per workgroup; `parts` workgroups per unit (OUTS3 launches
// only): each runs the unit's SPF and streams one 1/parts prefix range of
// its RouteDb, part 0 also writes dist / nh. A launch of few units (one
// rank's shard of the C3 sources) so keeps enough waves streaming per CU.
template <int W, bool ROUTES, bool MODS, bool DIFF, int QMODE, bool OUTS3, int B = kBlock>
__device__ __forceinline__ void spf_frontier_body(
    const ogs_graph& g, const ogs_prefix_table& pt, const uint32_t* __restrict__ key,
    const uint64_t* __restrict__ chunks, const uint32_t* __restrict__ nChunk,
    uint32_t cap, const ogs_unit* __restrict__ units, uint32_t flags,
    uint32_t* __restrict__ oDist, uint32_t* __restrict__ oNh, const ogs_spf_out& out,
    const ogs_unit_mods& mods, const ogs_route_diff& diff, uint32_t parts) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  static_assert(B == kBlock || (OUTS3 && !MODS && !DIFF && (QMODE == 0 || QMODE == 4)),
                "other block sizes only for the all-sources stream");
  const uint32_t u0 = OUTS3 ? blockIdx.x / parts : blockIdx.x;
  const uint32_t part = OUTS3 ? blockIdx.x - u0 * parts : 0u;
  const ogs_unit unit = units[u0];
  const uint32_t s = unit.src;
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const uint32_t Sn = uint32_t(g.max_nodes);

  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* dist = reinterpret_cast<uint32_t*>(smem);              // [Sn]
  uint32_t* nh = dist + ((Sn + 3u) & ~3u);                           // [Sn*W]
  uint16_t* stamp = reinterpret_cast<uint16_t*>(nh + ((Sn * W + 3u) & ~3u));  // [Sn]
  // queue form: u32 stamps [Sn] over the same start, then two u16 lists
  uint32_t* stamp32 = reinterpret_cast<uint32_t*>(stamp);
  uint16_t* q0 = reinterpret_cast<uint16_t*>(stamp32 + ((Sn + 3u) & ~3u));
  uint16_t* q1 = q0 + ((Sn + 1u) & ~1u);
  uint32_t* ninfo = (flags & kFlagNinfoGlobal)
      ? nullptr
      : reinterpret_cast<uint32_t*>(q1 + ((Sn + 1u) & ~1u));
  __shared__ uint32_t qcnt[3];

  DeadEdges dead;
#pragma unroll
  for (int k = 0; k < kMaxDead; ++k) {
    dead.e[k] = (MODS && k < mods.dead_per_unit)
        ? mods.dead_edges[size_t(u0) * mods.dead_per_unit + k]
        : OGS_NODE_NONE;
  }
  uint64_t tp[5] = {0, 0, 0, 0, 0};
#ifdef OGS_STAMPS
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  constexpr bool PACKED = QMODE >= 2;
  static_assert(!PACKED || W == 1, "packed words hold one next-hop word");
  uint64_t* dn64 = reinterpret_cast<uint64_t*>(smem);  // PACKED: over dist + nh
  if constexpr (QMODE == 4) {  // packed words, chunk scan
    frontier_spf_packed<MODS, B>(N, s, g.edges + e0, chunks + size_t(unit.topo) * cap,
                              nChunk[unit.topo], (flags & OGS_F_HOP_METRIC) != 0, gRow, e0,
                              dn64, reinterpret_cast<uint8_t*>(stamp), tp, dead,
                              (flags & kFlagScanRound1) == 0, (flags & kFlagSlotWalk) != 0,
                              (flags & kFlagNoPreload) == 0);
  } else if constexpr (PACKED) {
    queue_spf_packed<MODS>(N, s, g.edges + e0, gRow, e0, nflags,
                           (flags & OGS_F_HOP_METRIC) != 0, dn64, stamp32, q0, q1,
                           qcnt, ninfo, tp, dead);
  } else if constexpr (QMODE == 1) {
    queue_spf<W, MODS>(N, s, g.edges + e0, gRow, e0, nflags,
                       (flags & OGS_F_HOP_METRIC) != 0, dist, nh, stamp32, q0, q1,
                       qcnt, ninfo, tp, dead);
  } else {
    frontier_spf<W, MODS, B>(N, s, g.edges + e0, chunks + size_t(unit.topo) * cap,
                          nChunk[unit.topo], (flags & OGS_F_HOP_METRIC) != 0, gRow,
                          e0, dist, nh, stamp, tp, dead,
                          (flags & kFlagScanRound1) == 0, (flags & kFlagSlotWalk) != 0);
  }

  auto dOf = [&](uint32_t v) -> uint32_t {
    if constexpr (PACKED) return static_cast<uint32_t>(dn64[v]);
    else return dist[v];
  };
  auto nOf = [&](uint32_t v, int w) -> uint32_t {
    if constexpr (PACKED) return static_cast<uint32_t>(dn64[v] >> 32);
    else return nh[v * W + w];
  };
  for (uint32_t v = tid; part == 0u && v < N; v += B) {
    if (oDist) oDist[size_t(u0) * Sn + v] = dOf(v);
#pragma unroll
    for (int w = 0; w < W; ++w) {
      if (oNh) oNh[(size_t(u0) * W + w) * Sn + v] = nOf(v, w);
    }
  }
  if constexpr (ROUTES) {
    // per-node record flags (8 bits) over the dead stamps (u8 stamps in
    // the packed chunk scan: one byte per node there)
    using RMeta = std::conditional_t<QMODE == 4, uint8_t, uint16_t>;
    RMeta* rMeta = reinterpret_cast<RMeta*>(stamp);
    for (uint32_t v = tid; v < N; v += B) {
      uint32_t cnt = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) cnt += __popc(nOf(v, w));
      rMeta[v] = RMeta(node_route_meta(v, s, dOf(v) != kInf, cnt, nflags[v]));
    }
    __syncthreads();
    const uint32_t Sp = uint32_t(pt.max_prefixes);
    const uint32_t p0 = pt.pfx_base[unit.topo];
    const uint32_t P = pt.pfx_base[unit.topo + 1] - p0;
    const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0,
                       (flags & OGS_F_V4_OVER_V6) != 0,
                       (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
    __shared__ uint32_t cnt[2];
    if constexpr (DIFF) {
      if (tid < 2) cnt[tid] = 0u;
      __syncthreads();
    }
    const DiffCtx dc{diff.base_meta, diff.base_metric, diff.base_mask,
                     diff.changed + size_t(u0) * ((Sp + 31u) / 32u), cnt,
                     pt.adv_off + p0, diff.adv_class};
    auto rec = [&](uint32_t v, Rec<W>& r) {
      r.meta = rMeta[v];
      r.metric = (v == s) ? kInf : dOf(v);
#pragma unroll
      for (int w = 0; w < W; ++w) r.mask[w] = nOf(v, w);
    };
    // this part's prefix range, 4-aligned (16-B accesses)
    const uint32_t span = ((P + parts - 1u) / parts + 3u) & ~3u;
    const uint32_t lo = min(P, part * span), hi = min(P, lo + span);
    if constexpr (PACKED) {
      stream_routes<W, DIFF, OUTS3, B>(pt, key + size_t(unit.topo) * Sp, p0, P, Sp, u0, s,
                                       nflags, PackedView{dn64}, cfg, out, rec, &dc,
                                       (flags & kFlagNtStores) != 0, lo, hi);
    } else {
      stream_routes<W, DIFF, OUTS3, B>(pt, key + size_t(unit.topo) * Sp, p0, P, Sp, u0, s,
                                       nflags, SplitView<uint32_t, W>{dist, nh}, cfg, out,
                                       rec, &dc, (flags & kFlagNtStores) != 0, lo, hi);
    }
    if constexpr (DIFF) {
      __syncthreads();
      if (tid < 2) diff.counts[size_t(u0) * 2 + tid] = cnt[tid];
    }
  }
#ifdef OGS_STAMPS  // diagnostic build only: phase clocks per workgroup
  __syncthreads();
  // rows (W - 1) * 16384 + blockIdx.x: two width groups' launches overlap
  if (tid == 0 && blockIdx.x < kDiagWgs / 4) {
    uint32_t* st = g_diagStamps + (size_t(W - 1) * (kDiagWgs / 4) + blockIdx.x) * 8u;
    st[0] = uint32_t(tp[0] - t0);       // setup
    st[1] = uint32_t(tp[1] - tp[0]);    // dist phase
    st[2] = uint32_t(tp[2] - tp[1]);    // next-hop phase
    st[3] = uint32_t(__builtin_amdgcn_s_memtime() - tp[2]);  // outputs + routes
    st[4] = uint32_t(tp[3]);            // dist rounds
    st[5] = uint32_t(tp[4]);            // next-hop rounds
    st[6] = uint32_t(rt0);
    st[7] = uint32_t(__builtin_amdgcn_s_memrealtime());
  }
#endif
}

template <int W, bool ROUTES, bool MODS = false, bool DIFF = false,
          int QMODE = 0, bool OUTS3 = false, int B = kBlock>
__global__ __launch_bounds__(B) void spf_frontier_kernel(
    ogs_graph g, ogs_prefix_table pt, const uint32_t* __restrict__ key,
    const uint64_t* __restrict__ chunks, const uint32_t* __restrict__ nChunk,
    uint32_t cap, const ogs_unit* __restrict__ units, uint32_t flags,
    uint32_t* __restrict__ oDist, uint32_t* __restrict__ oNh, ogs_spf_out out,
    ogs_unit_mods mods, ogs_route_diff diff, uint32_t parts) {
  spf_frontier_body<W, ROUTES, MODS, DIFF, QMODE, OUTS3, B>(g, pt, key, chunks, nChunk, cap,
                                                             units, flags, oDist, oNh, out,
                                                             mods, diff, parts);
}

// "spf_seed_row" option: 1 (default) round 1 of the chunk-scan forms relaxes
// the source's row directly, 0 it scans every chunk record (A/B)
// EngineOptions::spfSeedRow (engine.h), default 1


// "spf_packed_scan" option: 1 (default) chunk-scan units with one-word
// next-hop sets relax packed {dist, nh} words in one phase
// (frontier_spf_packed), 0 the two-phase chunk scan (A/B)
// EngineOptions::spfPackedScan (engine.h), default 1

// "spf_queue" option: -1 (default) the queue form for sparse topologies
// (max degree <= 16, <= 65,535 nodes; one-phase packed words when the
// next-hop sets fit one word), 0 always the chunk scan (A/B, tests).
// EngineOptions::spfQueue (engine.h), default -1

// "spf_ninfo" option: 1 (default) the queue forms keep row begin | drained
// per node in LDS, 0 read them from the CSR (L2) -- 4 B/node less LDS, more
// units per CU --, -1 the CSR form whenever that raises the units per CU.
// EngineOptions::spfNinfo (engine.h), default 1

bool ninfo_in_lds(uint32_t Sn, int W) {
  if (opts().spfNinfo >= 0) return opts().spfNinfo != 0;
  constexpr uint32_t kCu = 160u * 1024u;
  return kCu / frontier_lds_bytes(Sn, W, true, true) >=
      kCu / frontier_lds_bytes(Sn, W, true, false);
}

// 0 chunk scan, 1 two-phase queue, 2 packed one-phase queue
int queue_mode(const ogs_graph& g, int W) {
  if (opts().spfQueue == 0 || g.max_nodes > 65535) return 0;
  if (frontier_lds_bytes(uint32_t(g.max_nodes), W, true) > 160u * 1024u) return 0;
  if (g.max_degree > 16) return 0;
  return W != 1 ? 1 : 2;
}

template <int W, bool ROUTES, bool MODS, bool DIFF, int QMODE, bool OUTS3 = false,
          int B = kBlock>
hipError_t launch_frontier_q(const ogs_graph& g, const ogs_prefix_table& pt,
                             const uint32_t* key, const uint64_t* chunks,
                             const uint32_t* nChunk, const ogs_unit* units,
                             int nUnits, uint32_t flags, uint32_t* dist,
                             uint32_t* nh, const ogs_spf_out& out,
                             hipStream_t stream, const ogs_unit_mods& mods,
                             const ogs_route_diff& diff, int parts = 1) {
  const bool scan = QMODE == 0 || QMODE == 4;  // chunk-scan forms: no lists
  const bool ninfo = scan || ninfo_in_lds(uint32_t(g.max_nodes), W);
  uint32_t lds =
      frontier_lds_bytes(uint32_t(g.max_nodes), W, !scan, ninfo, QMODE == 4);
  if (!ninfo) flags |= kFlagNinfoGlobal;
  if (!opts().spfSeedRow) flags |= kFlagScanRound1;
  if (opts().spfLaneWalk == 0 || (opts().spfLaneWalk < 0 && B < 512)) flags |= kFlagSlotWalk;
  if (!opts().spfPreload) flags |= kFlagNoPreload;
  if (opts().routeStoreNt & 1) flags |= kFlagNtStores;
  auto k = spf_frontier_kernel<W, ROUTES, MODS, DIFF, QMODE, OUTS3, B>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       int(lds));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(unsigned(nUnits) * unsigned(parts)), dim3(B), lds, stream, g, pt,
                     key, chunks, nChunk, chunk_cap(g), units, flags, dist, nh, out, mods,
                     diff, uint32_t(parts));
  return hipGetLastError();
}

// Geometry of an all-sources RouteDb launch (OUTS3): threads per workgroup
// and workgroups per unit. A whole-node build (C3 at N = 1: 1,824 + 256
// units) keeps 7 one-word units resident per CU, so 256-thread workgroups
// and one per unit fill the chip and HBM is the bound. One rank's shard at
// N = 4 / 8 (520 / 260 units on 256 CUs) leaves a CU one or two units: a
// unit's single workgroup then streams its 2.5-4.2 MB latency-bound (four
// waves, one key load in flight each) and the three-word units, 1.67x the
// bytes of the others, form the tail. There the stream is split over
// `parts` workgroups per unit, each running the SPF (L2-served, ~5 rounds)
// and writing one prefix range; wider units get proportionally more parts.
// Options "frontier_block" (0 auto, 256 / 512 / 1024), "frontier_parts"
// (workgroups per one-word unit, 0 auto) and "frontier_parts_wide" (per
// unit of wider next-hop sets, 0 auto) override the choice.
// EngineOptions::frontierBlock (engine.h), default 0
// EngineOptions::frontierParts (engine.h), default 0
// EngineOptions::frontierPartsWide (engine.h), default 0

namespace {
int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        n > 0) {
      cus = n;
    } else {
      cus = 256;
    }
  }
  return cus;
}
}  // namespace

// Workgroups per unit of the split stream (route_stream 4, after the LDS
// SPF). A launch of fewer than two units per CU (one rank's shard) splits
// each unit's records into parts of about 1 MiB, so the parts of every
// width group stream comparable bytes and outlast no one; larger launches
// keep one workgroup per unit ("frontier_parts" / "frontier_parts_wide"
// override, as for the fused launches).
void stream_parts(int nUnits, int W, int P, int* parts) {
  int k = W > 1 ? opts().frontierPartsWide : opts().frontierParts;
  if (!k) {
    const double unitBytes = double(P) * (8 + 4 * W);
    k = nUnits >= 2 * num_cus()
            ? 1
            : std::max(1, std::min(16, int(unitBytes / double(1u << 20) + 0.5)));
  }
  *parts = k;
}

void stream_geometry(int nUnits, int W, int* block, int* parts) {
  // the launch's streamed bytes per CU, in one-word units (12 B per prefix)
  const double load = double(nUnits) * (8 + 4 * W) / 12.0 / num_cus();
  int b = opts().frontierBlock, k = W > 1 ? opts().frontierPartsWide : opts().frontierParts;
  // Tuned on the C3 shards (profiles/r04_geometry_ab.log), where the one-
  // word group (load 7.1 / 3.6 / 1.8 / 0.9 at N = 1 / 2 / 4 / 8) runs beside
  // the three-word group (1.7 / 0.8 / 0.4 / 0.2) on a second stream: each
  // launch sizes itself by its own load.
  if (!b) b = load >= (W > 1 ? 1.2 : 5.0) ? 256 : 512;
  if (!k) {
    k = W > 1 ? std::max(1, std::min(8, int(0.83 / load + 0.5)))
              : (load >= 1.2 ? 1 : 2);
  }
  *block = b;
  *parts = k;
}

template <int W, bool ROUTES, bool MODS = false, bool DIFF = false>
hipError_t launch_frontier(const ogs_graph& g, const ogs_prefix_table& pt,
                           const uint32_t* key, const uint64_t* chunks,
                           const uint32_t* nChunk, const ogs_unit* units,
                           int nUnits, uint32_t flags, uint32_t* dist,
                           uint32_t* nh, const ogs_spf_out& out,
                           hipStream_t stream, const ogs_unit_mods& mods = {},
                           const ogs_route_diff& diff = {}) {
  const int qm = queue_mode(g, W);
  // chunk scan with one-word next-hop sets: the one-phase packed form
  constexpr int kScanMode = W == 1 ? 4 : 0;
  const bool packedScan = W == 1 && opts().spfPackedScan && qm == 0;
  // the all-sources RouteDb stream writes exactly meta / metric / mask:
  // unconditional stores (stream_routes OUTS3), geometry by stream_geometry
  if constexpr (ROUTES && !MODS && !DIFF) {
    if (qm == 0 && out.meta && out.metric && out.mask && !out.sel) {
      int b = kBlock, k = 1;
      stream_geometry(nUnits, W, &b, &k);
      auto go = [&](auto qmode, auto block) {
        return launch_frontier_q<W, ROUTES, MODS, DIFF, decltype(qmode)::value, true,
                                 decltype(block)::value>(
            g, pt, key, chunks, nChunk, units, nUnits, flags, dist, nh, out, stream, mods,
            diff, k);
      };
      using Q4 = std::integral_constant<int, kScanMode>;
      using Q0 = std::integral_constant<int, 0>;
      using B2 = std::integral_constant<int, 256>;
      using B5 = std::integral_constant<int, 512>;
      using B10 = std::integral_constant<int, 1024>;
      if (packedScan) {
        return b == 1024 ? go(Q4{}, B10{}) : b == 512 ? go(Q4{}, B5{}) : go(Q4{}, B2{});
      }
      return b == 1024 ? go(Q0{}, B10{}) : b == 512 ? go(Q0{}, B5{}) : go(Q0{}, B2{});
    }
  }
  if (packedScan) {
    return launch_frontier_q<W, ROUTES, MODS, DIFF, kScanMode>(
        g, pt, key, chunks, nChunk, units, nUnits, flags, dist, nh, out, stream, mods, diff);
  }
  if constexpr (W == 1) {
    if (qm == 2) {
      return launch_frontier_q<W, ROUTES, MODS, DIFF, 2>(
          g, pt, key, chunks, nChunk, units, nUnits, flags, dist, nh, out, stream,
          mods, diff);
    }
  }
  if (qm != 0) {
    return launch_frontier_q<W, ROUTES, MODS, DIFF, 1>(
        g, pt, key, chunks, nChunk, units, nUnits, flags, dist, nh, out, stream,
        mods, diff);
  }
  return launch_frontier_q<W, ROUTES, MODS, DIFF, 0>(
      g, pt, key, chunks, nChunk, units, nUnits, flags, dist, nh, out, stream,
      mods, diff);
}

// "spf_frontier" option: 1 (default) large topologies use this kernel for
// their SPF, 0 the multi-source edge sweep (spf_route_ms.hip).
// EngineOptions::spfFrontier (engine.h), default 1

bool frontier_fits(const ogs_graph& g, uint32_t flags, int W) {
  if (!opts().spfFrontier || (flags & OGS_F_WIDE_METRIC)) return false;
  if (g.max_nodes > 30000 || g.max_degree > OGS_MAX_DEGREE) return false;  // u16 stamps
  return frontier_lds_bytes(uint32_t(g.max_nodes), W) <= 160u * 1024u;
}

// Scratch of the chunk lists of every topology of the batch.
size_t chunk_scratch_bytes(const ogs_graph& g) {
  return (size_t(g.num_topos) * chunk_cap(g) * 8 + size_t(g.num_topos) * 4 + 255) &
      ~size_t(255);
}

hipError_t prep_chunks(const ogs_graph& g, void* scratch, hipStream_t stream,
                       uint64_t** chunks, uint32_t** nChunk) {
  *chunks = static_cast<uint64_t*>(scratch);
  *nChunk = reinterpret_cast<uint32_t*>(*chunks + size_t(g.num_topos) * chunk_cap(g));
  hipLaunchKernelGGL(chunk_prep_kernel, dim3(g.num_topos), dim3(kBlock), 0, stream,
                     g, chunk_cap(g), *chunks, *nChunk);
  return hipGetLastError();
}

// SPF only over chunk lists already prepared (prep_chunks) in `scratch`
// (dist / next-hop sets of unit i at dist + i * Sn, nh + i * W * Sn).
hipError_t launch_frontier_spf_prepared(const ogs_graph& g, const ogs_unit* units,
                                        int nUnits, uint32_t flags, int W, uint32_t* dist,
                                        uint32_t* nh, void* scratch, hipStream_t stream) {
  uint64_t* chunks = static_cast<uint64_t*>(scratch);
  const uint32_t* nChunk =
      reinterpret_cast<const uint32_t*>(chunks + size_t(g.num_topos) * chunk_cap(g));
  const ogs_prefix_table pt{};
  const ogs_spf_out none{};
  switch (W) {
    case 1: return launch_frontier<1, false>(g, pt, nullptr, chunks, nChunk, units, nUnits, flags, dist, nh, none, stream);
    case 2: return launch_frontier<2, false>(g, pt, nullptr, chunks, nChunk, units, nUnits, flags, dist, nh, none, stream);
    case 3: return launch_frontier<3, false>(g, pt, nullptr, chunks, nChunk, units, nUnits, flags, dist, nh, none, stream);
    case 4: return launch_frontier<4, false>(g, pt, nullptr, chunks, nChunk, units, nUnits, flags, dist, nh, none, stream);
    case 8: return launch_frontier<8, false>(g, pt, nullptr, chunks, nChunk, units, nUnits, flags, dist, nh, none, stream);
    default: return hipErrorInvalidValue;
  }
}

// SPF only (dist / next-hop sets to HBM); `scratch` holds
// chunk_scratch_bytes(g). Call only when frontier_fits().
hipError_t launch_frontier_spf(const ogs_graph& g, const ogs_unit* units,
                               int nUnits, uint32_t flags, int W,
                               uint32_t* dist, uint32_t* nh, void* scratch,
                               hipStream_t stream) {
  uint64_t* chunks = nullptr;
  uint32_t* nChunk = nullptr;
  hipError_t e = prep_chunks(g, scratch, stream, &chunks, &nChunk);
  if (e != hipSuccess) return e;
  return launch_frontier_spf_prepared(g, units, nUnits, flags, W, dist, nh, scratch, stream);
}

// Fused frontier SPF + RouteDb stream (key = pfx_key_kernel output). W is
// 1, 2, 3 or 4 (3: sources of 65..96 links write three mask words, not four).
hipError_t launch_frontier_routes(const ogs_graph& g, const ogs_prefix_table& pt,
                                  const uint32_t* key, const ogs_unit* units,
                                  int nUnits, uint32_t flags, int W,
                                  const ogs_spf_out& out, void* scratch,
                                  hipStream_t stream) {
  uint64_t* chunks = nullptr;
  uint32_t* nChunk = nullptr;
  hipError_t e = prep_chunks(g, scratch, stream, &chunks, &nChunk);
  if (e != hipSuccess) return e;
  uint32_t* dist = static_cast<uint32_t*>(out.dist);
  switch (W) {
    case 1: return launch_frontier<1, true>(g, pt, key, chunks, nChunk, units, nUnits, flags, dist, out.nh, out, stream);
    case 2: return launch_frontier<2, true>(g, pt, key, chunks, nChunk, units, nUnits, flags, dist, out.nh, out, stream);
    case 3: return launch_frontier<3, true>(g, pt, key, chunks, nChunk, units, nUnits, flags, dist, out.nh, out, stream);
    case 4: return launch_frontier<4, true>(g, pt, key, chunks, nChunk, units, nUnits, flags, dist, out.nh, out, stream);
    default: return hipErrorInvalidValue;
  }
}

// ---- incremental link-failure variants (OGS_F_INCREMENTAL) -----------------
// A failed link changes nothing unless one of its directed edges is tight in
// the base SPF (base dist(u) + w == base dist(v), u relaxing): removing
// edges only lengthens paths, so a node whose base shortest-path DAG does
// not reach it through a failed tight edge keeps its distance, its tight
// predecessors and (by induction) its next-hop set. The variant's SPF is
// the base state with A = the failed tight edges' heads and their
// descendants in that DAG reset to unreachable and re-relaxed from A's
// boundary (packed queue rounds, same fixpoint as a full run: the boundary
// pushes its final words, A's nodes converge as in queue_spf_packed). Only
// prefixes with an advertiser in A can change route (a route depends on its
// advertisers' dist / next-hop sets: SpfSolver.cpp:160-311).
// LDS: dn64 [Sn] | stamp [Sn] | two u16 node lists [Sn] | A bitset.
// Descendant sets of the base tight DAG, one row per node (bit t of row v:
// t is reachable from v over base-tight edges (x -> t: x relaxes, the edge is
// up, base dist(x) + w == base dist(t))), v included. One wavefront per v,
// breadth-first in LDS. With these rows a variant's A is the OR of its
// seeds' rows -- no growth rounds in the repair kernel. Built once per
// launch over the base unit (units[0]); topologies up to kDescMaxN nodes.
constexpr uint32_t kDescMaxN = 16384;

__global__ __launch_bounds__(64) void tight_desc_kernel(ogs_graph g,
                                                        const ogs_unit* __restrict__ units,
                                                        uint32_t flags,
                                                        const uint32_t* __restrict__ bD,
                                                        uint32_t* __restrict__ desc,
                                                        uint32_t words) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int lane = threadIdx.x;
  const ogs_unit unit = units[0];
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const uint32_t v = blockIdx.x;
  if (v >= N) return;
  const uint32_t s = unit.src;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint64_t* __restrict__ edges = g.edges + e0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* bits = reinterpret_cast<uint32_t*>(smem);          // [words]
  uint16_t* q0 = reinterpret_cast<uint16_t*>(bits + words);    // [N]
  uint16_t* q1 = q0 + ((N + 1u) & ~1u);                        // [N]
  __shared__ uint32_t cnt;
  for (uint32_t w = lane; w < words; w += 64) bits[w] = 0u;
  if (lane == 0) cnt = 0u;
  __syncthreads();
  if (lane == 0) {
    bits[v >> 5] = 1u << (v & 31u);
    q0[0] = uint16_t(v);
  }
  __syncthreads();
  uint32_t n = 1;
  for (uint32_t r = 0; n; ++r) {
    const uint16_t* cur = (r & 1) ? q1 : q0;
    uint16_t* nxt = (r & 1) ? q0 : q1;
    for (uint32_t i = lane; i < n; i += 64) {
      const uint32_t x = cur[i];
      if (x != s && (nflags[x] & OGS_NODE_OVERLOADED)) continue;  // relaxes nothing
      const uint32_t dx = bD[x];
      if (dx == kInf) continue;
      const uint32_t b = gRow[x] - e0;
      for_row(edges, b, gRow[x + 1] - e0 - b, [&](uint32_t, uint64_t y) {
        const uint32_t lo = static_cast<uint32_t>(y);
        if (lo & OGS_EDGE_DOWN) return;
        const uint32_t t = edge_dst(lo);
        if (dx + (hop ? 1u : static_cast<uint32_t>(y >> 32)) != bD[t]) return;
        const uint32_t m = 1u << (t & 31u);
        if (!(atomicOr(&bits[t >> 5], m) & m)) nxt[atomicAdd(&cnt, 1u)] = uint16_t(t);
      });
    }
    __syncthreads();
    n = cnt;
    __syncthreads();
    if (lane == 0) cnt = 0u;
    __syncthreads();
  }
  uint32_t* row = desc + size_t(v) * words;
  for (uint32_t w = lane; w < words; w += 64) row[w] = bits[w];
}

// "c4_desc" option: 1 (default) the repair's A from precomputed descendant
// rows where the topology has <= kDescMaxN nodes, 0 the growth rounds (A/B)
// EngineOptions::c4Desc (engine.h), default 1

// scratch the descendant rows need (0: not used for this graph)
size_t desc_scratch_bytes(const ogs_graph& g) {
  const uint32_t Sn = uint32_t(g.max_nodes);
  if (!opts().c4Desc || Sn > kDescMaxN) return 0;
  return size_t(Sn) * ((Sn + 31u) / 32u) * 4u;
}

uint32_t repair_lds_bytes(uint32_t Sn) {
  return 8u * Sn + 4u * ((Sn + 3u) & ~3u) + 2u * 2u * ((Sn + 1u) & ~1u) +
      4u * ((Sn + 31u) / 32u) + 16u;
}

template <bool CHANGED_ONLY>
__global__ __launch_bounds__(kBlock) void spf_variant_repair_kernel(
    ogs_graph g, ogs_prefix_table pt, const uint32_t* __restrict__ key,
    const ogs_unit* __restrict__ units, uint32_t flags, uint32_t* __restrict__ oDist,
    uint32_t* __restrict__ oNh, ogs_spf_out out, ogs_unit_mods mods,
    ogs_route_diff diff, const uint32_t* __restrict__ desc) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  const uint32_t u0 = blockIdx.x;
  const ogs_unit unit = units[u0];
  const uint32_t s = unit.src;
  const uint32_t nb = g.node_base[unit.topo];
  const uint32_t N = g.node_base[unit.topo + 1] - nb;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint64_t* __restrict__ edges = g.edges + e0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const uint32_t Sn = uint32_t(g.max_nodes);
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0;
  const uint32_t* __restrict__ bD = diff.base_dist;
  const uint32_t* __restrict__ bN = diff.base_nh;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* dn = reinterpret_cast<uint64_t*>(smem);                      // [Sn]
  uint32_t* stamp = reinterpret_cast<uint32_t*>(dn + Sn);                // [Sn]
  uint16_t* q0 = reinterpret_cast<uint16_t*>(stamp + ((Sn + 3u) & ~3u));  // [Sn]
  uint16_t* q1 = q0 + ((Sn + 1u) & ~1u);                                 // [Sn]
  uint32_t* inA = reinterpret_cast<uint32_t*>(q1 + ((Sn + 1u) & ~1u));   // [Sn/32]
  __shared__ uint32_t qcnt[3], cnt[2];
  auto isA = [&](uint32_t v) { return (inA[v >> 5] >> (v & 31u)) & 1u; };
  auto relaxes = [&](uint32_t v) { return v == s || !(nflags[v] & OGS_NODE_OVERLOADED); };

  DeadEdges dead;
#pragma unroll
  for (int k = 0; k < kMaxDead; ++k) {
    dead.e[k] = k < mods.dead_per_unit ? mods.dead_edges[size_t(u0) * mods.dead_per_unit + k]
                                       : OGS_NODE_NONE;
  }
  for (uint32_t w = tid; w < (N + 31u) / 32u; w += kBlock) inA[w] = 0u;
  if (tid < 3) qcnt[tid] = 0u;
  if (tid < 2) cnt[tid] = 0u;
  __syncthreads();
  // ---- seeds: heads of the failed edges that are tight in the base --------
  // (the seed's edge straight from the list: indexing `dead` by tid would put
  // the array in scratch memory, and every edge test of the rounds with it)
  const uint32_t seedEdge = (tid < kMaxDead && tid < mods.dead_per_unit)
      ? mods.dead_edges[size_t(u0) * mods.dead_per_unit + tid]
      : OGS_NODE_NONE;
  if (seedEdge != OGS_NODE_NONE) {
    const uint32_t e = seedEdge;
    const uint32_t u = g.edge_src[e0 + e];
    const uint64_t x = edges[e];
    const uint32_t lo = static_cast<uint32_t>(x);
    const uint32_t v = edge_dst(lo);
    const uint32_t w = hop ? 1u : static_cast<uint32_t>(x >> 32);
    if (!(lo & OGS_EDGE_DOWN) && relaxes(u) && bD[u] != kInf && bD[u] + w == bD[v]) {
      if (!(atomicOr(&inA[v >> 5], 1u << (v & 31u)) & (1u << (v & 31u)))) {
        q1[atomicAdd(&qcnt[1], 1u)] = uint16_t(v);
      }
    }
  }
  __syncthreads();
  uint32_t n = qcnt[1];
  if (CHANGED_ONLY && n == 0) {  // no failed link on a shortest path: no change
    if (tid < 2) diff.counts[size_t(u0) * 2 + tid] = 0u;
    if (oDist || oNh) {
      for (uint32_t v = tid; v < N; v += kBlock) {
        if (oDist) oDist[size_t(u0) * Sn + v] = bD[v];
        if (oNh) oNh[size_t(u0) * Sn + v] = bN[v];
      }
    }
    return;
  }
  for (uint32_t v = tid; v < N; v += kBlock) {
    dn[v] = uint64_t(bD[v]) | (uint64_t(bN[v]) << 32);
    stamp[v] = 0u;
  }
  if (desc) {  // ---- A = OR of the seeds' precomputed descendant rows ------
    const uint32_t words = (N + 31u) / 32u;
    for (uint32_t w = tid; w < words; w += kBlock) {
      uint32_t a = 0u;
      for (uint32_t i = 0; i < n; ++i) a |= desc[size_t(q1[i]) * words + w];
      inA[w] = a;
    }
    n = 0;
  }
  __syncthreads();
  // ---- A: the seeds' descendants in the base tight DAG (list rounds) ------
  for (uint32_t r = 1; n; ++r) {
    if (tid == 0) qcnt[(r + 2) % 3] = 0u;
    const uint16_t* cur = (r & 1) ? q1 : q0;
    uint16_t* nxt = (r & 1) ? q0 : q1;
    for (uint32_t i = tid; i < n; i += kBlock) {
      const uint32_t x = cur[i];
      if (!relaxes(x)) continue;
      const uint32_t dx = static_cast<uint32_t>(dn[x]);
      const uint32_t b = gRow[x] - e0;
      for_row(edges, b, gRow[x + 1] - e0 - b, [&](uint32_t, uint64_t y) {
        const uint32_t lo = static_cast<uint32_t>(y);
        if (lo & OGS_EDGE_DOWN) return;
        const uint32_t t = edge_dst(lo);
        if (dx + (hop ? 1u : static_cast<uint32_t>(y >> 32)) != static_cast<uint32_t>(dn[t])) {
          return;
        }
        if (!(atomicOr(&inA[t >> 5], 1u << (t & 31u)) & (1u << (t & 31u)))) {
          nxt[atomicAdd(&qcnt[(r + 1) % 3], 1u)] = uint16_t(t);
        }
      });
    }
    __syncthreads();
    n = qcnt[(r + 1) % 3];
  }
  // ---- reset A, seed its boundary, re-relax --------------------------------
  __syncthreads();  // every thread has read the last (zero) count
  if (tid < 3) qcnt[tid] = 0u;
  for (uint32_t v = tid; v < N; v += kBlock) {
    if (isA(v)) dn[v] = uint64_t(kInf);
  }
  __syncthreads();
  for (uint32_t x = tid; x < N; x += kBlock) {
    if (!isA(x)) continue;
    const uint32_t b = gRow[x] - e0, m = gRow[x + 1] - e0 - b;
    for (uint32_t j = 0; j < m; ++j) {  // links are two-way: out-neighbours = in-neighbours
      const uint32_t p = edge_dst(static_cast<uint32_t>(edges[b + j]));
      if (isA(p) || !relaxes(p) || static_cast<uint32_t>(dn[p]) == kInf) continue;
      if (atomicMax(&stamp[p], 1u) < 1u) q1[atomicAdd(&qcnt[1], 1u)] = uint16_t(p);
    }
  }
  __syncthreads();
  packed_rounds<true>(s, edges, gRow, e0, nflags, hop, dn, stamp, q0, q1, qcnt,
                             nullptr, dead, 1u, qcnt[1]);
  __syncthreads();
  if (oDist || oNh) {
    for (uint32_t v = tid; v < N; v += kBlock) {
      if (oDist) oDist[size_t(u0) * Sn + v] = static_cast<uint32_t>(dn[v]);
      if (oNh) oNh[size_t(u0) * Sn + v] = static_cast<uint32_t>(dn[v] >> 32);
    }
  }

  // ---- routes --------------------------------------------------------------
  const uint32_t Sp = uint32_t(pt.max_prefixes);
  const uint32_t p0 = pt.pfx_base[unit.topo];
  const uint32_t P = pt.pfx_base[unit.topo + 1] - p0;
  const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0, (flags & OGS_F_V4_OVER_V6) != 0,
                     (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
  const DiffCtx dc{diff.base_meta, diff.base_metric, diff.base_mask,
                   diff.changed + size_t(u0) * ((Sp + 31u) / 32u), cnt, pt.adv_off + p0,
                   diff.adv_class};
  const uint32_t* tkey = key + size_t(unit.topo) * Sp;
  auto nodeRec = [&](uint32_t v, Rec<1>& r) {
    const uint64_t x = dn[v];
    const uint32_t d = static_cast<uint32_t>(x), nv = static_cast<uint32_t>(x >> 32);
    r.meta = node_route_meta(v, s, d != kInf, __popc(nv), nflags[v]);
    r.metric = (v == s) ? kInf : d;
    r.mask[0] = nv;
  };
  if constexpr (!CHANGED_ONLY) {
    stream_routes<1, true>(pt, tkey, p0, P, Sp, u0, s, nflags, PackedView{dn}, cfg, out,
                           nodeRec, &dc, (flags & kFlagNtStores) != 0);
  } else {
    const bool v4Gated = !cfg.enableV4 && !cfg.v4OverV6;
    uint32_t upd = 0, del = 0;
    for (uint32_t p = tid; p < P; p += kBlock) {
      const uint32_t k = tkey[p];
      bool hit = false;
      if (!(k & kKeySlow)) {
        hit = isA(k & kKeyNode);
      } else {
        for (uint32_t a = pt.adv_off[p0 + p]; a < pt.adv_off[p0 + p + 1]; ++a) {
          const uint32_t v = pt.adv_node[a];
          hit |= v != OGS_NODE_NONE && isA(v);
        }
      }
      if (!hit) continue;  // every advertiser keeps its base state
      Rec<1> r;
      if (!(k & kKeySlow)) {
        if ((k & kKeyV4) && v4Gated) continue;  // the gate's record never changes
        nodeRec(k & kKeyNode, r);
        r.sel = (r.meta & OGS_ROUTE_SELECTED) ? 1u : 0u;
      } else {
        route_one<uint32_t, 1>(pt, p0 + p, s, nflags, PackedView{dn}, cfg, r.meta, r.metric,
                               r.mask, r.sel);
      }
      if (!route_changed<1>(r, dc, Sp, p, upd, del)) continue;
      atomicOr(dc.changed + p / 32u, 1u << (p % 32u));
      const size_t o = size_t(u0) * Sp + p;
      if (out.meta) out.meta[o] = r.meta;
      if (out.metric) static_cast<uint32_t*>(out.metric)[o] = r.metric;
      if (out.sel) out.sel[o] = r.sel;
      if (out.mask) out.mask[o] = r.mask[0];
    }
    if (upd) atomicAdd(&cnt[0], upd);
    if (del) atomicAdd(&cnt[1], del);
  }
  __syncthreads();
  if (tid < 2) diff.counts[size_t(u0) * 2 + tid] = cnt[tid];
}

// ogs_spf_routes_variants with OGS_F_INCREMENTAL (W = 1); false when the
// repair does not apply (the caller then runs the full recompute).
bool launch_variants_repair(const ogs_graph& g, const ogs_prefix_table& pt,
                            const uint32_t* key, const ogs_unit* units, int n,
                            uint32_t flags, int W, const ogs_spf_out& out,
                            const ogs_unit_mods* mods, ogs_route_diff* diff,
                            void* scratch, hipStream_t stream, hipError_t* err) {
  if (!(flags & OGS_F_INCREMENTAL) || !mods || !diff || !diff->base_dist || !diff->base_nh ||
      W != 1 || mods->dead_per_unit > kMaxDead || g.max_nodes > 65535) {
    return false;
  }
  const uint32_t lds = repair_lds_bytes(uint32_t(g.max_nodes));
  if (lds > 160u * 1024u) return false;
  const bool changedOnly = (flags & OGS_F_CHANGED_ONLY) != 0;
  auto k = changedOnly ? spf_variant_repair_kernel<true> : spf_variant_repair_kernel<false>;
  if (lds > 64 * 1024) {
    *err = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (*err != hipSuccess) return true;
  }
  // descendant rows of the base tight DAG (every variant shares topology,
  // source and base SPF: units[0] / diff->base_dist): from the caller's
  // cache when it holds them, else built (into the cache when given)
  uint32_t* desc = nullptr;
  const uint32_t Sn = uint32_t(g.max_nodes);
  const bool cached = desc_scratch_bytes(g) && diff->base_desc;
  if (cached && diff->base_desc_valid) {
    desc = diff->base_desc;
  } else if (desc_scratch_bytes(g) && (cached || scratch)) {
    const uint32_t words = (Sn + 31u) / 32u;
    desc = cached ? diff->base_desc : static_cast<uint32_t*>(scratch);
    const size_t dl = size_t(words) * 4u + 2u * 2u * ((Sn + 1u) & ~1u);
    hipLaunchKernelGGL(tight_desc_kernel, dim3(Sn), dim3(64), dl, stream, g, units, flags,
                       diff->base_dist, desc, words);
    *err = hipGetLastError();
    if (*err != hipSuccess) return true;
    if (cached) diff->base_desc_valid = 1;  // the caller's cache now holds them
  }
  hipLaunchKernelGGL(k, dim3(n), dim3(kBlock), lds, stream, g, pt, key, units,
                     flags | ((opts().routeStoreNt & 1) ? kFlagNtStores : 0u),
                     static_cast<uint32_t*>(out.dist), out.nh, out, *mods, *diff, desc);
  *err = hipGetLastError();
  return true;
}

// Link-failure variants with an optional route diff (fused SPF + RouteDb).
template <int W>
hipError_t launch_variants_w(const ogs_graph& g, const ogs_prefix_table& pt,
                             const uint32_t* key, const uint64_t* chunks,
                             const uint32_t* nChunk, const ogs_unit* units,
                             int n, uint32_t flags, const ogs_spf_out& out,
                             const ogs_unit_mods* mods, const ogs_route_diff* diff,
                             hipStream_t stream) {
  uint32_t* dist = static_cast<uint32_t*>(out.dist);
  const ogs_unit_mods m = mods ? *mods : ogs_unit_mods{};
  const ogs_route_diff d = diff ? *diff : ogs_route_diff{};
  if (mods && diff) return launch_frontier<W, true, true, true>(g, pt, key, chunks, nChunk, units, n, flags, dist, out.nh, out, stream, m, d);
  if (mods) return launch_frontier<W, true, true, false>(g, pt, key, chunks, nChunk, units, n, flags, dist, out.nh, out, stream, m, d);
  if (diff) return launch_frontier<W, true, false, true>(g, pt, key, chunks, nChunk, units, n, flags, dist, out.nh, out, stream, m, d);
  return launch_frontier<W, true>(g, pt, key, chunks, nChunk, units, n, flags, dist, out.nh, out, stream);
}

hipError_t launch_frontier_variants(const ogs_graph& g, const ogs_prefix_table& pt,
                                    const uint32_t* key, const ogs_unit* units,
                                    int n, uint32_t flags, int W,
                                    const ogs_spf_out& out,
                                    const ogs_unit_mods* mods,
                                    ogs_route_diff* diff, void* scratch,
                                    hipStream_t stream) {
  hipError_t e = hipSuccess;
  if (launch_variants_repair(g, pt, key, units, n, flags, W, out, mods, diff, scratch, stream,
                             &e)) {
    return e;
  }
  uint64_t* chunks = nullptr;
  uint32_t* nChunk = nullptr;
  e = prep_chunks(g, scratch, stream, &chunks, &nChunk);
  if (e != hipSuccess) return e;
  switch (W) {
    case 1: return launch_variants_w<1>(g, pt, key, chunks, nChunk, units, n, flags, out, mods, diff, stream);
    case 2: return launch_variants_w<2>(g, pt, key, chunks, nChunk, units, n, flags, out, mods, diff, stream);
    case 4: return launch_variants_w<4>(g, pt, key, chunks, nChunk, units, n, flags, out, mods, diff, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace ogs

#ifdef OGS_STAMPS
extern "C" int ogs_diag_stamps(uint32_t* host, int32_t words) {
  const size_t n = std::min<size_t>(size_t(words), size_t(ogs::kDiagWgs) * 8);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ogs::g_diagStamps), n * 4, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
