// spf_lds.hip — all-sources SPF with the topology resident in LDS (C3
// fabric: 2,080 nodes, 43,008 directed edges, every node a source).
//
// Same fixpoint as spf_frontier.hip (reference: LinkState::runSpf,
// LinkState.cpp:720-820; proof sketch in spf_core.h): distances are the least
// solution of dist(v) = min over relaxing u of dist(u) + w(u, v), next-hop
// sets the least solution of NH(v) = U over tight u of (u == src ?
// {slot(src->v)} : NH(u)). What differs is where the topology lives. The
// frontier kernel reads chunk records and edges from L2 every round, so a
// round is a chain of dependent L2 round trips -- hidden when 7 units share
// a CU (a whole-node build), exposed when one rank's shard leaves a CU one or
// two units (N = 4 / 8 GPUs: 60+ us per SPF, phase stamps in DESIGN §3.3).
// Here one 1024-thread workgroup per CU stages a compact image of the CSR
// into LDS ONCE (2 B per edge: 15-bit neighbour | down bit; chunk -> node
// table; row offsets; node flags: 124 KB for C3) and then solves its share
// of the units back to back with every round served from LDS.
//
// Edge weights: when every up edge of the topology has the same weight (the
// fabric's metric 1, or OGS_F_HOP_METRIC) that weight is a constant; other
// topologies read the weight word of each relaxed edge from the CSR (L2),
// exact either way.
//
// Outputs: dist[u*Sn + v], nh[(u*W + w)*Sn + v] (ogs_spf_out layout); the
// RouteDb stream (route_stream_kernel, any number of workgroups per unit)
// reads them back (route_stream.hip, "route_stream" option 4).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "openr_gpu.h"
#include "route_core.h"
#include "spf_core.h"

namespace ogs {

namespace {

constexpr uint32_t kDown16 = 0x8000u;     // eimg: edge down
constexpr uint32_t kNodeMax = 0x7FFFu;    // 15-bit neighbour ids
constexpr uint32_t kLdsChunk = 8;         // edges per chunk (one lane's push)
constexpr int kLdsBlock = 1024;

__host__ __device__ inline uint32_t al16(uint32_t x) { return (x + 15u) & ~15u; }

// internal launch flag: the CAS (W = 1) / two-phase (W > 1) rounds instead
// of the three-pass rounds ("spf_lds_form" option 1, A/B)
constexpr uint32_t kFlagLdsCasForm = 1u << 25;

// Byte layout of one topology's image (global, then the same block in LDS):
// header (16 B, global only) | eimg u16[E] | cnode u16[cap] | row u32[N+1] |
// first u16[N] | flags u8[N], sections 16-B aligned, sized by the batch's
// maxima so every topology (and the LDS copy) shares the offsets.
struct LdsImage {
  uint32_t eimg, cnode, row, first, flags, block;  // offsets in the block
  uint32_t state;                                  // per-unit state bytes
  uint32_t stride;                                 // header + block
};

__host__ LdsImage lds_image(const ogs_graph& g, int W) {
  const uint32_t N = uint32_t(g.max_nodes), E = uint32_t(g.max_edges);
  const uint32_t cap = E / kLdsChunk + N;
  LdsImage L{};
  L.eimg = 0;
  L.cnode = L.eimg + al16(2u * E);
  L.row = L.cnode + al16(2u * cap);
  L.first = L.row + al16(4u * (N + 1u));
  L.flags = L.first + al16(2u * N);
  L.block = L.flags + al16(N);
  // the larger of the forms' states: three-pass {dist, prev, nh[W], u8
  // stamps}; W == 1 packed {dist | nh} words + u8 stamps; W > 1 two-phase
  // {dist, nh[W], u16 stamps}
  L.state = std::max(al16(4u * N) * 2u + al16(4u * N * uint32_t(W)) + al16(N),
                     W == 1 ? al16(8u * N) + al16(N)
                            : al16(4u * N) + al16(4u * N * uint32_t(W)) + al16(2u * N));
  L.stride = 16u + L.block;
  return L;
}

// Image build, once per call: lds_scan_kernel (one workgroup per topology:
// row offsets, node flags, chunk -> node table; header {chunks, weight min,
// weight max, 0}) then lds_edges_kernel (many workgroups: the 2-B edge words
// and the min / max weight of the up edges). Header of topology t at
// img + t * L.stride; the weights are uniform iff min == max.
__global__ __launch_bounds__(kLdsBlock) void lds_scan_kernel(ogs_graph g, LdsImage L,
                                                            uint8_t* __restrict__ img) {
  constexpr uint32_t B = kLdsBlock;
  __shared__ uint32_t wsum[B / 64];
  __shared__ uint32_t base;
  const uint32_t t = blockIdx.x, tid = threadIdx.x;
  const uint32_t nb = g.node_base[t];
  const uint32_t N = g.node_base[t + 1] - nb;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  uint8_t* hdr = img + size_t(t) * L.stride;
  uint8_t* blk = hdr + 16;
  uint16_t* __restrict__ cnode = reinterpret_cast<uint16_t*>(blk + L.cnode);
  uint32_t* __restrict__ row = reinterpret_cast<uint32_t*>(blk + L.row);
  uint16_t* __restrict__ first = reinterpret_cast<uint16_t*>(blk + L.first);
  uint8_t* __restrict__ fl = blk + L.flags;
  if (tid == 0) base = 0u;
  for (uint32_t v = tid; v <= N; v += B) row[v] = gRow[v] - e0;
  for (uint32_t v = tid; v < N; v += B) fl[v] = g.node_flags[nb + v];
  __syncthreads();
  // chunk ids: exclusive scan of ceil(deg / 8) over the nodes, tile by tile
  const int lane = int(tid & 63u), wave = int(tid >> 6);
  for (uint32_t t0 = 0; t0 < N; t0 += B) {
    const uint32_t v = t0 + tid;
    const uint32_t deg = v < N ? gRow[v + 1] - gRow[v] : 0u;
    const uint32_t n = (deg + kLdsChunk - 1u) / kLdsChunk;
    uint32_t inc = n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (lane >= d) inc += y;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t off = base;
    for (int w = 0; w < wave; ++w) off += wsum[w];
    __syncthreads();
    if (tid == B - 1u) base = off + inc;
    const uint32_t at = off + inc - n;
    if (v < N) first[v] = uint16_t(at);
    for (uint32_t k = 0; k < n; ++k) cnode[at + k] = uint16_t(v);
    __syncthreads();
  }
  if (tid == 0) {
    uint32_t* h = reinterpret_cast<uint32_t*>(hdr);
    h[0] = base;
    h[1] = 0xFFFFFFFFu;  // weight min / max of the up edges (lds_edges_kernel)
    h[2] = 0u;
    h[3] = 0u;
  }
}

constexpr uint32_t kEdgesPerThread = 8;

__global__ __launch_bounds__(kBlock) void lds_edges_kernel(ogs_graph g, LdsImage L,
                                                          uint8_t* __restrict__ img) {
  const uint32_t t = blockIdx.y;
  const uint32_t nb = g.node_base[t];
  const uint32_t N = g.node_base[t + 1] - nb;
  const uint32_t e0 = g.row_ptr[nb];
  const uint32_t E = g.row_ptr[nb + N] - e0;
  uint8_t* hdr = img + size_t(t) * L.stride;
  uint16_t* __restrict__ eimg = reinterpret_cast<uint16_t*>(hdr + 16 + L.eimg);
  const uint64_t* __restrict__ edges = g.edges + e0;
  const uint32_t base = blockIdx.x * kBlock * kEdgesPerThread + threadIdx.x;
  uint64_t x[kEdgesPerThread];
#pragma unroll
  for (uint32_t k = 0; k < kEdgesPerThread; ++k) {
    const uint32_t e = base + k * kBlock;
    x[k] = e < E ? edges[e] : uint64_t(OGS_EDGE_DOWN);
  }
  uint32_t lo = 0xFFFFFFFFu, hi = 0u;
#pragma unroll
  for (uint32_t k = 0; k < kEdgesPerThread; ++k) {
    const uint32_t e = base + k * kBlock;
    const uint32_t w = static_cast<uint32_t>(x[k]);
    const bool down = (w & OGS_EDGE_DOWN) != 0u;
    if (e < E) eimg[e] = uint16_t(edge_dst(w) | (down ? kDown16 : 0u));
    if (!down) {
      lo = min(lo, static_cast<uint32_t>(x[k] >> 32));
      hi = max(hi, static_cast<uint32_t>(x[k] >> 32));
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    lo = min(lo, __shfl_xor(lo, d, 64));
    hi = max(hi, __shfl_xor(hi, d, 64));
  }
  if ((threadIdx.x & 63u) == 0u) {
    uint32_t* h = reinterpret_cast<uint32_t*>(hdr);
    if (lo != 0xFFFFFFFFu) atomicMin(&h[1], lo);
    if (hi != 0u) atomicMax(&h[2], hi);
  }
}

#ifdef OGS_STAMPS
// diagnostic build: per workgroup {staging, first unit's SPF, rounds, the
// first unit's round 2..9 cycles, units, kernel cycles, 0...} (16 words),
// rows (W - 1) * 4096 + blockIdx.x; read with ogs_diag_lds_stamps
constexpr uint32_t kLdsDiagWgs = 4096;
__device__ uint32_t g_ldsStamps[4 * kLdsDiagWgs * 16];
#endif

// SPF of the workgroup's units over the LDS image. W == 1: packed
// {dist, next-hop word} per node, one phase (every push a 64-bit LDS
// compare-and-swap: a shorter candidate replaces, an equal one ORs its
// bits in). W > 1: a distance phase (atomicMin), then a next-hop phase
// (atomicOr along tight edges), as frontier_spf.
template <int W>
__global__ __launch_bounds__(kLdsBlock) void spf_lds_kernel(
    ogs_graph g, LdsImage L, const uint8_t* __restrict__ img,
    const ogs_unit* __restrict__ units, int nUnits, uint32_t flags,
    uint32_t* __restrict__ oDist, uint32_t* __restrict__ oNh) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  constexpr uint32_t B = kLdsBlock;
  const uint32_t tid = threadIdx.x;
  const uint32_t Sn = uint32_t(g.max_nodes);
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0u;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* blk = smem;
  const uint16_t* eimg = reinterpret_cast<const uint16_t*>(blk + L.eimg);
  const uint16_t* cnode = reinterpret_cast<const uint16_t*>(blk + L.cnode);
  const uint32_t* row = reinterpret_cast<const uint32_t*>(blk + L.row);
  const uint16_t* first = reinterpret_cast<const uint16_t*>(blk + L.first);
  const uint8_t* nfl = reinterpret_cast<const uint8_t*>(blk + L.flags);
  char* st = blk + L.block;
  // three-pass form (default)
  uint32_t* prev = reinterpret_cast<uint32_t*>(st + al16(4u * Sn));
  uint32_t* nh3 = reinterpret_cast<uint32_t*>(st + 2u * al16(4u * Sn));
  uint8_t* stamp3 = reinterpret_cast<uint8_t*>(st + 2u * al16(4u * Sn) + al16(4u * Sn * W));
  const bool threePass = (flags & kFlagLdsCasForm) == 0u;
  // W == 1 packed form
  uint64_t* dn = reinterpret_cast<uint64_t*>(st);
  uint8_t* stamp8 = reinterpret_cast<uint8_t*>(st + al16(8u * Sn));
  // W > 1
  uint32_t* dist = reinterpret_cast<uint32_t*>(st);
  uint32_t* nh = reinterpret_cast<uint32_t*>(st + al16(4u * Sn));
  uint16_t* stamp16 = reinterpret_cast<uint16_t*>(st + al16(4u * Sn) + al16(4u * Sn * W));

  uint32_t staged = 0xFFFFFFFFu;
  uint32_t C = 0, uniform = 0, w0 = 0, N = 0, e0 = 0;
#ifdef OGS_STAMPS
  uint32_t diag[16] = {};
  const uint64_t k0 = __builtin_amdgcn_s_memtime();
  uint64_t tr = k0;
  bool firstUnit = true;
  auto mark = [&](int slot) {  // cycles since the last mark of the first unit
    const uint64_t now = __builtin_amdgcn_s_memtime();
    if (firstUnit && slot < 16) diag[slot] = uint32_t(now - tr);
    tr = now;
  };
#else
  auto mark = [](int) {};
#endif
  for (int u = int(blockIdx.x); u < nUnits; u += int(gridDim.x)) {
    const ogs_unit unit = units[u];
    if (unit.topo != staged) {
      __syncthreads();  // the previous unit's state reads are done
      const uint8_t* hdr = img + size_t(unit.topo) * L.stride;
      const uint4* src = reinterpret_cast<const uint4*>(hdr + 16);
      uint4* dst = reinterpret_cast<uint4*>(blk);
      for (uint32_t i = tid; i < L.block / 16u; i += B) dst[i] = src[i];
      const uint32_t* h = reinterpret_cast<const uint32_t*>(hdr);
      C = h[0];
      uniform = h[1] == h[2] ? 1u : 0u;  // every up edge of this weight
      w0 = h[1];
      const uint32_t nb = g.node_base[unit.topo];
      N = g.node_base[unit.topo + 1] - nb;
      e0 = g.row_ptr[nb];
      staged = unit.topo;
      __syncthreads();
    }
    mark(0);  // staging (the first unit only)
    const uint64_t* __restrict__ edges = g.edges + e0;
    auto weight = [&](uint32_t e) -> uint32_t {
      return hop ? 1u : uniform ? w0 : static_cast<uint32_t>(edges[e] >> 32);
    };
    const uint32_t s = unit.src;
    const uint32_t sb = row[s], se = row[s + 1];
    if (threePass) {
      // One phase without compare-and-swap: every round is (1) atomicMin of
      // the active nodes' candidates into dist, (2) a node pass -- a node
      // whose distance fell drops its next hops and is stamped for the next
      // round --, (3) atomicOr of the active nodes' next hops along the edges
      // that are tight NOW. A push from a longer stale distance ORs nothing
      // (not tight), a node whose bits grew is stamped too: the least
      // fixpoint of spf_core.h, in the rounds of the packed form, with
      // fire-and-forget LDS atomics instead of contended CAS loops.
      for (uint32_t v = tid; v < N; v += B) {
        dist[v] = (v == s) ? 0u : kInf;
        prev[v] = dist[v];
        stamp3[v] = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) nh3[v * W + w] = 0u;
      }
      __syncthreads();
      auto nodePass = [&](uint32_t r, bool& changed) {
        for (uint32_t v = tid; v < N; v += B) {
          const uint32_t d = dist[v];
          if (d < prev[v]) {
            prev[v] = d;
#pragma unroll
            for (int w = 0; w < W; ++w) nh3[v * W + w] = 0u;
            stamp3[v] = uint8_t(r + 1u);
            changed = true;
          }
        }
      };
      // round 1: the source's row (slot j = j-th edge of the row)
      {
        bool changed = false;
        for (uint32_t j = tid; j < se - sb; j += B) {
          const uint32_t x = eimg[sb + j];
          if (x & kDown16) continue;
          atomicMin(&dist[x & kNodeMax], weight(sb + j));
        }
        __syncthreads();
        nodePass(1u, changed);
        __syncthreads();
        for (uint32_t j = tid; j < se - sb && j < 32u * W; j += B) {
          const uint32_t x = eimg[sb + j];
          if (x & kDown16) continue;
          const uint32_t t = x & kNodeMax;
          if (weight(sb + j) != dist[t]) continue;
          atomicOr(&nh3[t * W + (j >> 5)], 1u << (j & 31u));
          stamp3[t] = 2;
        }
        __syncthreads();
      }
      // the thread's chunk slots whose node is stamped for round r and
      // relaxes (LinkState.cpp:741-752: not a hard-drained node other than
      // the source; the source itself is never stamped again)
      auto scan = [&](uint32_t r, auto&& fn) {
        for (uint32_t c0 = tid; c0 < C; c0 += 4u * B) {
          uint32_t cs[4], vs[4];
          bool act[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            cs[k] = c0 + uint32_t(k) * B;
            vs[k] = cs[k] < C ? cnode[cs[k]] : 0u;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            act[k] = cs[k] < C && stamp3[vs[k]] == uint8_t(r) &&
                !(nfl[vs[k]] & OGS_NODE_OVERLOADED);
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (act[k]) fn(cs[k], vs[k]);
          }
        }
      };
      auto edges8 = [&](uint32_t c, uint32_t v, uint32_t (&x)[kLdsChunk],
                        uint32_t (&dt)[kLdsChunk]) {
        const uint32_t b = row[v] + kLdsChunk * (c - first[v]);
        const uint32_t n = min(kLdsChunk, row[v + 1] - b);
#pragma unroll
        for (uint32_t i = 0; i < kLdsChunk; ++i) x[i] = i < n ? eimg[b + i] : kDown16;
#pragma unroll
        for (uint32_t i = 0; i < kLdsChunk; ++i) dt[i] = dist[x[i] & kNodeMax];
        return b;
      };
      for (uint32_t r = 2;; ++r) {
        bool changed = false;
        scan(r, [&](uint32_t c, uint32_t v) {  // (1) distances
          const uint32_t dv = dist[v];
          uint32_t x[kLdsChunk], dt[kLdsChunk];
          const uint32_t b = edges8(c, v, x, dt);
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) {
            if (x[i] & kDown16) continue;
            const uint32_t cand = dv + weight(b + i);
            if (cand < dt[i]) atomicMin(&dist[x[i] & kNodeMax], cand);
          }
        });
        __syncthreads();
        nodePass(r, changed);  // (2)
        __syncthreads();
        scan(r, [&](uint32_t c, uint32_t v) {  // (3) next hops along tight edges
          const uint32_t dv = dist[v];
          uint32_t nv[W];
#pragma unroll
          for (int w = 0; w < W; ++w) nv[w] = nh3[v * W + w];
          uint32_t x[kLdsChunk], dt[kLdsChunk];
          const uint32_t b = edges8(c, v, x, dt);
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) {
            if ((x[i] & kDown16) || dv + weight(b + i) != dt[i]) continue;
            const uint32_t t = x[i] & kNodeMax;
            bool add = false;
#pragma unroll
            for (int k = 0; k < W; ++k) {
              const uint32_t a = nv[k] & ~nh3[t * W + k];
              if (a) {
                atomicOr(&nh3[t * W + k], a);
                add = true;
              }
            }
            if (add) {
              stamp3[t] = uint8_t(r + 1u);
              changed = true;
            }
          }
        });
        const bool more = __syncthreads_or(changed) != 0;
        mark(int(r) + 1);
#ifdef OGS_STAMPS
        if (firstUnit) diag[2] = r;
#endif
        if (!more) break;
      }
      for (uint32_t v = tid; v < N; v += B) {
        oDist[size_t(u) * Sn + v] = dist[v];
#pragma unroll
        for (int w = 0; w < W; ++w) oNh[(size_t(u) * W + w) * Sn + v] = nh3[v * W + w];
      }
    } else if constexpr (W == 1) {
      for (uint32_t v = tid; v < N; v += B) {
        dn[v] = (v == s) ? 0ull : uint64_t(kInf);
        stamp8[v] = (v == s) ? 1 : 0;
      }
      __syncthreads();
      // one push of edge e (local id) from v {dv, bits} in round r
      auto push = [&](uint32_t e, uint32_t dv, uint32_t bits, uint32_t r,
                      bool& changed) {
        const uint32_t x = eimg[e];
        if (x & kDown16) return;
        const uint32_t t = x & kNodeMax;
        const uint32_t c = dv + weight(e);
        uint64_t old = dn[t];
        for (;;) {
          const uint32_t dt = static_cast<uint32_t>(old), nt = static_cast<uint32_t>(old >> 32);
          if (c > dt || (c == dt && !(bits & ~nt))) return;
          const uint64_t nw = c < dt ? (uint64_t(c) | (uint64_t(bits) << 32))
                                     : (uint64_t(dt) | (uint64_t(nt | bits) << 32));
          const uint64_t seen = atomicCAS(reinterpret_cast<unsigned long long*>(&dn[t]),
                                          static_cast<unsigned long long>(old),
                                          static_cast<unsigned long long>(nw));
          if (seen == old) {
            stamp8[t] = uint8_t(r + 1u);
            changed = true;
            return;
          }
          old = seen;
        }
      };
      // round 1: the source's row, one edge per thread (slot j = j-th edge)
      {
        bool changed = false;
        for (uint32_t j = tid; j < se - sb; j += B) {
          push(sb + j, 0u, j < 32u ? 1u << j : 0u, 1u, changed);
        }
        __syncthreads();
      }
      const uint32_t* dn32 = reinterpret_cast<const uint32_t*>(dn);  // dist = low word
      for (uint32_t r = 2;; ++r) {
        bool changed = false;
        // one chunk of v: its 8 edge words and their targets' distances read
        // first (independent LDS reads), then a compare-and-swap only where
        // the push can change the target (distances only fall, so a stale
        // preload never drops a useful push)
        auto chunk = [&](uint32_t c, uint32_t v) {
          const uint64_t xv = dn[v];
          const uint32_t dv = static_cast<uint32_t>(xv), nv = static_cast<uint32_t>(xv >> 32);
          const uint32_t b = row[v] + kLdsChunk * (c - first[v]);
          const uint32_t n = min(kLdsChunk, row[v + 1] - b);
          uint32_t x[kLdsChunk], dt[kLdsChunk];
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) x[i] = i < n ? eimg[b + i] : kDown16;
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) dt[i] = dn32[2u * (x[i] & kNodeMax)];
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) {
            if (x[i] & kDown16) continue;
            const uint32_t cand = dv + weight(b + i);
            if (cand > dt[i]) continue;
            // the source contributes its link slot, others NH(v) (LinkState.cpp:808-811)
            const uint32_t slot = b + i - sb;
            const uint32_t bits = v == s ? (slot < 32u ? 1u << slot : 0u) : nv;
            const uint32_t t = x[i] & kNodeMax;
            uint64_t old = dn[t];
            for (;;) {
              const uint32_t d0 = static_cast<uint32_t>(old), n0 = static_cast<uint32_t>(old >> 32);
              if (cand > d0 || (cand == d0 && !(bits & ~n0))) break;
              const uint64_t nw = cand < d0 ? (uint64_t(cand) | (uint64_t(bits) << 32))
                                            : (uint64_t(d0) | (uint64_t(n0 | bits) << 32));
              const uint64_t seen = atomicCAS(reinterpret_cast<unsigned long long*>(&dn[t]),
                                              static_cast<unsigned long long>(old),
                                              static_cast<unsigned long long>(nw));
              if (seen == old) {
                stamp8[t] = uint8_t(r + 1u);
                changed = true;
                break;
              }
              old = seen;
            }
          }
        };
        // four chunk slots per step: nodes and stamps read before any push
        for (uint32_t c0 = tid; c0 < C; c0 += 4u * B) {
          uint32_t cs[4], vs[4];
          bool act[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            cs[k] = c0 + uint32_t(k) * B;
            vs[k] = cs[k] < C ? cnode[cs[k]] : 0u;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            // LinkState.cpp:741-752: a hard-drained node other than the source does not relax
            act[k] = cs[k] < C && stamp8[vs[k]] == uint8_t(r) &&
                (!(nfl[vs[k]] & OGS_NODE_OVERLOADED) || vs[k] == s);
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (act[k]) chunk(cs[k], vs[k]);
          }
        }
        const bool more = __syncthreads_or(changed) != 0;
        mark(int(r) + 1);  // round r: slots 3..
#ifdef OGS_STAMPS
        if (firstUnit) diag[2] = r;
#endif
        if (!more) break;
      }
      for (uint32_t v = tid; v < N; v += B) {
        const uint64_t x = dn[v];
        oDist[size_t(u) * Sn + v] = static_cast<uint32_t>(x);
        oNh[size_t(u) * Sn + v] = static_cast<uint32_t>(x >> 32);
      }
    } else {
      for (uint32_t v = tid; v < N; v += B) {
        dist[v] = (v == s) ? 0u : kInf;
        stamp16[v] = (v == s) ? 1 : 0;
#pragma unroll
        for (int w = 0; w < W; ++w) nh[v * W + w] = 0u;
      }
      __syncthreads();
      // ---- distances ----
      for (uint32_t j = tid; j < se - sb; j += B) {
        const uint32_t x = eimg[sb + j];
        if (x & kDown16) continue;
        const uint32_t t = x & kNodeMax, c = weight(sb + j);
        if (c < dist[t]) {
          atomicMin(&dist[t], c);
          stamp16[t] = 2;
        }
      }
      __syncthreads();
      // the chunk slots of this thread whose node is stamped for round r and
      // relaxes (a hard-drained node other than the source does not,
      // LinkState.cpp:741-752; the next-hop phase skips the source too)
      auto scan = [&](uint32_t r, bool skipSource, auto&& fn) {
        for (uint32_t c0 = tid; c0 < C; c0 += 4u * B) {
          uint32_t cs[4], vs[4];
          bool act[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            cs[k] = c0 + uint32_t(k) * B;
            vs[k] = cs[k] < C ? cnode[cs[k]] : 0u;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const bool drained = (nfl[vs[k]] & OGS_NODE_OVERLOADED) != 0;
            act[k] = cs[k] < C && stamp16[vs[k]] == uint16_t(r) &&
                (skipSource ? (vs[k] != s && !drained) : (!drained || vs[k] == s));
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (act[k]) fn(cs[k], vs[k]);
          }
        }
      };
      auto edges8 = [&](uint32_t c, uint32_t v, uint32_t (&x)[kLdsChunk], uint32_t (&dt)[kLdsChunk]) {
        const uint32_t b = row[v] + kLdsChunk * (c - first[v]);
        const uint32_t n = min(kLdsChunk, row[v + 1] - b);
#pragma unroll
        for (uint32_t i = 0; i < kLdsChunk; ++i) x[i] = i < n ? eimg[b + i] : kDown16;
#pragma unroll
        for (uint32_t i = 0; i < kLdsChunk; ++i) dt[i] = dist[x[i] & kNodeMax];
        return b;
      };
      uint32_t r = 2;
      for (;; ++r) {
        bool changed = false;
        scan(r, false, [&](uint32_t c, uint32_t v) {
          const uint32_t dv = dist[v];
          uint32_t x[kLdsChunk], dt[kLdsChunk];
          const uint32_t b = edges8(c, v, x, dt);
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) {
            if (x[i] & kDown16) continue;
            const uint32_t cand = dv + weight(b + i);
            if (cand < dt[i]) {
              atomicMin(&dist[x[i] & kNodeMax], cand);
              stamp16[x[i] & kNodeMax] = uint16_t(r + 1u);
              changed = true;
            }
          }
        });
        if (!__syncthreads_or(changed)) break;
      }
      // ---- next hops: seeds from the source's row, then tight pushes ----
      const uint32_t r0 = r + 1u;
      for (uint32_t j = tid; j < se - sb && j < 32u * W; j += B) {
        const uint32_t x = eimg[sb + j];
        if (x & kDown16) continue;
        const uint32_t t = x & kNodeMax;
        if (weight(sb + j) == dist[t]) {
          atomicOr(&nh[t * W + (j >> 5)], 1u << (j & 31u));
          stamp16[t] = uint16_t(r0);
        }
      }
      __syncthreads();
      for (r = r0;; ++r) {
        bool changed = false;
        scan(r, true, [&](uint32_t c, uint32_t v) {
          const uint32_t dv = dist[v];
          uint32_t nv[W];
#pragma unroll
          for (int w = 0; w < W; ++w) nv[w] = nh[v * W + w];
          uint32_t x[kLdsChunk], dt[kLdsChunk];
          const uint32_t b = edges8(c, v, x, dt);
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) {
            if (x[i] & kDown16) continue;
            const uint32_t t = x[i] & kNodeMax;
            if (dv + weight(b + i) != dt[i]) continue;  // not tight
            bool add = false;
#pragma unroll
            for (int k = 0; k < W; ++k) {
              const uint32_t a = nv[k] & ~nh[t * W + k];
              if (a) {
                atomicOr(&nh[t * W + k], a);
                add = true;
              }
            }
            if (add) {
              stamp16[t] = uint16_t(r + 1u);
              changed = true;
            }
          }
        });
        if (!__syncthreads_or(changed)) break;
      }
      for (uint32_t v = tid; v < N; v += B) {
        oDist[size_t(u) * Sn + v] = dist[v];
#pragma unroll
        for (int w = 0; w < W; ++w) oNh[(size_t(u) * W + w) * Sn + v] = nh[v * W + w];
      }
    }
    __syncthreads();  // state and outputs of this unit done before the next
#ifdef OGS_STAMPS
    if (firstUnit) {
      diag[1] = uint32_t(__builtin_amdgcn_s_memtime() - k0);  // staging + first unit
      firstUnit = false;
    }
    ++diag[11];
#endif
  }
#ifdef OGS_STAMPS
  diag[12] = uint32_t(__builtin_amdgcn_s_memtime() - k0);
  if (threadIdx.x == 0 && blockIdx.x < kLdsDiagWgs) {
    uint32_t* o = g_ldsStamps + (size_t(W - 1) * kLdsDiagWgs + blockIdx.x) * 16u;
    for (int i = 0; i < 16; ++i) o[i] = diag[i];
  }
#endif
}

int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
           n > 0)
        ? n
        : 256;
  }
  return cus;
}

}  // namespace

// Scratch of the LDS images (workspace) and whether the batch qualifies:
// nodes fit 15 bits, chunk ids 16 bits, the image + one unit's state fit LDS.
size_t lds_image_bytes(const ogs_graph& g, int W) {
  if (g.max_nodes <= 0 || uint32_t(g.max_nodes) > kNodeMax || W < 1 || W > 4) return 0;
  const uint32_t cap = uint32_t(g.max_edges) / kLdsChunk + uint32_t(g.max_nodes);
  if (cap > 0xFFFFu || uint32_t(g.max_edges) > 0xFFFFFFu) return 0;
  const LdsImage L = lds_image(g, W);
  if (L.block + L.state > 160u * 1024u) return 0;
  return (size_t(g.num_topos) * L.stride + 255u) & ~size_t(255);
}

// SPF of every unit into dist / nh (u32 distances, W next-hop words): image
// build (one workgroup per topology), then one persistent 1024-thread
// workgroup per CU over the units. Call only when lds_image_bytes() != 0.
int g_spfLdsForm = 0;  // "spf_lds_form": 0 three-pass rounds, 1 CAS / two-phase (A/B)

hipError_t launch_spf_lds(const ogs_graph& g, const ogs_unit* units, int nUnits,
                          uint32_t flags, int W, uint32_t* dist, uint32_t* nh,
                          void* scratch, hipStream_t stream) {
  if (g_spfLdsForm) flags |= kFlagLdsCasForm;
  const LdsImage L = lds_image(g, W);
  uint8_t* img = static_cast<uint8_t*>(scratch);
  hipLaunchKernelGGL(lds_scan_kernel, dim3(g.num_topos), dim3(kLdsBlock), 0, stream, g, L, img);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t per = kBlock * kEdgesPerThread;
  hipLaunchKernelGGL(lds_edges_kernel,
                     dim3((uint32_t(std::max(g.max_edges, 1)) + per - 1u) / per, g.num_topos),
                     dim3(kBlock), 0, stream, g, L, img);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t lds = L.block + L.state;
  const int grid = std::max(1, std::min(nUnits, num_cus()));
  auto go = [&](auto k) {
    if (lds > 64u * 1024u) {
      hipError_t a = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
      if (a != hipSuccess) return a;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(kLdsBlock), lds, stream, g, L,
                       static_cast<const uint8_t*>(img), units, nUnits, flags, dist, nh);
    return hipGetLastError();
  };
  switch (W) {
    case 1: return go(spf_lds_kernel<1>);
    case 2: return go(spf_lds_kernel<2>);
    case 3: return go(spf_lds_kernel<3>);
    case 4: return go(spf_lds_kernel<4>);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace ogs

#ifdef OGS_STAMPS
extern "C" int ogs_diag_lds_stamps(uint32_t* host, int32_t words) {
  const size_t n = std::min<size_t>(size_t(words), size_t(4) * ogs::kLdsDiagWgs * 16);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ogs::g_ldsStamps), n * 4, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
