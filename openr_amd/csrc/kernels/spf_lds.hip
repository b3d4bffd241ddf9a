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
  L.state = W == 1 ? al16(8u * N) + al16(N)                      // packed words, u8 stamps
                   : al16(4u * N) + al16(4u * N * uint32_t(W)) + al16(2u * N);
  L.stride = 16u + L.block;
  return L;
}

// header of topology t's image: {chunks, uniform (0/1), weight, 0}
// One workgroup per topology.
__global__ __launch_bounds__(kBlock) void lds_image_kernel(ogs_graph g, LdsImage L,
                                                          uint8_t* __restrict__ img) {
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ uint32_t base, wmin, wmax;
  const uint32_t t = blockIdx.x, tid = threadIdx.x;
  const uint32_t nb = g.node_base[t];
  const uint32_t N = g.node_base[t + 1] - nb;
  const uint32_t* __restrict__ gRow = g.row_ptr + nb;
  const uint32_t e0 = gRow[0];
  const uint32_t E = gRow[N] - e0;
  uint8_t* hdr = img + size_t(t) * L.stride;
  uint8_t* blk = hdr + 16;
  uint16_t* eimg = reinterpret_cast<uint16_t*>(blk + L.eimg);
  uint16_t* cnode = reinterpret_cast<uint16_t*>(blk + L.cnode);
  uint32_t* row = reinterpret_cast<uint32_t*>(blk + L.row);
  uint16_t* first = reinterpret_cast<uint16_t*>(blk + L.first);
  uint8_t* fl = blk + L.flags;
  if (tid == 0) {
    base = 0u;
    wmin = 0xFFFFFFFFu;
    wmax = 0u;
  }
  __syncthreads();
  uint32_t lo = 0xFFFFFFFFu, hi = 0u;
  for (uint32_t e = tid; e < E; e += kBlock) {
    const uint64_t x = g.edges[e0 + e];
    const uint32_t w = static_cast<uint32_t>(x);
    const bool down = (w & OGS_EDGE_DOWN) != 0u;
    eimg[e] = uint16_t(edge_dst(w) | (down ? kDown16 : 0u));
    if (!down) {
      lo = min(lo, static_cast<uint32_t>(x >> 32));
      hi = max(hi, static_cast<uint32_t>(x >> 32));
    }
  }
  atomicMin(&wmin, lo);
  atomicMax(&wmax, hi);
  for (uint32_t v = tid; v <= N; v += kBlock) row[v] = gRow[v] - e0;
  for (uint32_t v = tid; v < N; v += kBlock) fl[v] = g.node_flags[nb + v];
  // chunk ids: exclusive scan of ceil(deg / 8) over the nodes, tile by tile
  const int lane = int(tid & 63u), wave = int(tid >> 6);
  for (uint32_t t0 = 0; t0 < N; t0 += kBlock) {
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
    if (tid == kBlock - 1u) base = off + inc;
    const uint32_t at = off + inc - n;
    if (v < N) first[v] = uint16_t(at);
    for (uint32_t k = 0; k < n; ++k) cnode[at + k] = uint16_t(v);
    __syncthreads();
  }
  if (tid == 0) {
    uint32_t* h = reinterpret_cast<uint32_t*>(hdr);
    const bool uniform = wmin == wmax;
    h[0] = base;
    h[1] = uniform ? 1u : 0u;
    h[2] = uniform ? wmin : 0u;
    h[3] = 0u;
  }
}

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
  // W == 1
  uint64_t* dn = reinterpret_cast<uint64_t*>(st);
  uint8_t* stamp8 = reinterpret_cast<uint8_t*>(st + al16(8u * Sn));
  // W > 1
  uint32_t* dist = reinterpret_cast<uint32_t*>(st);
  uint32_t* nh = reinterpret_cast<uint32_t*>(st + al16(4u * Sn));
  uint16_t* stamp16 = reinterpret_cast<uint16_t*>(st + al16(4u * Sn) + al16(4u * Sn * W));

  uint32_t staged = 0xFFFFFFFFu;
  uint32_t C = 0, uniform = 0, w0 = 0, N = 0, e0 = 0;
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
      uniform = h[1];
      w0 = h[2];
      const uint32_t nb = g.node_base[unit.topo];
      N = g.node_base[unit.topo + 1] - nb;
      e0 = g.row_ptr[nb];
      staged = unit.topo;
      __syncthreads();
    }
    const uint64_t* __restrict__ edges = g.edges + e0;
    auto weight = [&](uint32_t e) -> uint32_t {
      return hop ? 1u : uniform ? w0 : static_cast<uint32_t>(edges[e] >> 32);
    };
    const uint32_t s = unit.src;
    const uint32_t sb = row[s], se = row[s + 1];
    if constexpr (W == 1) {
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
      for (uint32_t r = 2;; ++r) {
        bool changed = false;
        for (uint32_t c = tid; c < C; c += B) {
          const uint32_t v = cnode[c];
          if (stamp8[v] != uint8_t(r)) continue;
          if ((nfl[v] & OGS_NODE_OVERLOADED) && v != s) continue;  // LinkState.cpp:741-752
          const uint64_t xv = dn[v];
          const uint32_t dv = static_cast<uint32_t>(xv), nv = static_cast<uint32_t>(xv >> 32);
          const uint32_t b = row[v] + kLdsChunk * (c - first[v]);
          const uint32_t n = min(kLdsChunk, row[v + 1] - b);
          for (uint32_t i = 0; i < n; ++i) {
            // the source contributes its link slot, others NH(v) (LinkState.cpp:808-811)
            const uint32_t slot = b + i - sb;
            push(b + i, dv, v == s ? (slot < 32u ? 1u << slot : 0u) : nv, r, changed);
          }
        }
        if (!__syncthreads_or(changed)) break;
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
      uint32_t r = 2;
      for (;; ++r) {
        bool changed = false;
        for (uint32_t c = tid; c < C; c += B) {
          const uint32_t v = cnode[c];
          if (stamp16[v] != uint16_t(r)) continue;
          if ((nfl[v] & OGS_NODE_OVERLOADED) && v != s) continue;
          const uint32_t dv = dist[v];
          const uint32_t b = row[v] + kLdsChunk * (c - first[v]);
          const uint32_t n = min(kLdsChunk, row[v + 1] - b);
          for (uint32_t i = 0; i < n; ++i) {
            const uint32_t x = eimg[b + i];
            if (x & kDown16) continue;
            const uint32_t t = x & kNodeMax, cand = dv + weight(b + i);
            if (cand < dist[t]) {
              atomicMin(&dist[t], cand);
              stamp16[t] = uint16_t(r + 1u);
              changed = true;
            }
          }
        }
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
        for (uint32_t c = tid; c < C; c += B) {
          const uint32_t v = cnode[c];
          if (stamp16[v] != uint16_t(r) || v == s || (nfl[v] & OGS_NODE_OVERLOADED)) continue;
          const uint32_t dv = dist[v];
          uint32_t nv[W];
#pragma unroll
          for (int w = 0; w < W; ++w) nv[w] = nh[v * W + w];
          const uint32_t b = row[v] + kLdsChunk * (c - first[v]);
          const uint32_t n = min(kLdsChunk, row[v + 1] - b);
          for (uint32_t i = 0; i < n; ++i) {
            const uint32_t x = eimg[b + i];
            if (x & kDown16) continue;
            const uint32_t t = x & kNodeMax;
            if (dv + weight(b + i) != dist[t]) continue;  // not tight
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
        }
        if (!__syncthreads_or(changed)) break;
      }
      for (uint32_t v = tid; v < N; v += B) {
        oDist[size_t(u) * Sn + v] = dist[v];
#pragma unroll
        for (int w = 0; w < W; ++w) oNh[(size_t(u) * W + w) * Sn + v] = nh[v * W + w];
      }
    }
    __syncthreads();  // state and outputs of this unit done before the next
  }
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
hipError_t launch_spf_lds(const ogs_graph& g, const ogs_unit* units, int nUnits,
                          uint32_t flags, int W, uint32_t* dist, uint32_t* nh,
                          void* scratch, hipStream_t stream) {
  const LdsImage L = lds_image(g, W);
  uint8_t* img = static_cast<uint8_t*>(scratch);
  hipLaunchKernelGGL(lds_image_kernel, dim3(g.num_topos), dim3(kBlock), 0, stream, g, L, img);
  hipError_t e = hipGetLastError();
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
