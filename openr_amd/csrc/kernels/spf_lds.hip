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
// table with the node's drained bit; row offsets: 113 KB for C3) and then
// solves its share of the units back to back with every round served from
// LDS, each round visiting only the chunk records of its active nodes.
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
#include <mutex>
#include <cstdint>
#include <type_traits>

#include "openr_gpu.h"
#include "route_core.h"
#include "route_stream.h"
#include "spf_lds.h"
#include "spf_core.h"
#include "engine.h"

namespace ogs {

namespace {

constexpr uint32_t kDown16 = 0x8000u;     // eimg: edge down
constexpr uint32_t kNodeMax = 0x7FFFu;    // 15-bit neighbour ids
constexpr uint32_t kDrained16 = 0x8000u;  // cnode: the chunk's node is hard-drained
constexpr uint32_t kLdsChunk = 8;         // edges per chunk (one lane's push)
constexpr int kLdsBlock = 1024;
constexpr uint32_t kLdsDiagWgsItems = 1024;  // workgroups with item stamps (OGS_STAMPS)
// launch flag of the LDS forms (above the OGS_F_* bits): the BFS rounds'
// all-reached exit off ("lds_bfs_exit" 0, A/B)
constexpr uint32_t kFlagLdsNoBfsExit = 1u << 25;
// bits 20..23: the BFS rounds' pull ratio ("lds_pull"): a round pulls when
// 4 x (chunk records of unreached nodes) <= ratio x (the frontier's)
constexpr uint32_t kFlagLdsPullShift = 20;

__host__ __device__ inline uint32_t al16(uint32_t x) { return (x + 15u) & ~15u; }

// u8 round stamp of round r >= 1 in the general-weight rounds: 1..255
// cyclic, never 0 (= not pending); stamp_of(2) == 2 (the seed round's value)
__device__ __forceinline__ uint32_t stamp_of(uint32_t r) { return 1u + (r - 1u) % 255u; }

// chunk records of one topology: sum over nodes of ceil(deg / 8) <= (E + 7 N) / 8
__host__ __device__ inline uint32_t chunk_cap(uint32_t N, uint32_t E) {
  return (E + (kLdsChunk - 1u) * N) / kLdsChunk;
}

// Byte layout of one topology's image (global, then the same block in LDS):
// header (16 B, global only: {chunks, 0, 0, 0}) | eimg u16[E] | cnode u16[cap] | row u32[N+1] |
// first u16[N], sections 16-B aligned, sized by the batch's maxima so every
// topology (and the LDS copy) shares the offsets. Then, LDS only, one unit's
// state: dist u32[N] | nh u32[N * W] | stamp u8[N] | queue u16[cap].
struct LdsImage {
  uint32_t eimg, cnode, row, first, block;  // offsets in the block
  uint32_t nh, stamp, queue, state;         // offsets in the state; state bytes
  uint32_t stride;                          // header + block
};

__host__ LdsImage lds_image(const ogs_graph& g, int W) {
  const uint32_t N = uint32_t(g.max_nodes), E = uint32_t(g.max_edges);
  const uint32_t cap = chunk_cap(N, E);
  LdsImage L{};
  L.eimg = 0;
  L.cnode = L.eimg + al16(2u * E);
  L.row = L.cnode + al16(2u * cap);
  L.first = L.row + al16(4u * (N + 1u));
  L.block = L.first + al16(2u * N);
  L.nh = al16(4u * N);
  L.stamp = L.nh + al16(4u * N * uint32_t(W));
  L.queue = L.stamp + al16(N);
  L.state = L.queue + al16(2u * cap);
  L.stride = 16u + L.block;
  return L;
}

// Scratch of the LDS paths, one call: images [num_topos * stride] | weight
// min / max / asymmetry partials uint4[num_topos * nEB] (one per prep edge block) | work
// counter (u32, 256-B line) | unit ready flags u32[nUnits] (megakernel).
constexpr uint32_t kPrepEdgesPerThread = 2;
constexpr uint32_t kPrepEdges = kLdsBlock * kPrepEdgesPerThread;  // edges per prep edge block
constexpr uint32_t kPrepKeys = kLdsBlock;  // route keys per prep key block
struct LdsScratch {
  size_t mm, ctr, ready, bytes;
  uint32_t nEB;
};

__host__ LdsScratch lds_scratch(const ogs_graph& g, const LdsImage& L, int nUnits) {
  auto r256 = [](size_t x) { return (x + 255u) & ~size_t(255); };
  LdsScratch S{};
  S.nEB = (uint32_t(std::max(g.max_edges, 1)) + kPrepEdges - 1u) / kPrepEdges;
  S.mm = r256(size_t(g.num_topos) * L.stride);
  S.ctr = S.mm + r256(size_t(g.num_topos) * S.nEB * 16u);
  S.ready = S.ctr + 256u;
  S.bytes = S.ready + r256(size_t(std::max(nUnits, 1)) * 4u);
  return S;
}

// Prep, once per call, one launch of 1024-thread blocks in three roles:
//  blocks [0, T): topology t's row offsets, chunk -> node table (with the
//    node's drained bit) and header {chunks}; block 0 also zeroes the work
//    counter and the ready flags;
//  next T * nEB: 2,048 edges each -> the 2-B edge words and the block's
//    min / max weight over up edges (uniform weights iff min == max);
//  next T * nKB (when keys are asked for): 1,024 prefixes each -> the route
//    keys of route_stream.h (pfx_key_kernel's), u32 or packed u16.
// One prep block `blk` (a 1024-thread workgroup): the body of both the
// separate prep launch (lds_prep_kernel, blk = blockIdx.x) and the prep items
// at the head of the one-launch form's queue (spf_lds_route_kernel). `ctr` /
// `ready` (zeroed by block 0) are nullptr in the one-launch form, whose
// counters are epoch-based.
// Topology t's offsets: from topo_desc in one load when the caller passes
// it, else node_base / row_ptr (a dependent pair)
struct TopoSpan {
  uint32_t nb, N, e0, E;
};
__device__ __forceinline__ TopoSpan topo_span(const ogs_graph& g, uint32_t t) {
  if (g.topo_desc) {
    const uint4 d = *reinterpret_cast<const uint4*>(g.topo_desc + size_t(t) * 8u);
    return TopoSpan{d.x, d.y, d.z, d.w};
  }
  const uint32_t nb = g.node_base[t], N = g.node_base[t + 1] - nb;
  const uint32_t e0 = g.row_ptr[nb];
  return TopoSpan{nb, N, e0, g.row_ptr[nb + N] - e0};
}

__device__ __forceinline__ void lds_prep_block(
    const ogs_graph& g, const ogs_prefix_table& pt, void* __restrict__ key, uint32_t key16,
    uint32_t nKB, const LdsImage& L, uint8_t* __restrict__ img, uint4* __restrict__ mm,
    uint32_t nEB, uint32_t* __restrict__ ctr, uint32_t* __restrict__ ready, uint32_t nReady,
    uint32_t blk) {
  constexpr uint32_t B = kLdsBlock;
  __shared__ uint32_t wsum[B / 64];
  __shared__ uint32_t whi[B / 64];
  __shared__ uint32_t wasym[B / 64];
  __shared__ uint32_t base;
  const uint32_t T = uint32_t(g.num_topos), tid = threadIdx.x;
  const int lane = int(tid & 63u), wave = int(tid >> 6);
  if (blk < T) {
    const uint32_t t = blk;
    if (t == 0u && ctr) {
      if (tid == 0u) *ctr = 0u;
      for (uint32_t i = tid; i < nReady; i += B) ready[i] = 0u;
    }
    const TopoSpan sp = topo_span(g, t);
    const uint32_t nb = sp.nb, N = sp.N, e0 = sp.e0;
    const uint32_t* __restrict__ gRow = g.row_ptr + nb;
    uint8_t* hdr = img + size_t(t) * L.stride;
    uint8_t* b8 = hdr + 16;
    uint16_t* __restrict__ cnode = reinterpret_cast<uint16_t*>(b8 + L.cnode);
    uint32_t* __restrict__ row = reinterpret_cast<uint32_t*>(b8 + L.row);
    uint16_t* __restrict__ first = reinterpret_cast<uint16_t*>(b8 + L.first);
    // the first kPre tiles' degrees and drained bits in one round of loads
    // (C3's 2,080 nodes are three tiles), later tiles per tile
    constexpr uint32_t kPre = 4;
    uint32_t deg0[kPre], tag0[kPre];
#pragma unroll
    for (uint32_t k = 0; k < kPre; ++k) {
      const uint32_t v = k * B + tid;
      deg0[k] = v < N ? gRow[v + 1] - gRow[v] : 0u;
      tag0[k] = v < N && (g.node_flags[nb + v] & OGS_NODE_OVERLOADED) ? kDrained16 : 0u;
    }
    if (tid == 0) base = 0u;
    for (uint32_t v = tid; v <= N; v += B) row[v] = gRow[v] - e0;
    __syncthreads();
    // chunk ids: exclusive scan of ceil(deg / 8) over the nodes, tile by tile
    uint32_t ti = 0;
    for (uint32_t t0 = 0; t0 < N; t0 += B, ++ti) {
      const uint32_t v = t0 + tid;
      uint32_t deg = 0u, tag = 0u;
      if (ti < kPre) {
#pragma unroll
        for (uint32_t k = 0; k < kPre; ++k) {
          deg = ti == k ? deg0[k] : deg;
          tag = ti == k ? tag0[k] : tag;
        }
      } else if (v < N) {
        deg = gRow[v + 1] - gRow[v];
        tag = (g.node_flags[nb + v] & OGS_NODE_OVERLOADED) ? kDrained16 : 0u;
      }
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
      if (v < N) {
        first[v] = uint16_t(at);
        for (uint32_t k = 0; k < n; ++k) cnode[at + k] = uint16_t(v | tag);
      }
      __syncthreads();
    }
    if (tid == 0) {
      uint32_t* h = reinterpret_cast<uint32_t*>(hdr);
      h[0] = base;  // chunk records
      h[1] = N;
      h[2] = e0;
      h[3] = 0u;
    }
    return;
  }
  blk -= T;
  if (blk < T * nEB) {
    const uint32_t t = blk / nEB, eb = blk - t * nEB;
    const TopoSpan sp = topo_span(g, t);
    const uint32_t nb = sp.nb, N = sp.N, e0 = sp.e0, E = sp.E;
    uint16_t* __restrict__ eimg = reinterpret_cast<uint16_t*>(img + size_t(t) * L.stride + 16 + L.eimg);
    const uint64_t* __restrict__ edges = g.edges + e0;
    const uint32_t e00 = eb * kPrepEdges + tid;
    uint64_t x[kPrepEdgesPerThread];
#pragma unroll
    for (uint32_t k = 0; k < kPrepEdgesPerThread; ++k) {
      const uint32_t e = e00 + k * B;
      x[k] = e < E ? edges[e] : uint64_t(OGS_EDGE_DOWN);
    }
    uint32_t lo = 0xFFFFFFFFu, hi = 0u;
    // symmetry (the BFS pull's precondition): each edge u -> v has its
    // reverse v -> u (rslot, or rslot_ext past 511) in the same up / down
    // state; unknown (no edge_src, saturated slot without rslot_ext) = asym.
    // A thread's edges are checked independently, so each dependent step
    // (slot -> reverse row -> reverse edge) issues its loads for all of them
    // at once.
    bool asym = g.edge_src == nullptr;
    uint32_t rs[kPrepEdgesPerThread], src[kPrepEdgesPerThread];
#pragma unroll
    for (uint32_t k = 0; k < kPrepEdgesPerThread; ++k) {
      const uint32_t e = e00 + k * B;
      const uint32_t w = static_cast<uint32_t>(x[k]);
      const bool down = (w & OGS_EDGE_DOWN) != 0u;
      if (e < E) eimg[e] = uint16_t(edge_dst(w) | (down ? kDown16 : 0u));
      if (!down) {
        lo = min(lo, static_cast<uint32_t>(x[k] >> 32));
        hi = max(hi, static_cast<uint32_t>(x[k] >> 32));
      }
      rs[k] = (w >> OGS_EDGE_RSLOT_SHIFT) & OGS_EDGE_RSLOT_MASK;
      src[k] = 0u;
      if (!asym && e < E) {
        src[k] = g.edge_src[e0 + e];
        if (rs[k] == OGS_EDGE_RSLOT_MASK && g.rslot_ext) rs[k] = g.rslot_ext[e0 + e];
      }
    }
    if (!asym) {
      uint32_t rb[kPrepEdgesPerThread], re[kPrepEdgesPerThread];
#pragma unroll
      for (uint32_t k = 0; k < kPrepEdgesPerThread; ++k) {
        const uint32_t v = edge_dst(static_cast<uint32_t>(x[k]));
        rb[k] = re[k] = 0u;
        if (e00 + k * B < E && v < N) {
          rb[k] = g.row_ptr[nb + v] - e0;
          re[k] = g.row_ptr[nb + v + 1] - e0;
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < kPrepEdgesPerThread; ++k) {
        const uint32_t e = e00 + k * B;
        if (e >= E) continue;
        const uint32_t w = static_cast<uint32_t>(x[k]);
        // rs still saturated: past 511 with no rslot_ext; rb == re: v >= N
        bool bad = rs[k] == OGS_EDGE_RSLOT_MASK && !g.rslot_ext;
        bad = bad || rb[k] + rs[k] >= re[k];
        if (!bad) {
          const uint32_t rw = static_cast<uint32_t>(edges[rb[k] + rs[k]]);
          bad = edge_dst(rw) != src[k] ||
              ((rw & OGS_EDGE_DOWN) != 0u) != ((w & OGS_EDGE_DOWN) != 0u);
        }
        asym = asym || bad;
      }
    }
    const uint32_t anyAsym = __ballot(asym) != 0ull ? 1u : 0u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      lo = min(lo, __shfl_xor(lo, d, 64));
      hi = max(hi, __shfl_xor(hi, d, 64));
    }
    if (lane == 0) {
      wsum[wave] = lo;
      whi[wave] = hi;
      wasym[wave] = anyAsym;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t as = wasym[0];
      for (uint32_t w = 1; w < B / 64u; ++w) {
        lo = min(lo, wsum[w]);
        hi = max(hi, whi[w]);
        as |= wasym[w];
      }
      mm[size_t(t) * nEB + eb] = make_uint4(lo, hi, as, 0u);
    }
    return;
  }
  blk -= T * nEB;
  if (key && blk < T * nKB) {
    const uint32_t t = blk / nKB, p0 = (blk - t * nKB) * kPrepKeys + tid;
    const uint32_t Sp = uint32_t(pt.max_prefixes);
#pragma unroll
    for (uint32_t j = 0; j < kPrepKeys / B; ++j) {
      const uint32_t p = p0 + j * B;
      if (p < Sp) {
        const uint32_t k = prefix_key(pt, t, p);
        if (key16) {
          static_cast<uint16_t*>(key)[size_t(t) * Sp + p] = key16_of(k);
        } else {
          static_cast<uint32_t*>(key)[size_t(t) * Sp + p] = k;
        }
      }
    }
  }
}

__global__ __launch_bounds__(kLdsBlock) void lds_prep_kernel(
    ogs_graph g, ogs_prefix_table pt, void* __restrict__ key, uint32_t key16, uint32_t nKB,
    LdsImage L,
    uint8_t* __restrict__ img, uint4* __restrict__ mm, uint32_t nEB, uint32_t* __restrict__ ctr,
    uint32_t* __restrict__ ready, uint32_t nReady) {
  lds_prep_block(g, pt, key, key16, nKB, L, img, mm, nEB, ctr, ready, nReady, blockIdx.x);
}

#ifdef OGS_STAMPS
// diagnostic build: item timeline of spf_lds_route_kernel, per workgroup up
// to kItemStamps items x 4 words {kind << 28 | unit, start, ready, end} on
// the 100 MHz realtime clock (kind 1 SPF, 2 stream item, 3 join); read with
// ogs_diag_item_stamps (tools/c3_timeline.py)
constexpr uint32_t kItemStamps = 64;
__device__ uint32_t g_itemStamps[kLdsDiagWgsItems * kItemStamps * 4];
#endif
#ifdef OGS_STAMPS
// diagnostic build: per workgroup 32 words {staging, first unit's SPF
// (incl. staging), rounds, units, kernel cycles, first unit's queue total,
// 0, 0, then rounds 2..9 of the first unit x (queue, distances, next hops)
// cycles}, rows (W - 1) * 4096 + blockIdx.x; read with ogs_diag_lds_stamps
constexpr uint32_t kLdsDiagWgs = 4096;
__device__ uint32_t g_ldsStamps[4 * kLdsDiagWgs * 32];
#endif

// SPF of the workgroup's units over the LDS image. Every round r:
//  (0) queue: the chunk records whose node is stamped r and relaxes (one
//      pass over the chunk table, a wave-aggregated append);
//  (1) distances: atomicMin of each queued chunk's candidates; a push that
//      lowers its target stamps it r + 1 and clears its next hops;
//  (2) next hops: atomicOr of each still-current queued node's next-hop
//      words along the edges that are tight NOW; a target whose words grew
//      is stamped r + 1.
// A push from a longer stale distance ORs nothing (not tight); a node whose
// distance later falls drops what it had. The least fixpoint of spf_core.h
// with fire-and-forget LDS atomics, and every chunk record is visited only
// in the rounds its node is active (each once, on unit-weight BFS layers).
//
// Per-workgroup staging state (the topology whose image is in LDS) and the
// diagnostics policy of spf_lds_unit: NoDiag in product builds; the
// OGS_STAMPS build's LdsStamps records the first unit's phase cycles.
struct LdsWg {
  uint32_t staged = 0xFFFFFFFFu;
  uint32_t C = 0, uniform = 0, w0 = 0, N = 0, e0 = 0;
  uint32_t sym = 0;  // every edge's reverse present, same up / down state
};

struct NoDiag {
  __device__ void mark(uint32_t) {}
  __device__ void rounds(uint32_t) {}
  __device__ void queued(uint32_t) {}
  __device__ void unit_done() {}
};

#ifdef OGS_STAMPS
struct LdsStamps {
  uint32_t* diag;
  bool on, first = true;
  uint64_t k0, tr;
  uint32_t units = 0, q = 0;
  __device__ LdsStamps(int W)
      : diag(g_ldsStamps + (size_t(W - 1) * kLdsDiagWgs + blockIdx.x) * 32u),
        on(threadIdx.x == 0u && blockIdx.x < kLdsDiagWgs),
        k0(__builtin_amdgcn_s_memtime()),
        tr(k0) {}
  __device__ void mark(uint32_t slot) {  // cycles since the last mark of the first unit
    const uint64_t now = __builtin_amdgcn_s_memtime();
    if (on && first && slot < 32u) diag[slot] = uint32_t(now - tr);
    tr = now;
  }
  __device__ void rounds(uint32_t r) {
    if (on && first) diag[2] = r;
  }
  __device__ void queued(uint32_t n) { q += n; }
  __device__ void unit_done() {
    if (on && first) {
      diag[1] = uint32_t(__builtin_amdgcn_s_memtime() - k0);  // staging + first unit
      diag[5] = q;
    }
    first = false;
    ++units;
  }
  __device__ void finish() {
    if (on) {
      diag[3] = units;
      diag[4] = uint32_t(__builtin_amdgcn_s_memtime() - k0);
    }
  }
};
#endif

// lds_stage: topology t's image (built by the prep launch) into this
// workgroup's LDS, with its header {chunk records, nodes, first edge} and
// the edge blocks' weight / symmetry partials -- every load of it issued in
// one round (eight 16-B loads in flight per lane: C3's 113 KB image is one
// batch), no dependent global load after the copy.
__device__ __forceinline__ void lds_stage(const ogs_graph& g, const LdsImage& L,
                                          const uint8_t* __restrict__ img,
                                          const uint4* __restrict__ mm, uint32_t nEB, uint32_t t,
                                          char* blk, LdsWg& wg) {
  constexpr uint32_t B = kLdsBlock;
  const uint32_t tid = threadIdx.x;
  __syncthreads();  // the previous unit's state reads are done
  const uint8_t* hdr = img + size_t(t) * L.stride;
  const uint4* src = reinterpret_cast<const uint4*>(hdr + 16);
  uint4* dst = reinterpret_cast<uint4*>(blk);
  const uint4 h = *reinterpret_cast<const uint4*>(hdr);
  uint32_t lo = 0xFFFFFFFFu, hi = 0u, asym = 0u;
  for (uint32_t b = 0; b < nEB; ++b) {
    const uint4 x = mm[size_t(t) * nEB + b];
    lo = min(lo, x.x);
    hi = max(hi, x.y);
    asym |= x.z;
  }
  const uint32_t n16 = L.block / 16u;
  for (uint32_t i0 = 0; i0 < n16; i0 += 8u * B) {
    uint4 x[8];
#pragma unroll
    for (uint32_t k = 0; k < 8u; ++k) {
      const uint32_t i = i0 + k * B + tid;
      x[k] = i < n16 ? src[i] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (uint32_t k = 0; k < 8u; ++k) {
      const uint32_t i = i0 + k * B + tid;
      if (i < n16) dst[i] = x[k];
    }
  }
  wg.C = h.x;
  wg.N = h.y;
  wg.e0 = h.z;
  wg.uniform = lo == hi ? 1u : 0u;  // every up edge of this weight
  wg.w0 = lo;
  wg.sym = asym ? 0u : 1u;
  wg.staged = t;
  __syncthreads();
}

// spf_lds_unit: the SPF of unit u (index into the launch's dist / nh rows)
// by this workgroup, its topology's image staged on first use and kept.
// smem: the dynamic LDS (image block, then the unit's state laid out by L,
// whose next-hop region may be sized for a wider W than this one).
template <int W, typename Diag>
__device__ __forceinline__ void spf_lds_unit(
    const ogs_graph& g, const LdsImage& L, const uint8_t* __restrict__ img,
    const uint4* __restrict__ mm, uint32_t nEB, const ogs_unit unit, uint32_t u,
    uint32_t flags, uint32_t* __restrict__ oDist, uint32_t* __restrict__ oNh, char* smem,
    uint32_t* qCount, LdsWg& wg, Diag& dg) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  constexpr uint32_t B = kLdsBlock;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t Sn = uint32_t(g.max_nodes);
  const bool hop = (flags & OGS_F_HOP_METRIC) != 0u;
  char* blk = smem;
  const uint16_t* eimg = reinterpret_cast<const uint16_t*>(blk + L.eimg);
  const uint16_t* cnode = reinterpret_cast<const uint16_t*>(blk + L.cnode);
  const uint32_t* row = reinterpret_cast<const uint32_t*>(blk + L.row);
  const uint16_t* first = reinterpret_cast<const uint16_t*>(blk + L.first);
  char* st = blk + L.block;
  uint32_t* dist = reinterpret_cast<uint32_t*>(st);
  uint32_t* nh = reinterpret_cast<uint32_t*>(st + L.nh);
  uint8_t* stamp = reinterpret_cast<uint8_t*>(st + L.stamp);
  uint16_t* queue = reinterpret_cast<uint16_t*>(st + L.queue);
  uint32_t& staged = wg.staged;
  uint32_t& C = wg.C;
  uint32_t& uniform = wg.uniform;
  uint32_t& w0 = wg.w0;
  uint32_t& N = wg.N;
  uint32_t& e0 = wg.e0;
  auto mark = [&](uint32_t slot) { dg.mark(slot); };
  {
    if (unit.topo != staged) lds_stage(g, L, img, mm, nEB, unit.topo, blk, wg);
    mark(0);  // staging (the first unit only)
    const uint64_t* __restrict__ edges = g.edges + e0;
    const uint32_t wc = hop ? 1u : w0;  // the weight when it is one constant
    const bool constW = hop || uniform;
    auto weight = [&](uint32_t e) -> uint32_t {
      return constW ? wc : static_cast<uint32_t>(edges[e] >> 32);
    };
    const uint32_t s = unit.src;
    const uint32_t sb = row[s], se = row[s + 1];
    const uint32_t sym = wg.sym;
    // BFS layers (one constant weight > 0) keep no round stamps: stamp[v]
    // holds v's hard-drained bit instead (the node pass and the pull read it)
    const bool bfs = constW && wc > 0u;
    for (uint32_t v = tid; v < N; v += B) {
      dist[v] = (v == s) ? 0u : kInf;
      stamp[v] = bfs && row[v + 1] > row[v] && (cnode[first[v]] & kDrained16) ? 1 : 0;
#pragma unroll
      for (int w = 0; w < W; ++w) nh[v * W + w] = 0u;
    }
    if (tid < 6u) qCount[tid] = 0u;
    __syncthreads();
    // round 1: the source's row (slot j = j-th edge of the row; the source
    // relaxes even when drained, LinkState.cpp:741-752)
    for (uint32_t j = tid; j < se - sb; j += B) {
      const uint32_t x = eimg[sb + j];
      if (x & kDown16) continue;
      atomicMin(&dist[x & kNodeMax], weight(sb + j));
    }
    __syncthreads();
    for (uint32_t j = tid; j < se - sb && j < 32u * W; j += B) {
      const uint32_t x = eimg[sb + j];
      if (x & kDown16) continue;
      const uint32_t t = x & kNodeMax;
      if (weight(sb + j) != dist[t]) continue;
      atomicOr(&nh[t * W + (j >> 5)], 1u << (j & 31u));
      if (!bfs) stamp[t] = 2;
    }
    __syncthreads();
    // rounds 2.., specialised on whether the weight is one constant (no
    // per-edge weight reads at all) or read per edge from the CSR
    auto rounds = [&](auto constant, auto layered) {
      constexpr bool kConst = decltype(constant)::value;
      constexpr bool kBfs = decltype(layered)::value;
      auto wt = [&](uint32_t e) -> uint32_t {
        if constexpr (kConst) {
          return wc;
        } else {
          return static_cast<uint32_t>(edges[e] >> 32);
        }
      };
      // one queued chunk: its node, edge words, targets' distances and the
      // candidates, every LDS / weight read issued before any push
      struct Chunk {
        uint32_t v, dv;
        uint32_t x[kLdsChunk], dt[kLdsChunk], cand[kLdsChunk];
      };
      auto load = [&](uint32_t q, Chunk& k) {
        const uint32_t c = queue[q];
        k.v = cnode[c] & kNodeMax;
        k.dv = dist[k.v];
        const uint32_t b = row[k.v] + kLdsChunk * (c - first[k.v]);
        const uint32_t n = min(kLdsChunk, row[k.v + 1] - b);
        // the words past the row are read too (inside LDS; branch-free) and
        // masked down
#pragma unroll
        for (uint32_t i = 0; i < kLdsChunk; ++i) k.x[i] = eimg[b + i];
#pragma unroll
        for (uint32_t i = 0; i < kLdsChunk; ++i) k.x[i] = i < n ? k.x[i] : kDown16;
#pragma unroll
        for (uint32_t i = 0; i < kLdsChunk; ++i) {
          k.dt[i] = dist[k.x[i] & kNodeMax];
          k.cand[i] = k.dv + ((k.x[i] & kDown16) ? 0u : wt(b + i));
        }
      };
      for (uint32_t r = 2;; ++r) {
        // the queue is walked transposed: lane l of a wave takes entries
        // l * M + j (M = ceil(nq / 64)), so the lanes of one instruction
        // hold chunks of nodes far apart in the queue (other pods / planes)
        // instead of neighbours pushing into the same targets -- same-address
        // LDS atomics within one instruction serialise
        uint32_t* qc = &qCount[r & 1u];
        if constexpr (kBfs) {
          // one constant weight wc > 0: the rounds are BFS layers; layer
          // r - 1 (distance (r - 1) wc) is final with complete next hops.
          // (0) the queue of the frontier's chunk records (four per thread
          // per step, the workgroup stepping together: every lane takes part
          // in the ballots), whether any node is still unreached, and how
          // many chunk records the unreached nodes own (the pull's work; the
          // push's is the queue)
          const uint64_t lay = uint64_t(r - 1u) * wc;
          uint32_t* cost = &qCount[2u + 2u * (r & 1u)];  // unreached chunk records
          // "any node unreached": on symmetric graphs every node with an
          // in-edge owns a chunk record, so the chunk count below decides it
          // (no separate node scan, a plain barrier); otherwise scan the nodes
          bool unreached = false;
          if (!sym) {
            for (uint32_t v = tid; v < N; v += B) unreached |= dist[v] == kInf;
          }
          uint32_t unrCh = 0;  // wave-uniform
          for (uint32_t c0 = 0; c0 < C; c0 += 4u * B) {
            uint32_t cs[4], vs[4], dk[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              cs[k] = c0 + uint32_t(k) * B + tid;
              vs[k] = cs[k] < C ? cnode[cs[k]] : kDrained16;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) dk[k] = cs[k] < C ? dist[vs[k] & kNodeMax] : 0u;
            uint64_t m[4];
            uint32_t tot = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              unrCh += uint32_t(__popcll(__ballot(dk[k] == kInf)));
              m[k] = __ballot(!(vs[k] & kDrained16) && uint64_t(dk[k]) == lay);
              tot += uint32_t(__popcll(m[k]));
            }
            if (tot == 0u) continue;  // wave-uniform
            uint32_t at = 0;
            if (lane == 0u) at = atomicAdd(qc, tot);
            at = __shfl(at, 0, 64);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t lo = static_cast<uint32_t>(m[k]), hi = static_cast<uint32_t>(m[k] >> 32);
              const uint32_t before = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
              if ((m[k] >> lane) & 1u) queue[at + before] = uint16_t(cs[k]);
              at += uint32_t(__popcll(m[k]));
            }
          }
          if (lane == 0u && unrCh) atomicAdd(cost, unrCh);
          if (sym) {
            __syncthreads();
          } else {
            unreached = __syncthreads_or(unreached);
          }
          mark(8u + 3u * (r - 2u));
          const uint32_t nq = *qc;
          const uint32_t pullT = *cost;
          if (sym) unreached = pullT != 0u;
          // no frontier: the fixpoint; nothing unreached: layer r is empty
          // -- round r's pushes can neither reach a node nor be tight
          if (nq == 0u) break;
          if (!unreached && !(flags & kFlagLdsNoBfsExit)) break;
          dg.queued(nq);
          if (tid == 0u) {  // next round's counters
            const uint32_t o = (r + 1u) & 1u;
            qCount[o] = 0u;
            qCount[2u + 2u * o] = 0u;
          }
          const uint32_t ratio = (flags >> kFlagLdsPullShift) & 0xFu;
          if (sym && ratio && 4u * uint64_t(pullT) <= uint64_t(ratio) * nq) {
            // pull (direction-optimising BFS): fewer chunk records (edges / 8)
            // of unreached nodes than of the frontier. Each unreached node
            // scans its own row -- with every edge's reverse present and of
            // the same up / down state (sym, checked by the prep) and one
            // weight, v -> u up means u -> v relaxes -- and ORs the next hops
            // of its neighbours in layer r - 1 that are not drained (the
            // source is layer 0, never such a neighbour): no LDS atomics,
            // one store per reached node
            const uint32_t cand = uint32_t(lay) + wc;
            // one chunk (<= 8 edges) of an unreached node: OR the next hops
            // of its tight, not drained neighbours into acc
            auto pullChunk = [&](uint32_t j0, uint32_t e, uint32_t (&acc)[W]) {
              uint32_t x[kLdsChunk], du[kLdsChunk], dr[kLdsChunk];
#pragma unroll
              for (uint32_t i = 0; i < kLdsChunk; ++i) x[i] = j0 + i < e ? eimg[j0 + i] : kDown16;
#pragma unroll
              for (uint32_t i = 0; i < kLdsChunk; ++i) {
                du[i] = dist[x[i] & kNodeMax];
                dr[i] = stamp[x[i] & kNodeMax];
              }
              // branch-free: every neighbour's words are read (padding lanes
              // read node 0) and masked, so the 8 x W reads issue together
              bool found = false;
              uint32_t nb[kLdsChunk][W];
#pragma unroll
              for (uint32_t i = 0; i < kLdsChunk; ++i) {
#pragma unroll
                for (int w = 0; w < W; ++w) nb[i][w] = nh[(x[i] & kNodeMax) * W + w];
              }
#pragma unroll
              for (uint32_t i = 0; i < kLdsChunk; ++i) {
                const bool t = !(x[i] & kDown16) && !dr[i] && uint64_t(du[i]) == lay;
                found |= t;
#pragma unroll
                for (int w = 0; w < W; ++w) acc[w] |= t ? nb[i][w] : 0u;
              }
              return found;
            };
            // (a) per unreached node its first chunk; further chunks of
            // long rows go to a list (the queue array: the frontier queue is
            // not used by a pull) for (b), one thread per chunk. Writes here
            // only touch nodes unreached at the pass start (distance kInf),
            // which no read in this pass can take for layer r - 1
            uint32_t* oc = &qCount[3u + 2u * (r & 1u)];  // the list's count
            if (tid == 0u) *oc = 0u;
            __syncthreads();
            for (uint32_t v = tid; v < N; v += B) {
              if (dist[v] != kInf) continue;
              const uint32_t b = row[v], e = row[v + 1];
              uint32_t acc[W];
#pragma unroll
              for (int w = 0; w < W; ++w) acc[w] = 0u;
              const bool found = b < e && pullChunk(b, min(e, b + kLdsChunk), acc);
              if (e > b + kLdsChunk) {
                const uint32_t f = first[v], n = (e - b + kLdsChunk - 1u) / kLdsChunk;
                const uint32_t at = atomicAdd(oc, n - 1u);
                for (uint32_t k = 1; k < n; ++k) queue[at + k - 1u] = uint16_t(f + k);
              }
              if (found) {
                dist[v] = cand;
#pragma unroll
                for (int w = 0; w < W; ++w) nh[v * W + w] = acc[w];
              }
            }
            __syncthreads();
            // (b) the listed chunks: distance by plain stores (every finder
            // stores the same), next hops by atomicOr. (Walked in list order:
            // the transposed walk of the push queue measured 1.8x slower here,
            // profiles/r05_lds_stamps_n8_pulltransposed.log)
            const uint32_t no = *oc;
            for (uint32_t i = tid; i < no; i += B) {
              const uint32_t c = queue[i];
              const uint32_t v = cnode[c] & kNodeMax;
              const uint32_t b = row[v] + kLdsChunk * (c - first[v]);
              uint32_t acc[W];
#pragma unroll
              for (int w = 0; w < W; ++w) acc[w] = 0u;
              if (pullChunk(b, min(row[v + 1], b + kLdsChunk), acc)) {
                dist[v] = cand;
#pragma unroll
                for (int w = 0; w < W; ++w) {
                  if (acc[w]) atomicOr(&nh[v * W + w], acc[w]);
                }
              }
            }
            __syncthreads();
            mark(8u + 3u * (r - 2u) + 2u);
            dg.rounds(r);
            continue;
          }
          // push: the nodes queued are layer r - 1; a target is either
          // unreached (dt = kInf: it joins layer r, every lane that finds it
          // so stores the same distance) or already at cand (layer r, tight)
          // or nearer (not tight). One pass: distances by plain stores, next
          // hops by fire-and-forget atomicOr; layer membership is the
          // distance itself
          const uint32_t M = (nq + 63u) >> 6;
          auto entry = [&](uint32_t i) { return (i & 63u) * M + (i >> 6); };
          for (uint32_t i = tid; i < 64u * M; i += B) {
            const uint32_t q = entry(i);
            if (q >= nq) continue;
            Chunk k;
            load(q, k);
            uint32_t nv[W];
#pragma unroll
            for (int w = 0; w < W; ++w) nv[w] = nh[k.v * W + w];
#pragma unroll
            for (uint32_t e = 0; e < kLdsChunk; ++e) {
              if ((k.x[e] & kDown16) || (k.dt[e] != kInf && k.dt[e] != k.cand[e])) continue;
              const uint32_t t = k.x[e] & kNodeMax;
              if (k.dt[e] == kInf) dist[t] = k.cand[e];
#pragma unroll
              for (int w = 0; w < W; ++w) {
                if (nv[w]) atomicOr(&nh[t * W + w], nv[w]);
              }
            }
          }
          __syncthreads();
          mark(8u + 3u * (r - 2u) + 2u);
          dg.rounds(r);
          continue;
        }
        // general weights. Round stamps: 1..255, 0 = not pending
        const uint32_t stCur = stamp_of(r), stPrev = stamp_of(r - 1u), stNext = stamp_of(r + 1u);
        // (0) the queue of round r: four chunk slots per thread per step, the
        // workgroup stepping together (every lane takes part in the ballots)
        for (uint32_t c0 = 0; c0 < C; c0 += 4u * B) {
          uint32_t cs[4], vs[4];
          bool act[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            cs[k] = c0 + uint32_t(k) * B + tid;
            vs[k] = cs[k] < C ? cnode[cs[k]] : kDrained16;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            // exact u8 stamps: st(r) cycles through 1..255 and a node still
            // carrying last round's value (pushed then, unchanged since) is
            // cleared here, so every live stamp is st(r) or 0 -- a stale
            // stamp never matches again after 255 rounds (it would re-queue
            // settled nodes every round: no fixpoint exit on paths of 256+
            // hops), and unreached nodes are never queued
            const uint32_t v = vs[k] & kNodeMax;
            const uint32_t sv = stamp[v];
            if (sv == stPrev) stamp[v] = 0;
            act[k] = !(vs[k] & kDrained16) && sv == stCur;
          }
          uint64_t m[4];
          uint32_t tot = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            m[k] = __ballot(act[k]);
            tot += uint32_t(__popcll(m[k]));
          }
          if (tot == 0u) continue;  // wave-uniform
          uint32_t at = 0;
          if (lane == 0u) at = atomicAdd(qc, tot);
          at = __shfl(at, 0, 64);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t lo = static_cast<uint32_t>(m[k]), hi = static_cast<uint32_t>(m[k] >> 32);
            const uint32_t before = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
            if (act[k]) queue[at + before] = uint16_t(cs[k]);
            at += uint32_t(__popcll(m[k]));
          }
        }
        __syncthreads();
        mark(8u + 3u * (r - 2u));
        const uint32_t nq = *qc;
        if (nq == 0u) break;  // nothing stamped r: the fixpoint
        dg.queued(nq);
        if (tid == 0u) qCount[(r + 1u) & 1u] = 0u;  // next round's counter
        const uint32_t M = (nq + 63u) >> 6;
        auto entry = [&](uint32_t i) { return (i & 63u) * M + (i >> 6); };
        // (1) distances. A push with cand < dt (dt read during this pass;
        // distances only fall) lowers its target whatever else lands there,
        // so it restarts the target's next hops without the atomic's return
        // value: every LDS operation here is fire-and-forget
        for (uint32_t i = tid; i < 64u * M; i += B) {
          const uint32_t q = entry(i);
          if (q >= nq) continue;
          Chunk k;
          load(q, k);
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) {
            if ((k.x[i] & kDown16) || k.cand[i] >= k.dt[i]) continue;
            const uint32_t t = k.x[i] & kNodeMax;
            atomicMin(&dist[t], k.cand[i]);
            stamp[t] = uint8_t(stNext);
#pragma unroll
            for (int w = 0; w < W; ++w) nh[t * W + w] = 0u;
          }
        }
        __syncthreads();
        mark(8u + 3u * (r - 2u) + 1u);
        // (2) next hops along tight edges, from the queued nodes still at the
        // distance they were queued with: the targets' words read first, then
        // fire-and-forget atomicOr of the missing bits
        for (uint32_t i = tid; i < 64u * M; i += B) {
          const uint32_t q = entry(i);
          if (q >= nq) continue;
          Chunk k;
          load(q, k);
          if (stamp[k.v] != stCur) continue;
          uint32_t nv[W];
#pragma unroll
          for (int w = 0; w < W; ++w) nv[w] = nh[k.v * W + w];
          bool tight[kLdsChunk];
          uint32_t have[kLdsChunk][W];
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) {
            tight[i] = !(k.x[i] & kDown16) && k.cand[i] == k.dt[i];
#pragma unroll
            for (int w = 0; w < W; ++w) {
              have[i][w] = nh[(k.x[i] & kNodeMax) * W + w];
              have[i][w] = tight[i] ? have[i][w] : ~0u;
            }
          }
#pragma unroll
          for (uint32_t i = 0; i < kLdsChunk; ++i) {
            const uint32_t t = k.x[i] & kNodeMax;
            bool add = false;
#pragma unroll
            for (int w = 0; w < W; ++w) {
              const uint32_t a = nv[w] & ~have[i][w];
              if (a) {
                atomicOr(&nh[t * W + w], a);
                add = true;
              }
            }
            if (add) stamp[t] = uint8_t(stNext);
          }
        }
        __syncthreads();
        mark(8u + 3u * (r - 2u) + 2u);
        dg.rounds(r);
      }
    };
    if (constW && wc > 0u) {
      rounds(std::true_type{}, std::true_type{});
    } else if (constW) {
      rounds(std::true_type{}, std::false_type{});
    } else {
      rounds(std::false_type{}, std::false_type{});
    }
    for (uint32_t v = tid; v < N; v += B) {
      oDist[size_t(u) * Sn + v] = dist[v];
#pragma unroll
      for (int w = 0; w < W; ++w) oNh[(size_t(u) * W + w) * Sn + v] = nh[v * W + w];
    }
    __syncthreads();  // state and outputs of this unit done before the next
    dg.unit_done();
  }
}

template <int W>
__global__ __launch_bounds__(kLdsBlock) void spf_lds_kernel(
    ogs_graph g, LdsImage L, const uint8_t* __restrict__ img, const uint4* __restrict__ mm,
    uint32_t nEB, const ogs_unit* __restrict__ units, int nUnits, uint32_t flags,
    uint32_t* __restrict__ oDist, uint32_t* __restrict__ oNh) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint32_t qCount[6];
  LdsWg wg;
#ifdef OGS_STAMPS
  LdsStamps dg(W);
#else
  NoDiag dg;
#endif
  for (int u = int(blockIdx.x); u < nUnits; u += int(gridDim.x)) {
    spf_lds_unit<W>(g, L, img, mm, nEB, units[u], uint32_t(u), flags, oDist, oNh, smem, qCount,
                    wg, dg);
  }
#ifdef OGS_STAMPS
  dg.finish();
#endif
}

// The unit's SPF state as published in HBM (ogs_spf_out layout), for the
// stream's route_one on SLOW prefixes.
template <int W>
struct PublishedView {
  const uint32_t* d;  // dist + u*Sn
  const uint32_t* n;  // nh + u*W*Sn
  uint32_t Sn;
  __device__ __forceinline__ uint32_t dist(uint32_t v) const { return d[v]; }
  __device__ __forceinline__ uint32_t nh(uint32_t v, int w) const {
    return n[size_t(w) * Sn + v];
  }
};

// Unit groups of one launch of the one-launch form: each group's units
// share a next-hop width W and output arrays (ogs_spf_routes_groups). Global
// unit index gu = group base + local index; groups are laid out widest
// first (their SPFs are the slowest, so they start first).
constexpr int kMaxLdsGroups = 4;
struct LdsGroup {
  const ogs_unit* units;
  uint32_t n, base, W, outs3;
  uint32_t* dist;  // [n * Sn] published SPF rows
  uint32_t* nh;    // [n * W * Sn]
  ogs_spf_out out;
};
struct LdsGroups {
  LdsGroup g[kMaxLdsGroups];
  uint32_t n;
};

// One stream item: prefix range `part` (of P) of local unit u of group grp,
// from the published SPF rows: per-node records into LDS, then the rows.
template <int W, typename KeyT>
__device__ __forceinline__ void lds_stream_item(const ogs_graph& g, const ogs_prefix_table& pt,
                                                const KeyT* __restrict__ key,
                                                const LdsGroup& grp, uint32_t u, uint32_t part,
                                                uint32_t P, uint32_t flags, uint32_t* rec0) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const uint32_t tid = threadIdx.x;
  const uint32_t Sn = uint32_t(g.max_nodes), Sp = uint32_t(pt.max_prefixes);
  const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0, (flags & OGS_F_V4_OVER_V6) != 0,
                     (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
  const ogs_unit unit = grp.units[u];
  const uint32_t t = unit.topo, s = unit.src;
  const uint32_t nb = g.node_base[t];
  const uint32_t N = g.node_base[t + 1] - nb;
  // the prefix range's bounds load with the node range (one round), not
  // after the records' barrier
  const uint32_t p0 = pt.pfx_base[t];
  const uint32_t Pn = pt.pfx_base[t + 1] - p0;
  const uint8_t* __restrict__ nflags = g.node_flags + nb;
  const PublishedView<W> sv{grp.dist + size_t(u) * Sn, grp.nh + size_t(u) * W * Sn, Sn};
  uint32_t* rMeta = rec0;
  uint32_t* rMetric = rMeta + Sn;
  uint32_t* rMask = rMetric + Sn;  // [W][Sn]
  // the records of K nodes per thread per batch: every row load of the batch
  // is issued before the first record is built (one L2 round trip per batch
  // of K x 1024 nodes instead of one per 1024)
  constexpr int K = 3;
  for (uint32_t v0 = tid; v0 < N; v0 += K * kLdsBlock) {
    uint32_t d[K], m[K][W];
    uint8_t nf[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t v = v0 + uint32_t(k) * kLdsBlock;
      const uint32_t vc = v < N ? v : v0;  // clamped: unconditional loads
      d[k] = sv.dist(vc);
      nf[k] = nflags[vc];
#pragma unroll
      for (int w = 0; w < W; ++w) m[k][w] = sv.nh(vc, w);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t v = v0 + uint32_t(k) * kLdsBlock;
      if (v >= N) break;
      uint32_t cnt = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) cnt += __popc(m[k][w]);
      rMeta[v] = node_route_meta(v, s, d[k] != kInf, cnt, nf[k]);
      rMetric[v] = (v == s) ? kInf : d[k];
#pragma unroll
      for (int w = 0; w < W; ++w) rMask[w * Sn + v] = m[k][w];
    }
  }
  __syncthreads();
  const uint32_t span = ((Pn + P - 1u) / P + 3u) & ~3u;
  const uint32_t lo = min(Pn, part * span), hi = min(Pn, lo + span);
  auto rec = [&](uint32_t v, Rec<W>& r) {
    r.meta = rMeta[v];
    r.metric = rMetric[v];
#pragma unroll
    for (int w = 0; w < W; ++w) r.mask[w] = rMask[w * Sn + v];
  };
  const bool nt = (flags & kFlagNtStores) != 0;
  if (grp.outs3) {
    stream_routes<W, false, true, kLdsBlock>(pt, key + size_t(t) * Sp, p0, Pn, Sp, u, s, nflags,
                                             sv, cfg, grp.out, rec, nullptr, nt, lo, hi);
  } else {
    stream_routes<W, false, false, kLdsBlock>(pt, key + size_t(t) * Sp, p0, Pn, Sp, u, s,
                                              nflags, sv, cfg, grp.out, rec, nullptr, nt, lo,
                                              hi);
  }
  __syncthreads();  // the records are read before the next item reuses LDS
}

// SPF and RouteDb stream in ONE persistent launch (route_stream 5): each
// workgroup takes items from a device-wide counter --
//   items [0, G): the SPF of unit i (G = min(units, grid): every workgroup
//     starts with one);
//   then per stream slot b, P + 1 items: the SPF of unit G + b (when there
//     is one), then the P prefix ranges of slot b's unit
// (unit = global index over the groups, widest group first). Stream slot b
// is unit b, except that with a lead (sharded builds: every workgroup's
// first SPF is its only one) the first `lead` slots are narrow units, whose
// SPFs finish first, then the Uw wide ones, then the rest: the first
// stream items do not wait on the slow wide SPFs, and the wide units' large
// items still come early instead of at the launch's tail. The slots' units
// are a bijection whose SPF is always handed out earlier (Uw <= G), so a
// stream item only ever waits for an SPF that a running workgroup holds and
// the spin always ends; a shard with a few more units than CUs streams
// other units' rows while its last SPFs run. The last U - U1 slots stream in
// P2 > P ranges: small items at the end of the queue shorten the launch's
// tail (profiles/r05_c3_timeline_*.log: a workgroup's idle tail is about
// half an item). Hand-off (MI355X_MICROARCH.md, inter-workgroup
// visibility): the SPF's dist / nh rows are plain stores, drained by every
// wave, then a barrier, lane 0's agent release and a relaxed agent flag
// store; a stream item's lane 0 polls the flag (relaxed agent loads), takes
// an agent acquire, and the workgroup reads the rows after a barrier.
struct LdsSchedule {
  uint32_t P, P2, U1;  // ranges per slot: P for slots [0, U1), P2 after
  uint32_t lead, Uw;   // slot -> unit: lead narrow units before the Uw wide
};

// WMAX: the widest next-hop width the launch's groups use (3 or 4). The
// kernel runs at 1024 threads per workgroup, so every wave has 128 VGPRs;
// with the W = 4 SPF / stream paths compiled in, the kernel spilled 44 B per
// lane to scratch (and 60 B at 8f3cd6b), which cost the whole-node C3 build
// 1.134 vs 1.088 ms and 62 MB of scratch reads per build
// (profiles/r06_c3_bisect.log); a launch whose groups are at most 3 words
// wide takes the WMAX = 3 form, which has no W = 4 path and no spills.
template <typename KeyT, int WMAX>
__global__ __launch_bounds__(kLdsBlock) void spf_lds_route_kernel(
    ogs_graph g, ogs_prefix_table pt, const KeyT* __restrict__ key, LdsImage L,
    const uint8_t* __restrict__ img, const uint4* __restrict__ mm, uint32_t nEB,
    LdsGroups grps, uint32_t flags, uint32_t* __restrict__ ctr, uint32_t* __restrict__ ready,
    LdsSchedule sch) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint32_t qCount[6];
  __shared__ uint32_t item;
  const uint32_t tid = threadIdx.x;
  const LdsGroup& last = grps.g[grps.n - 1u];
  const uint32_t U = last.base + last.n;
  const uint32_t G = min(U, gridDim.x);
  const uint32_t P = sch.P, P2 = sch.P2, U1 = sch.U1;
  const uint32_t headItems = U1 * (P + 1u);
  const uint32_t total = G + headItems + (U - U1) * (P2 + 1u);
  auto slotUnit = [&](uint32_t b) -> uint32_t {
    if (b < sch.lead) return sch.Uw + b;
    if (b < sch.lead + sch.Uw) return b - sch.lead;
    return b;
  };
  LdsWg wg;
  NoDiag dg;
#ifdef OGS_STAMPS
  uint32_t nStamp = 0;
  uint32_t* st = g_itemStamps + size_t(blockIdx.x) * kItemStamps * 4u;
  const bool stOn = tid == 0u && blockIdx.x < kLdsDiagWgsItems;
  auto rt = [] { return uint32_t(__builtin_amdgcn_s_memrealtime()); };
#define OGS_ITEM_STAMP(kind, unit, t0, t1)                                       \
  if (stOn && nStamp < kItemStamps) {                                            \
    st[4 * nStamp + 0] = (uint32_t(kind) << 28) | (unit);                        \
    st[4 * nStamp + 1] = (t0);                                                   \
    st[4 * nStamp + 2] = (t1);                                                   \
    st[4 * nStamp + 3] = rt();                                                   \
    ++nStamp;                                                                    \
  }
#else
#define OGS_ITEM_STAMP(kind, unit, t0, t1)
#endif
  // one topology (every unit's): its image is staged while the first item
  // is fetched, the counter's round trip hidden behind the image loads
  bool preStage = g.num_topos == 1;
  for (;;) {
#ifdef OGS_STAMPS
    const uint32_t tItem = rt();
#endif
    uint32_t fetched = 0u;
    if (tid == 0u) fetched = atomicAdd(ctr, 1u);
    if (preStage) {
      lds_stage(g, L, img, mm, nEB, 0u, smem, wg);
      preStage = false;
    }
    if (tid == 0u) item = fetched;
    __syncthreads();
    const uint32_t i0 = item;
    __syncthreads();  // every lane has read item before lane 0 takes the next
    if (i0 >= total) break;
    const uint32_t i = i0;
    uint32_t gu = i, part = 0, parts = P;
    bool spf = true;
    if (i >= G) {
      uint32_t j = i - G, r, b;
      if (j < headItems) {
        b = j / (P + 1u);
        r = j - b * (P + 1u);
      } else {
        j -= headItems;
        const uint32_t k = j / (P2 + 1u);
        r = j - k * (P2 + 1u);
        b = U1 + k;
        parts = P2;
      }
      if (r == 0u) {
        gu = G + b;
        if (gu >= U) continue;
      } else {
        spf = false;
        part = r - 1u;
        gu = slotUnit(b);
      }
    }
    uint32_t gi = 0;
    while (gi + 1u < grps.n && gu >= grps.g[gi + 1u].base) ++gi;
    const LdsGroup& grp = grps.g[gi];
    const uint32_t u = gu - grp.base;
    if (spf) {
      const ogs_unit unit = grp.units[u];
      switch (grp.W) {
        case 1: spf_lds_unit<1>(g, L, img, mm, nEB, unit, u, flags, grp.dist, grp.nh, smem, qCount, wg, dg); break;
        case 2: spf_lds_unit<2>(g, L, img, mm, nEB, unit, u, flags, grp.dist, grp.nh, smem, qCount, wg, dg); break;
        case 3: spf_lds_unit<3>(g, L, img, mm, nEB, unit, u, flags, grp.dist, grp.nh, smem, qCount, wg, dg); break;
        default:
          if constexpr (WMAX >= 4) {
            spf_lds_unit<4>(g, L, img, mm, nEB, unit, u, flags, grp.dist, grp.nh, smem, qCount, wg, dg);
          }
          break;
      }
      // publish: every wave's row stores drained, barrier, release, flag
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0u) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&ready[gu], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      OGS_ITEM_STAMP(1u, gu, tItem, tItem);
      continue;
    }
    if (tid == 0u) {
      while (__hip_atomic_load(&ready[gu], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(8);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
#ifdef OGS_STAMPS
    const uint32_t tReady = rt();
#endif
    // the per-node records go to the state region (the image stays)
    uint32_t* rec0 = reinterpret_cast<uint32_t*>(smem + L.block);
    switch (grp.W) {
      case 1: lds_stream_item<1, KeyT>(g, pt, key, grp, u, part, parts, flags, rec0); break;
      case 2: lds_stream_item<2, KeyT>(g, pt, key, grp, u, part, parts, flags, rec0); break;
      case 3: lds_stream_item<3, KeyT>(g, pt, key, grp, u, part, parts, flags, rec0); break;
      default:
        if constexpr (WMAX >= 4) lds_stream_item<4, KeyT>(g, pt, key, grp, u, part, parts, flags, rec0);
        break;
    }
    OGS_ITEM_STAMP(2u, gu, tItem, tReady);
  }
#undef OGS_ITEM_STAMP
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

// Workspace bytes of the LDS paths for this batch (lds_scratch), or 0 when
// it does not qualify: nodes fit 15 bits, chunk ids 16 bits, the image + one
// unit's state (and the megakernel's per-node records) fit LDS.
size_t lds_scratch_bytes(const ogs_graph& g, int W, int nUnits) {
  if (g.max_nodes <= 0 || uint32_t(g.max_nodes) > kNodeMax || W < 1 || W > 4) return 0;
  const uint32_t cap = chunk_cap(uint32_t(g.max_nodes), uint32_t(g.max_edges));
  if (cap > 0xFFFFu || uint32_t(g.max_edges) > 0xFFFFFFu) return 0;
  const LdsImage L = lds_image(g, W);
  const uint32_t recs = uint32_t(g.max_nodes) * uint32_t(2 + W) * 4u;
  if (L.block + std::max(L.state, recs) + 512u > 160u * 1024u) return 0;  // + static LDS
  return lds_scratch(g, L, nUnits).bytes;
}

// Prep launch (lds_prep_kernel): images, weight partials, counters, and the
// route keys when key != nullptr.
hipError_t launch_lds_prep(const ogs_graph& g, const ogs_prefix_table* pt, void* key,
                           bool key16, int W, int nUnits, void* scratch, hipStream_t stream) {
  const LdsImage L = lds_image(g, W);
  const LdsScratch S = lds_scratch(g, L, nUnits);
  uint8_t* base = static_cast<uint8_t*>(scratch);
  const uint32_t T = uint32_t(g.num_topos);
  const uint32_t Sp = pt ? uint32_t(pt->max_prefixes) : 0u;
  const uint32_t nKB = key && Sp ? (Sp + kPrepKeys - 1u) / kPrepKeys : 0u;
  const ogs_prefix_table ptv = pt ? *pt : ogs_prefix_table{};
  hipLaunchKernelGGL(lds_prep_kernel, dim3(T * (1u + S.nEB + nKB)), dim3(kLdsBlock), 0, stream,
                     g, ptv, nKB ? key : nullptr, key16 ? 1u : 0u, nKB, L, base,
                     reinterpret_cast<uint4*>(base + S.mm), S.nEB,
                     reinterpret_cast<uint32_t*>(base + S.ctr),
                     reinterpret_cast<uint32_t*>(base + S.ready), uint32_t(nUnits));
  return hipGetLastError();
}

template <typename K>
static hipError_t allow_lds(K k, uint32_t lds) {
  if (lds <= 64u * 1024u) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                             hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
}

// SPF of every unit into dist / nh (u32 distances, W next-hop words) after
// launch_lds_prep: one persistent 1024-thread workgroup per CU over the
// units. Call only when lds_scratch_bytes() != 0.
hipError_t launch_spf_lds(const ogs_graph& g, const ogs_unit* units, int nUnits,
                          uint32_t flags, int W, uint32_t* dist, uint32_t* nh,
                          void* scratch, hipStream_t stream) {
  const LdsImage L = lds_image(g, W);
  const LdsScratch S = lds_scratch(g, L, nUnits);
  const uint8_t* img = static_cast<const uint8_t*>(scratch);
  const uint4* mm = reinterpret_cast<const uint4*>(img + S.mm);
  const uint32_t lds = L.block + L.state;
  const int grid = std::max(1, std::min(nUnits, num_cus()));
  if (!opts().ldsBfsExit) flags |= kFlagLdsNoBfsExit;
  flags |= uint32_t(opts().ldsPull & 0xF) << kFlagLdsPullShift;
  auto go = [&](auto k) {
    hipError_t a = allow_lds(k, lds);
    if (a != hipSuccess) return a;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kLdsBlock), lds, stream, g, L, img, mm, S.nEB,
                       units, nUnits, flags, dist, nh);
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

// "lds_parts": prefix ranges per unit in the one-launch form (0 = by
// regime, default); "lds_grid": its workgroups (0 = one per CU).
// EngineOptions::ldsParts (engine.h), default 0
// EngineOptions::ldsGrid (engine.h), default 0
// "lds_key16": packed 16-bit route keys on topologies of <= 16,384 nodes
// (1, default) or u32 keys (0, A/B)
// EngineOptions::ldsKey16 (engine.h), default 1
// EngineOptions::ldsTail (engine.h), default 1
// "lds_bfs_exit": the BFS rounds stop once every node is reached (1,
// default) or run the empty last layer (0, A/B): C3 N = 8 shard 0.1695 vs
// 0.1732 ms (profiles/r05_c3_ab_bfs_exit.log)
// EngineOptions::ldsBfsExit (engine.h), default 1
// "lds_pull": BFS rounds pull when 4 x (chunk records of the unreached
// nodes) <= lds_pull x (the frontier's); 0 always push (A/B)
// EngineOptions::ldsPull (engine.h), default 6
// "lds_lead": narrow units streamed before the wide group (0, default:
// none; -1 one grid's worth of stream items on sharded builds; measured at
// the N = 8 shard 0.1752 vs 0.1711 ms without, N = 4 0.3031 vs 0.3074 with
// the tail change alone: profiles/r05_c3_lead_tail_ab_n*.log);
// "lds_tail_parts": ranges per unit of the launch's last units (0 auto)
// EngineOptions::ldsLead (engine.h), default 0
// EngineOptions::ldsTailParts (engine.h), default 0

bool lds_key16(const ogs_graph& g) {
  return opts().ldsKey16 && g.max_nodes > 0 && uint32_t(g.max_nodes) <= kKey16MaxNodes;
}

// SPF + RouteDb stream of every group in one persistent launch
// (spf_lds_route_kernel) after launch_lds_prep (keys, and the image laid out
// for the widest group; nUnits = all groups' units). groups: n <= 4, widest
// first, each with its published dist / nh rows. key16: lds_key16(g).
hipError_t launch_spf_lds_routes(const ogs_graph& g, const ogs_prefix_table& pt,
                                 const void* key, bool key16, const LdsRouteGroup* groups,
                                 int n, uint32_t flags, void* scratch, hipStream_t stream) {
  if (n < 1 || n > kMaxLdsGroups) return hipErrorInvalidValue;
  int Wmax = 1, U = 0;
  LdsGroups G{};
  G.n = uint32_t(n);
  for (int i = 0; i < n; ++i) {
    const LdsRouteGroup& x = groups[i];
    if (x.W < 1 || x.W > 4) return hipErrorInvalidValue;
    Wmax = std::max(Wmax, x.W);
    G.g[i] = LdsGroup{x.units, uint32_t(x.n), uint32_t(U), uint32_t(x.W),
                      (x.out.meta && x.out.metric && x.out.mask && !x.out.sel) ? 1u : 0u,
                      x.dist, x.nh, x.out};
    U += x.n;
  }
  const LdsImage L = lds_image(g, Wmax);
  const LdsScratch S = lds_scratch(g, L, U);
  uint8_t* base = static_cast<uint8_t*>(scratch);
  const uint4* mm = reinterpret_cast<const uint4*>(base + S.mm);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(base + S.ctr);
  uint32_t* ready = reinterpret_cast<uint32_t*>(base + S.ready);
  // the prep launch: images, weight partials, zeroed counters, route keys
  hipError_t e = launch_lds_prep(g, &pt, const_cast<void*>(key), key16, Wmax, U, scratch, stream);
  if (e != hipSuccess) return e;
  const uint32_t recs = uint32_t(g.max_nodes) * uint32_t(2 + Wmax) * 4u;
  const uint32_t lds = L.block + std::max(L.state, recs);
  const int grid = std::max(1, opts().ldsGrid > 0 ? opts().ldsGrid : num_cus());
  // prefix ranges per unit: "lds_parts", or 0 = by regime -- 2 when every
  // workgroup has four or more units (whole-node builds: fewer record
  // rebuilds), 4 below that (sharded builds: more items to balance a few
  // units per CU); profiles/r04_lds_store_parts_ab.log
  const uint32_t P = opts().ldsParts > 0 ? uint32_t(opts().ldsParts)
                                    : (uint32_t(U) >= 4u * uint32_t(grid) ? 2u : 4u);
  const bool sharded = uint32_t(U) < 4u * uint32_t(grid);
  // the launch's last units stream in P2 > P ranges ("lds_tail" 1,
  // default): whole-node builds the last grid's worth of units in 4,
  // sharded builds the last grid's worth of ITEMS in "lds_tail_parts"
  // (auto 8); 0 every unit in P
  LdsSchedule sch{P, P, uint32_t(U), 0u, 0u};
  if (opts().ldsTail) {
    if (!sharded && P < 4u) {
      sch.P2 = 4u;
      sch.U1 = uint32_t(U - std::min(U, grid));
    } else if (sharded) {
      sch.P2 = opts().ldsTailParts > 0 ? uint32_t(opts().ldsTailParts) : 2u * P;
      const uint32_t tailUnits = std::min(uint32_t(U), (uint32_t(grid) + sch.P2 - 1u) / sch.P2);
      sch.U1 = uint32_t(U) - tailUnits;
    }
    if (sch.P2 <= P) sch.U1 = uint32_t(U);
  }
  // lead ("lds_lead"; -1: on sharded builds with several width groups, one
  // grid's worth of stream items of narrow units before the wide group,
  // whose SPFs finish last); needs Uw <= G (the slot map's SPFs are then
  // always handed out before their stream items)
  const uint32_t Uw = n > 1 ? uint32_t(groups[0].n) : 0u;
  const uint32_t Gl = std::min(uint32_t(U), uint32_t(grid));
  if (Uw > 0u && Uw <= Gl) {
    const uint32_t want = opts().ldsLead >= 0 ? uint32_t(opts().ldsLead)
                                         : (sharded ? (uint32_t(grid) + P - 1u) / P : 0u);
    sch.lead = std::min(want, uint32_t(U) - Uw);
    sch.Uw = sch.lead ? Uw : 0u;
  }
  if (opts().routeStoreNt & 1) flags |= kFlagNtStores;
  if (!opts().ldsBfsExit) flags |= kFlagLdsNoBfsExit;
  flags |= uint32_t(opts().ldsPull & 0xF) << kFlagLdsPullShift;
  auto go = [&](auto k, auto keyp) {
    hipError_t a = allow_lds(k, lds);
    if (a != hipSuccess) return a;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kLdsBlock), lds, stream, g, pt, keyp, L,
                       static_cast<const uint8_t*>(base), mm, S.nEB, G, flags, ctr, ready, sch);
    return hipGetLastError();
  };
  // the widest group picks the form (WMAX 3: no W = 4 path, no spills)
  if (Wmax <= 3) {
    return key16 ? go(spf_lds_route_kernel<uint16_t, 3>, static_cast<const uint16_t*>(key))
                 : go(spf_lds_route_kernel<uint32_t, 3>, static_cast<const uint32_t*>(key));
  }
  return key16 ? go(spf_lds_route_kernel<uint16_t, 4>, static_cast<const uint16_t*>(key))
               : go(spf_lds_route_kernel<uint32_t, 4>, static_cast<const uint32_t*>(key));
}

}  // namespace ogs

#ifdef OGS_STAMPS
extern "C" int ogs_diag_item_stamps(uint32_t* host, int32_t words) {
  const size_t n = std::min<size_t>(size_t(words), size_t(ogs::kLdsDiagWgsItems) * ogs::kItemStamps * 4);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ogs::g_itemStamps), n * 4, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int ogs_diag_item_stamps_clear() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(ogs::g_itemStamps)) != hipSuccess) return -1;
  return hipMemset(p, 0, sizeof(ogs::g_itemStamps)) == hipSuccess ? 0 : -1;
}
extern "C" int ogs_diag_lds_stamps(uint32_t* host, int32_t words) {
  const size_t n = std::min<size_t>(size_t(words), size_t(4) * ogs::kLdsDiagWgs * 32);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ogs::g_ldsStamps), n * 4, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
