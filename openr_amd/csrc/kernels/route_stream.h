// route_stream.h — the RouteDb write stream of one unit (device code),
// shared by route_stream_kernel (SPF state read back from HBM) and the fused
// frontier SPF + RouteDb kernel (SPF state still in LDS).
//
// A single-advertiser prefix's route depends only on its advertiser v
// (SpfSolver::createRouteForPrefix, SpfSolver.cpp:160-311, on a one-entry
// segment; selectBestRoutes 455-551 and addBestPaths 595-639 degenerate):
//   unreachable v         -> reason UNREACHABLE          (217-223)
//   v == source           -> SELECTED, reason SELF        (253-258)
//   no next hop           -> reason NO_NEXTHOP            (605-607)
//   else                  -> VALID, metric dist(v), mask NH(v)
// plus DRAINED when v is hard-drained or has a metric increment
// (isNodeDrained, 543-551) and LOCAL when v is the source. So the stream
// keeps one record per NODE and gathers it per prefix; every other prefix
// (several advertisements, minNexthop, advertiser without adjacency DB) runs
// the full route_one (route_core.h). The per-prefix choice is precomputed
// once per call into a u32 key (pfx_key_kernel).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "route_core.h"
#include "spf_core.h"

namespace ogs {

constexpr uint32_t kKeySlow = 0x80000000u;  // run route_one
constexpr uint32_t kKeyV4 = 0x40000000u;    // prefix is IPv4 (run-time gate)
constexpr uint32_t kKeyNode = OGS_EDGE_DST_MASK;

// Record flags of a single-advertiser prefix advertised by v.
__device__ __forceinline__ uint32_t node_route_meta(uint32_t v, uint32_t s,
                                                    bool reachable,
                                                    uint32_t nhCount,
                                                    uint8_t nflag) {
  uint32_t meta = (v == s) ? OGS_ROUTE_LOCAL : 0u;
  if (!reachable) return meta | (OGS_REASON_UNREACHABLE << OGS_ROUTE_REASON_SHIFT);
  meta |= OGS_ROUTE_SELECTED;
  if (nflag & (OGS_NODE_OVERLOADED | OGS_NODE_METRICINC)) meta |= OGS_ROUTE_DRAINED;
  if (v == s) return meta | (OGS_REASON_SELF << OGS_ROUTE_REASON_SHIFT);
  return meta | (nhCount ? OGS_ROUTE_VALID
                         : (OGS_REASON_NO_NEXTHOP << OGS_ROUTE_REASON_SHIFT));
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Route key of prefix p (local index) of topology t (pfx_key_kernel / the
// LDS paths' prep kernel): the single advertiser's node | v4 bit, or SLOW.
__device__ __forceinline__ uint32_t prefix_key(const ogs_prefix_table& pt, uint32_t t,
                                               uint32_t p) {
  const uint32_t p0 = pt.pfx_base[t];
  const uint32_t P = pt.pfx_base[t + 1] - p0;
  uint32_t k = kKeySlow;
  if (p < P) {
    const uint32_t gp = p0 + p;
    const uint32_t a0 = pt.adv_off[gp], a1 = pt.adv_off[gp + 1];
    const uint8_t f = pt.pfx_flags[gp];
    if (a1 - a0 == 1 && !(f & OGS_PFX_HAS_MIN_NH)) {
      const uint32_t n = pt.adv_node[a0];
      if (n != OGS_NODE_NONE) k = n | ((f & OGS_PFX_V4) ? kKeyV4 : 0u);
    }
  }
  return k;
}

// Packed 16-bit route keys (topologies of at most 16,384 nodes): node id in
// bits 0..13, v4 bit 14, SLOW bit 15 -- the u32 key's bits 30 / 31 moved
// down 16. Halves the stream's key reads (every unit reads the whole row).
constexpr uint32_t kKey16MaxNodes = 1u << 14;
__device__ __forceinline__ uint16_t key16_of(uint32_t k) {
  return uint16_t((k & 0x3FFFu) | ((k >> 16) & 0xC000u));
}
__device__ __forceinline__ uint32_t key_of(uint16_t h) {
  return (uint32_t(h) & 0x3FFFu) | ((uint32_t(h) & 0xC000u) << 16);
}
__device__ __forceinline__ uint32_t key_of(uint32_t k) { return k; }

// one 16-B output store (route_core.h store_out: kFlagNtStores flavour)
__device__ __forceinline__ void store4(uint32_t* p, uint32_t a, uint32_t b, uint32_t c,
                                       uint32_t d, bool nt) {
  store_out(reinterpret_cast<u32x4*>(p), u32x4{a, b, c, d}, nt);
}

template <int W>
struct Rec {
  uint32_t meta, metric, mask[W], sel;
};

// Route diff against a base unit (ogs_route_diff; calculateUpdate,
// SpfSolver.cpp:21-56, RibUnicastEntry::operator==, RibEntry.h:81-87).
struct DiffCtx {
  const uint32_t* bMeta;    // [Sp]
  const uint32_t* bMetric;  // [Sp]
  const uint32_t* bMask;    // [W][Sp]
  uint32_t* changed;        // this unit's bitmap row (zeroed)
  uint32_t* counts;         // LDS {update, delete} accumulators
  const uint32_t* advOff;   // prefix p's first advertisement (pt.adv_off + p0)
  const uint32_t* advClass; // ogs_route_diff.adv_class or NULL
};

// Best-entry class of a valid route (ogs_route_diff.adv_class): the
// advertisement's entry as is, or with the hard-drain override.
__device__ __forceinline__ uint32_t best_class(const DiffCtx& d, uint32_t p, uint32_t meta) {
  const uint32_t a = d.advOff[p] + (meta >> OGS_ROUTE_BEST_SHIFT);
  return d.advClass[2u * a + ((meta & OGS_ROUTE_DRAINED) ? 1u : 0u)];
}

template <int W>
__device__ __forceinline__ bool route_changed(const Rec<W>& r, const DiffCtx& d,
                                              uint32_t Sp, uint32_t p,
                                              uint32_t& upd, uint32_t& del) {
  constexpr uint32_t kEq = OGS_ROUTE_DRAINED | OGS_ROUTE_LOCAL |
      (0xFFFFFFu << OGS_ROUTE_BEST_SHIFT);
  const uint32_t bm = d.bMeta[p];
  const bool va = r.meta & OGS_ROUTE_VALID, vb = bm & OGS_ROUTE_VALID;
  bool ch = va != vb;
  if (va && vb) {
    // bestPrefixEntry by value (RibEntry.h:81-87) when classes are given
    ch = (d.advClass ? (((r.meta ^ bm) & OGS_ROUTE_LOCAL) != 0u ||
                        best_class(d, p, r.meta) != best_class(d, p, bm))
                     : ((r.meta ^ bm) & kEq) != 0u) ||
        r.metric != d.bMetric[p];
#pragma unroll
    for (int w = 0; w < W; ++w) ch |= r.mask[w] != d.bMask[size_t(w) * Sp + p];
  }
  upd += (va && ch) ? 1u : 0u;
  del += (vb && !va) ? 1u : 0u;
  return ch;
}

// Streams unit u's route records of prefixes [lo, hi) (lo a multiple of 4;
// rows of stride Sp) with B threads. rec(v, r) fills meta / metric / mask of
// node v's record; sv is the unit's SPF state for route_one. Four
// consecutive prefixes per lane: one 16-B key load and one 16-B store per
// output array (non-temporal when nt). OUTS3: the caller guarantees meta,
// metric and mask outputs and no sel -- the stores are then unconditional,
// so every path leaves the same number of stores in flight and the key
// prefetch's wait stays partial (see the loop below).
template <int W, bool DIFF = false, bool OUTS3 = false, int B = kBlock, typename KeyT,
          typename View, typename RecFn>
__device__ __forceinline__ void stream_routes(
    const ogs_prefix_table& pt, const KeyT* __restrict__ tkey, uint32_t p0,
    uint32_t P, uint32_t Sp, size_t u, uint32_t s,
    const uint8_t* __restrict__ nflags, const View& sv, const RouteCfg& cfg,
    const ogs_spf_out& out, RecFn rec, const DiffCtx* diff = nullptr, bool nt = true,
    uint32_t lo = 0, uint32_t hi = 0xFFFFFFFFu) {
  uint32_t upd = 0, del = 0;
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const int tid = threadIdx.x;
  const bool v4Gated = !cfg.enableV4 && !cfg.v4OverV6;
  uint32_t* oMeta = out.meta ? out.meta + u * Sp : nullptr;
  uint32_t* oMetric =
      out.metric ? static_cast<uint32_t*>(out.metric) + u * Sp : nullptr;
  uint32_t* oSel = out.sel ? out.sel + u * Sp : nullptr;
  uint32_t* oMask = out.mask ? out.mask + u * W * Sp : nullptr;

  auto one = [&](uint32_t p, uint32_t k, Rec<W>& r) {
    if (!(k & kKeySlow)) {
      if ((k & kKeyV4) && v4Gated) {
        r.meta = OGS_REASON_V4_DISABLED << OGS_ROUTE_REASON_SHIFT;
        r.metric = kInf;
        r.sel = 0u;
#pragma unroll
        for (int w = 0; w < W; ++w) r.mask[w] = 0u;
        return;
      }
      rec(k & kKeyNode, r);
      r.sel = (r.meta & OGS_ROUTE_SELECTED) ? 1u : 0u;
    } else {
      route_one<uint32_t, W>(pt, p0 + p, s, nflags, sv, cfg, r.meta, r.metric,
                             r.mask, r.sel);
    }
  };

  // 16-B accesses need 16-B aligned rows: Sp % 4 == 0 and aligned bases
  const uintptr_t align = reinterpret_cast<uintptr_t>(out.meta) |
      reinterpret_cast<uintptr_t>(out.metric) |
      reinterpret_cast<uintptr_t>(out.sel) | reinterpret_cast<uintptr_t>(out.mask);
  const bool vec = (Sp & 3u) == 0u && (align & 15u) == 0u;
  hi = min(hi, P);
  lo = min(lo, hi);
  const uint32_t Pv = vec ? max(lo, hi & ~3u) : lo;
  auto quad = [&](uint32_t q, const uint4 k4) {
    Rec<W> r0, r1, r2, r3;
    one(q + 0, k4.x, r0);
    one(q + 1, k4.y, r1);
    one(q + 2, k4.z, r2);
    one(q + 3, k4.w, r3);
    if (OUTS3 || oMeta) store4(oMeta + q, r0.meta, r1.meta, r2.meta, r3.meta, nt);
    if (OUTS3 || oMetric) store4(oMetric + q, r0.metric, r1.metric, r2.metric, r3.metric, nt);
    if (!OUTS3 && oSel) store4(oSel + q, r0.sel, r1.sel, r2.sel, r3.sel, nt);
    if (OUTS3 || oMask) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        store4(oMask + size_t(w) * Sp + q, r0.mask[w], r1.mask[w], r2.mask[w], r3.mask[w],
               nt);
      }
    }
    if constexpr (DIFF) {
      // lane l holds prefixes q..q+3; the wave's 256 prefixes are 8 words:
      // word l (lanes 8l..8l+7) bit 4k+j = prefix 32l + 4k + j
      const uint64_t b0 = __ballot(route_changed<W>(r0, *diff, Sp, q + 0, upd, del));
      const uint64_t b1 = __ballot(route_changed<W>(r1, *diff, Sp, q + 1, upd, del));
      const uint64_t b2 = __ballot(route_changed<W>(r2, *diff, Sp, q + 2, upd, del));
      const uint64_t b3 = __ballot(route_changed<W>(r3, *diff, Sp, q + 3, upd, del));
      const int lane = threadIdx.x & 63;
      if (lane < 8) {
        uint32_t word = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int l = lane * 8 + k;
          word |= uint32_t((b0 >> l) & 1u) << (4 * k);
          word |= uint32_t((b1 >> l) & 1u) << (4 * k + 1);
          word |= uint32_t((b2 >> l) & 1u) << (4 * k + 2);
          word |= uint32_t((b3 >> l) & 1u) << (4 * k + 3);
        }
        // the wave's first prefix is q - 4 * lane (lane 0's q)
        const uint32_t w0 = (q - 4u * uint32_t(lane)) / 32u + uint32_t(lane);
        if (word) atomicOr(diff->changed + w0, word);
      }
    }
  };
  // Software-pipelined key loads: each quad's keys are loaded BEFORE the
  // previous quad's stores are issued. vmcnt counts loads and stores together
  // in issue order, so a key load issued after those stores would wait for
  // them to drain -- one store round trip per iteration. The first quad is
  // peeled and the loop unrolled by two with the key registers alternating,
  // so every entry to every use sees the same ops in flight (one key load +
  // the previous quad's stores) and the compiler keeps the wait partial.
  constexpr uint32_t kStep = uint32_t(B) * 4u;
  uint32_t q = lo + uint32_t(tid) * 4u;
  if (q < Pv) {
    auto keyAt = [&](uint32_t x) {  // clamped: unconditional prefetch
      if constexpr (sizeof(KeyT) == 2) {  // packed keys: one 8-B load per quad
        const uint2 h = *reinterpret_cast<const uint2*>(tkey + (x < Pv ? x : Pv - 4u));
        return make_uint4(key_of(uint16_t(h.x)), key_of(uint16_t(h.x >> 16)),
                          key_of(uint16_t(h.y)), key_of(uint16_t(h.y >> 16)));
      } else {
        return *reinterpret_cast<const uint4*>(tkey + (x < Pv ? x : Pv - 4u));
      }
    };
    uint4 ka = keyAt(q);
    uint4 kb = keyAt(q + kStep);
    quad(q, ka);
    q += kStep;
    while (q < Pv) {
      ka = keyAt(q + kStep);
      quad(q, kb);
      q += kStep;
      if (q >= Pv) break;
      kb = keyAt(q + kStep);
      quad(q, ka);
      q += kStep;
    }
  }
  for (uint32_t p = Pv + tid; p < hi; p += B) {  // tail / unaligned rows
    Rec<W> r;
    one(p, key_of(tkey[p]), r);
    if (oMeta) oMeta[p] = r.meta;
    if (oMetric) oMetric[p] = r.metric;
    if (oSel) oSel[p] = r.sel;
    if (oMask) {
#pragma unroll
      for (int w = 0; w < W; ++w) oMask[size_t(w) * Sp + p] = r.mask[w];
    }
    if constexpr (DIFF) {
      if (route_changed<W>(r, *diff, Sp, p, upd, del)) {
        atomicOr(diff->changed + p / 32u, 1u << (p % 32u));
      }
    }
  }
  if constexpr (DIFF) {
    if (upd) atomicAdd(diff->counts, upd);
    if (del) atomicAdd(diff->counts + 1, del);
  }
}

}  // namespace ogs
