// spf_route_wave.hip — one WAVEFRONT per (topology, source) unit, 32-bit
// distances, single-word next-hop sets: the C1/C2 hot path.
//
// Algorithm and outputs are those of spf_route.hip (reference mapping in its
// header). Measured on MI355X, a C2 launch is 4096 units all resident at
// once (16 waves/CU), and the relaxation rounds are bound by the per-round
// dependency chain (LDS gather -> ~10 dependent VALU ops -> ballot/branch)
// at 4 waves per SIMD. Measured and rejected (tools/ab_wave_opt.py,
// DESIGN.md §3): register-resident words gathered with ds_bpermute (no LDS
// traffic, no bank conflicts: same round time) and persistent waves running
// 2-4 units with the next unit's loads in flight during the rounds (half the
// waves per SIMD doubles the round latency). This variant cuts LDS
// instructions:
//  * per node ONE 64-bit LDS word {dist, next-hop bits}: one ds_read_b64
//    per edge instead of two ds_read_b32;
//  * branch-free relaxation: unusable edges read a dummy word, edges into
//    the source read a per-link-slot word, so a round is add/min/compare/or
//    only (VALU issue is the bound: 4 waves per SIMD, 4 cycles per op);
//  * nodes are relaxed in a host-chosen order (ogs_graph.slot_node): the
//    two BFS colour classes go to different 64-lane slots, so one round
//    advances two hops on bipartite topologies;
//  * edges (<= MAXD per node) and the node's own value stay in registers;
//  * one dependent global load for the unit's offsets (ogs_graph.topo_desc)
//    and one batch of staging loads for CSR + prefix table;
//  * single-advertiser prefixes take a straight-line route path; when every
//    prefix has exactly one advertisement at its own index (identity
//    segments) the route phase reads advertiser and flags from the staging
//    registers and the prefix tables never touch LDS.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "route_core.h"
#include "spf_core.h"
#include "engine.h"

namespace ogs {

constexpr uint32_t OGS_WAVE_OPT_BPERMUTE = 1;    // register-resident SPF words
constexpr uint32_t OGS_WAVE_OPT_REG_ROUTES = 2;  // identity-segment route path

// LDS image of one unit. Advertisement metrics are staged only when best
// route selection reads them; minNexthop is read from HBM on demand (only
// for prefixes flagged OGS_PFX_HAS_MIN_NH).
struct WaveLayout {
  uint32_t dn, dn32, row, edges, flags, advOff, advNode, advMetrics, pfxFlags,
      total;
  __host__ __device__ static WaveLayout make(uint32_t N, uint32_t E, uint32_t P,
                                             uint32_t A, bool brs) {
    WaveLayout L;
    uint32_t o = 0;
    const uint32_t P0 = N <= 64 ? 64 : N <= 128 ? 128 : 256;  // = 64 * NPL
    L.dn = o;  // P0 positions (later: N node words) + dummy + 8 source words + source self
    o += align16(uint64_t(P0 + 10) * 8);
    L.dn32 = o;  // narrow-form words, same positions (first: posOf scratch)
    o += align16(uint64_t(P0 + 10) * 4);  // + dummy, 8 source-slot words, source self
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
    o += brs ? align16(uint64_t(A) * 16) : 0u;
    L.pfxFlags = o;
    o += align16(P);
    L.total = o;
    return L;
  }
};

struct IdentitySlots {
  uint16_t v[256];
  constexpr IdentitySlots() : v() {
    for (int i = 0; i < 256; ++i) v[i] = uint16_t(i);
  }
};
__device__ IdentitySlots kIdentitySlots;

template <int K, typename T>
struct WStage {  // K elements per lane, all loads before any store
  T v[K];
  __device__ __forceinline__ void load(const T* __restrict__ src, uint32_t n,
                                       int lane) {
    if (n == 0) {  // keep v[] defined on every path (no stack copy)
#pragma unroll
      for (int k = 0; k < K; ++k) v[k] = T{};
      return;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t i = uint32_t(k * 64 + lane);
      v[k] = src[i < n ? i : n - 1];
    }
  }
  __device__ __forceinline__ void store(T* dst, uint32_t n, int lane) const {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t i = uint32_t(k * 64 + lane);
      if (i < n) dst[i] = v[k];
    }
  }
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Straight-line route for a prefix with exactly one advertisement (same
// result as route_one on a one-entry segment).
__device__ __forceinline__ void route_single(uint32_t n, int64_t minNh,
                                             uint32_t s, const uint8_t* nflags,
                                             const uint64_t* dn, uint32_t& meta,
                                             uint32_t& metric, uint32_t& mask) {
  meta = (n == s) ? OGS_ROUTE_LOCAL : 0u;
  metric = 0xFFFFFFFFu;
  mask = 0u;
  const uint64_t x = (n != OGS_NODE_NONE) ? dn[n] : ~0ull;
  const uint32_t d = static_cast<uint32_t>(x);
  if (n == OGS_NODE_NONE || d == 0xFFFFFFFFu) {
    meta |= OGS_REASON_UNREACHABLE << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  meta |= OGS_ROUTE_SELECTED;  // best index 0
  if (nflags[n] & (OGS_NODE_OVERLOADED | OGS_NODE_METRICINC)) {
    meta |= OGS_ROUTE_DRAINED;
  }
  if (n == s) {
    meta |= OGS_REASON_SELF << OGS_ROUTE_REASON_SHIFT;
    return;
  }
  mask = static_cast<uint32_t>(x >> 32);
  metric = d;
  const uint32_t cnt = __popc(mask);
  if (cnt == 0) {
    meta |= OGS_REASON_NO_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
  } else if (minNh != INT64_MIN && static_cast<uint64_t>(minNh) > cnt) {
    meta |= OGS_REASON_MIN_NEXTHOP << OGS_ROUTE_REASON_SHIFT;
  } else {
    meta |= OGS_ROUTE_VALID;
  }
}

// ---- pieces shared by the one-unit and the pair kernels ---------------------

// Pull rounds of one unit to the fixpoint in the unit's LDS image; the
// lane's node words come back in dcur / ncur (unreachable: kInf, {}).
// Narrow form (every path < 2^23, decided per unit): one 32-bit word per
// node, dist << 8 | next-hop bits (source degree <= 8). Adding w << 8 carries
// the next-hop bits along, all candidates tied with the minimum share its
// distance bits. Wide form (paths < 2^31 - 1, host-guaranteed): 64-bit
// {dist, nh} words, tie test by equality.
template <int NPL, int MAXD>
__device__ __forceinline__ void wave_spf(char* base, const WaveLayout& L, bool narrow,
                                         const uint32_t (&vk)[NPL],
                                         const uint32_t (&ea)[NPL][MAXD],
                                         const uint32_t (&ew)[NPL][MAXD], uint32_t s,
                                         int lane, uint32_t (&dcur)[NPL],
                                         uint32_t (&ncur)[NPL], uint32_t& rounds) {
  constexpr uint32_t P0 = NPL * 64;
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  (void)rounds;
  if (narrow) {
    // The next-hop byte is stored COMPLEMENTED (dist << 8 | ~nh & 0xFF):
    // with hi = min | 0xFF, min(cand, hi) is the candidate itself when it
    // ties the minimum distance and hi otherwise, so the AND over the edges
    // is {min dist, ~(OR of the tied next-hop sets)} -- min + and per edge,
    // no compare / select pairs. Unreachable = 0x800000FF (dist field 2^23,
    // empty set); unusable edges read the dummy word with weight 0.
    // Every lane is stable at the fixpoint -- empty positions read only the
    // dummy, the source's lane only word P0 + 9 (= its own {0, {}}) -- so
    // convergence is ONE test per round: did any lane's word change. (Per
    // round, measured alone with the diagnostic stamps build: 838 cycles
    // with the per-slot ballots against the active mask and the early exit
    // after a separated slot, 550 with no test at all.)
    constexpr uint32_t kUnr = 0x800000FFu;
    uint32_t* d32 = reinterpret_cast<uint32_t*>(base + L.dn32);
    uint32_t ws[NPL][MAXD], ra[NPL][MAXD], cur[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const bool src = vk[k] == s;
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        ra[k][j] = src ? P0 + 9 : ea[k][j];
        ws[k][j] = src ? 0u : ew[k][j] << 8;
      }
      cur[k] = src ? 0xFFu : kUnr;
      d32[k * 64 + lane] = cur[k];
    }
    if (lane == 0) {
      d32[P0] = kUnr;
      d32[P0 + 9] = 0xFFu;
    }
    if (lane < 8) d32[P0 + 1 + lane] = ~(1u << lane) & 0xFFu;
    wave_sync();
    for (;;) {
      uint32_t chg = 0u;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        uint32_t cand[MAXD];
        uint32_t best = kUnr;
#pragma unroll
        for (int j = 0; j < MAXD; ++j) {
          cand[j] = d32[ra[k][j]] + ws[k][j];
          best = cand[j] < best ? cand[j] : best;
        }
        const uint32_t hiB = best | 0xFFu;
        uint32_t word = hiB;
#pragma unroll
        for (int j = 0; j < MAXD; ++j) word &= cand[j] < hiB ? cand[j] : hiB;
        chg |= word ^ cur[k];
        cur[k] = word;
        d32[k * 64 + lane] = word;
      }
#ifdef OGS_STAMPS
      ++rounds;
#endif
      if (__builtin_amdgcn_ballot_w64(chg != 0u) == 0ull) break;
      wave_sync();
    }
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const bool unr = cur[k] >= 0x80000000u;
      dcur[k] = unr ? kInf : cur[k] >> 8;
      ncur[k] = unr ? 0u : ~cur[k] & 0xFFu;
    }
  } else {
    // 64-bit {dist, nh} words (paths < 2^31 - 1); the same single
    // convergence test per round as the narrow form (the source's lane reads
    // only word P0 + 9 = {0, {}}, empty positions only the dummy)
    constexpr uint32_t kUnr = 0x80000000u;
    uint64_t* dn = reinterpret_cast<uint64_t*>(base + L.dn);
    uint32_t we[NPL][MAXD], ra[NPL][MAXD];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const bool src = vk[k] == s;
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        ra[k][j] = src ? P0 + 9 : ea[k][j];
        // unusable: dummy {kUnr} + 2^31-1 = 2^32-1, never wins, never wraps
        we[k][j] = src ? 0u : ea[k][j] == P0 ? kUnr - 1 : ew[k][j];
      }
      dcur[k] = src ? 0u : kUnr;
      ncur[k] = 0u;
      dn[k * 64 + lane] = dcur[k];
    }
    if (lane == 0) {
      dn[P0] = uint64_t(kUnr);
      dn[P0 + 9] = 0ull;
    }
    if (lane < 8) dn[P0 + 1 + lane] = uint64_t(1u << lane) << 32;
    wave_sync();
    for (;;) {
      uint32_t chg = 0u;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        uint64_t x[MAXD];
#pragma unroll
        for (int j = 0; j < MAXD; ++j) x[j] = dn[ra[k][j]];
        uint32_t best = kUnr;
        uint32_t cand[MAXD];
#pragma unroll
        for (int j = 0; j < MAXD; ++j) {
          cand[j] = static_cast<uint32_t>(x[j]) + we[k][j];
          best = cand[j] < best ? cand[j] : best;
        }
        uint32_t m = 0u;
#pragma unroll
        for (int j = 0; j < MAXD; ++j) {
          m |= (cand[j] == best) ? static_cast<uint32_t>(x[j] >> 32) : 0u;
        }
        chg |= (best ^ dcur[k]) | (m ^ ncur[k]);
        dcur[k] = best;
        ncur[k] = m;
        dn[k * 64 + lane] = uint64_t(best) | (uint64_t(m) << 32);
      }
#ifdef OGS_STAMPS
      ++rounds;
#endif
      if (__builtin_amdgcn_ballot_w64(chg != 0u) == 0ull) break;
      wave_sync();
    }
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      if (dcur[k] >= kUnr) {
        dcur[k] = kInf;
        ncur[k] = 0u;
      }
    }
  }
}

// Per-edge constants of the lane's positions from the per-position edge
// image (ogs_graph.slot_edges): word position (P0: dummy, P0 + 1 + r: the
// source through its link slot r) and weight (0 if unusable); wmax over the
// wave.
template <int NPL, int MAXD>
__device__ __forceinline__ uint32_t wave_edges_from_image(const uint32_t (&ie)[NPL][MAXD],
                                                          uint32_t posS, bool hop,
                                                          uint32_t (&ea)[NPL][MAXD],
                                                          uint32_t (&ew)[NPL][MAXD]) {
  constexpr uint32_t P0 = NPL * 64;
  uint32_t wmax = 0;
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
#pragma unroll
    for (int j = 0; j < MAXD; ++j) {
      const uint32_t x = ie[k][j];
      const uint32_t nbr = x & 0x1FFu;
      const bool ok = !(x & OGS_SLOT_EDGE_DOWN) &&
          !((x & OGS_SLOT_EDGE_DST_OVERLOADED) && nbr != posS);
      const uint32_t w = hop ? 1u : x >> 16;
      ea[k][j] = !ok ? P0
                     : (nbr == posS ? P0 + 1 + ((x >> OGS_SLOT_EDGE_RSLOT_SHIFT) & 7u) : nbr);
      ew[k][j] = ok ? w : 0u;
      wmax = ew[k][j] > wmax ? ew[k][j] : wmax;
    }
  }
  return wmax;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t t = __shfl_xor(x, o);
    x = t > x ? t : x;
  }
  return __builtin_amdgcn_readfirstlane(x);
}

// Route-phase tables of one unit: node flags into LDS, prefix tables into
// LDS unless they stay in the staging registers (identity segments: every
// prefix has exactly one advertisement, at its own index -- the route phase
// then reads advertiser and flags from the registers). Returns "identity".
template <int NPL, int KP>
__device__ __forceinline__ bool wave_stage_tables(
    const ogs_prefix_table& pt, int hasPrefixes, bool pfxFits, bool brs, uint32_t wopt,
    uint32_t N, uint32_t P, uint32_t A, uint32_t p0, uint32_t a0,
    const WStage<KP, uint32_t>& sOff, const WStage<KP, uint32_t>& sNode,
    const WStage<KP, uint8_t>& sPf, const WStage<KP, int4>& sMet,
    const WStage<NPL, uint8_t>& sFlag, char* base, const WaveLayout& L, int lane) {
  uint8_t* lflags = reinterpret_cast<uint8_t*>(base + L.flags);
  uint32_t* lAdvOff = reinterpret_cast<uint32_t*>(base + L.advOff);
  uint32_t* lAdvNode = reinterpret_cast<uint32_t*>(base + L.advNode);
  int4* lAdvMetrics = reinterpret_cast<int4*>(base + L.advMetrics);
  uint8_t* lPfxFlags = reinterpret_cast<uint8_t*>(base + L.pfxFlags);
  bool ident = false;
  if (hasPrefixes && pfxFits && A == P && (wopt & OGS_WAVE_OPT_REG_ROUTES)) {
    bool off = false;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const uint32_t i = uint32_t(k * 64 + lane);
      off |= i <= P && sOff.v[k] - a0 != i;
    }
    ident = __builtin_amdgcn_ballot_w64(off) == 0ull;
  }
  sFlag.store(lflags, N, lane);
  if (ident) {
    // tables stay in registers
  } else if (hasPrefixes && pfxFits) {
    sOff.store(lAdvOff, P + 1, lane);
    sNode.store(lAdvNode, A, lane);
    sMet.store(lAdvMetrics, brs ? A : 0u, lane);
    sPf.store(lPfxFlags, P, lane);
  } else if (hasPrefixes) {  // rare: long prefix tables, plain loop
    for (uint32_t i = lane; i <= P; i += 64) lAdvOff[i] = pt.adv_off[p0 + i];
    for (uint32_t i = lane; i < P; i += 64) lPfxFlags[i] = pt.pfx_flags[p0 + i];
    for (uint32_t i = lane; i < A; i += 64) {
      lAdvNode[i] = pt.adv_node[a0 + i];
      if (brs) lAdvMetrics[i] = reinterpret_cast<const int4*>(pt.adv_metrics)[a0 + i];
    }
  }
  return ident;
}

// SPF outputs and the fused RouteDb of one unit (LDS: final {dist, nh} words
// by node id, node flags, and the prefix tables unless `ident`).
template <int NPL, int KP>
__device__ __forceinline__ void wave_outputs(
    const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes, uint32_t flags,
    const ogs_spf_out& out, size_t uidx, uint32_t s, uint32_t N, uint32_t P, uint32_t a0,
    bool ident, const uint32_t (&vk)[NPL], const uint32_t (&dcur)[NPL],
    const uint32_t (&ncur)[NPL], const WStage<KP, uint32_t>& sNode,
    const WStage<KP, uint8_t>& sPf, char* base, const WaveLayout& L, int lane) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  const uint64_t* dn = reinterpret_cast<const uint64_t*>(base + L.dn);
  const uint8_t* lflags = reinterpret_cast<const uint8_t*>(base + L.flags);
  const uint32_t* lAdvOff = reinterpret_cast<const uint32_t*>(base + L.advOff);
  const uint32_t* lAdvNode = reinterpret_cast<const uint32_t*>(base + L.advNode);
  const int4* lAdvMetrics = reinterpret_cast<const int4*>(base + L.advMetrics);
  const uint8_t* lPfxFlags = reinterpret_cast<const uint8_t*>(base + L.pfxFlags);
  // ---- SPF outputs ----------------------------------------------------------
  const uint32_t Sn = g.max_nodes;
  const bool nt = (flags & kFlagNtStores) != 0;
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const uint32_t v = vk[k];
    if (v >= N) continue;
    // outputs are not re-read by the kernel: non-temporal or ordinary
    // stores by the launch's kFlagNtStores bit ("route_store_nt")
    if (out.dist) store_out(static_cast<uint32_t*>(out.dist) + uidx * Sn + v, dcur[k], nt);
    if (out.nh) store_out(out.nh + uidx * Sn + v, ncur[k], nt);
  }
  if (!hasPrefixes) return;

  // ---- fused RouteDb --------------------------------------------------------
  const RouteCfg cfg{(flags & OGS_F_ENABLE_V4) != 0,
                     (flags & OGS_F_V4_OVER_V6) != 0,
                     (flags & OGS_F_BEST_ROUTE_SELECTION) != 0};
  ogs_prefix_table lp{};
  lp.max_prefixes = pt.max_prefixes;
  lp.adv_off = lAdvOff;
  lp.adv_node = lAdvNode;
  lp.adv_metrics = reinterpret_cast<const int32_t*>(lAdvMetrics);
  lp.adv_min_nh = pt.adv_min_nh;  // HBM, absolute advertisement index
  lp.pfx_flags = lPfxFlags;
  const uint32_t Sp = pt.max_prefixes;
  if (ident) {
    // all of the lane's prefixes first (loads), then the stores
    uint32_t meta[KP], metric[KP], mask[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const uint32_t p = uint32_t(k * 64 + lane);
      const uint8_t pf = sPf.v[k];
      if ((pf & OGS_PFX_V4) && !cfg.enableV4 && !cfg.v4OverV6) {
        meta[k] = OGS_REASON_V4_DISABLED << OGS_ROUTE_REASON_SHIFT;  // route_one's gate
        metric[k] = kInf;
        mask[k] = 0u;
      } else {
        const int64_t minNh = (p < P && (pf & OGS_PFX_HAS_MIN_NH)) ? pt.adv_min_nh[a0 + p]
                                                                  : INT64_MIN;
        route_single(p < P ? sNode.v[k] : OGS_NODE_NONE, minNh, s, lflags, dn, meta[k],
                     metric[k], mask[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const uint32_t p = uint32_t(k * 64 + lane);
      if (p >= P) continue;
      const size_t o = uidx * Sp + p;
      if (out.meta) store_out(out.meta + o, meta[k], nt);
      if (out.metric) store_out(static_cast<uint32_t*>(out.metric) + o, metric[k], nt);
      if (out.sel) store_out(out.sel + o, (meta[k] & OGS_ROUTE_SELECTED) ? 1u : 0u, nt);
      if (out.mask) store_out(out.mask + o, mask[k], nt);
    }
  }
  for (uint32_t p = ident ? P : lane; p < P; p += 64) {
    uint32_t meta, metric, mask, selBits;
    const uint32_t b0 = lAdvOff[p] - a0, b1 = lAdvOff[p + 1] - a0;
    const uint8_t pf = lPfxFlags[p];
    const bool gated = (pf & OGS_PFX_V4) && !cfg.enableV4 && !cfg.v4OverV6;
    if (b1 - b0 == 1 && !gated) {
      const int64_t minNh = (pf & OGS_PFX_HAS_MIN_NH) ? pt.adv_min_nh[a0 + b0]
                                                      : INT64_MIN;
      route_single(lAdvNode[b0], minNh, s, lflags, dn, meta, metric, mask);
      selBits = (meta & OGS_ROUTE_SELECTED) ? 1u : 0u;
    } else {
      uint32_t mk[1];
      // route_one indexes the prefix table by prefix; rebase the segment
      lp.adv_node = lAdvNode - a0;
      lp.adv_metrics = reinterpret_cast<const int32_t*>(lAdvMetrics - a0);
      route_one<uint32_t, 1>(lp, p, s, lflags, PackedView{dn}, cfg, meta,
                             metric, mk, selBits);
      mask = mk[0];
    }
    const size_t o = uidx * Sp + p;
    if (out.meta) store_out(out.meta + o, meta, nt);
    if (out.metric) store_out(static_cast<uint32_t*>(out.metric) + o, metric, nt);
    if (out.sel) store_out(out.sel + o, selBits, nt);
    if (out.mask) store_out(out.mask + o, mask, nt);
  }
}

template <int NPL, int MAXD, int UPB>
__global__ __launch_bounds__(64 * UPB) void spf_route_wave_kernel(
    ogs_graph g, ogs_prefix_table pt, int hasPrefixes,
    const ogs_unit* __restrict__ units, int nUnits, uint32_t flags,
    ogs_spf_out out, uint32_t ldsPerUnit, uint32_t maxA, uint32_t wopt) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  // wave-uniform by construction; readfirstlane lets the compiler prove it,
  // so the unit record and its descriptor come through scalar loads
  const int uib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int uidx = blockIdx.x * UPB + uib;
  if (uidx >= nUnits) return;
  uint32_t rounds = 0;
#ifdef OGS_STAMPS  // diagnostic build only: phase clocks into out.sel
  const uint64_t tStart = __builtin_amdgcn_s_memtime();
  const uint64_t rtStart = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  uint64_t tDesc = 0, tStaged = 0, tSpf = 0;
#endif

  // ---- unit offsets -------------------------------------------------------
  const ogs_unit unit = units[uidx];
  const uint32_t s = unit.src;
  // relaxation order (slot_order.h): position k*64+lane -> node id; loaded
  // with the staging batch below
  const bool perm = g.slot_node && g.slot_stride == NPL * 64;
  uint32_t vk[NPL];
  uint32_t nb, N, e0, E, p0 = 0, P = 0, a0 = 0, A = 0;
  if (g.topo_desc) {
    // batch builds put unit i on topology i: the descriptor of topology
    // uidx is loaded together with the unit record (one scalar latency
    // instead of two dependent ones) and reloaded only when it is not
    const uint4* td = reinterpret_cast<const uint4*>(g.topo_desc);
    const uint32_t guess = uint32_t(uidx) < uint32_t(g.num_topos) ? uint32_t(uidx) : 0u;
    uint4 x = td[2 * guess];
    uint4 y = td[2 * guess + 1];
    // opaque to the optimiser (otherwise it folds the guess into a load at
    // unit.topo, i.e. back into two dependent latencies); readfirstlane
    // returns the values to scalar registers
    asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w), "+v"(y.x),
                 "+v"(y.y), "+v"(y.z), "+v"(y.w));
    x.x = __builtin_amdgcn_readfirstlane(x.x);
    x.y = __builtin_amdgcn_readfirstlane(x.y);
    x.z = __builtin_amdgcn_readfirstlane(x.z);
    x.w = __builtin_amdgcn_readfirstlane(x.w);
    y.x = __builtin_amdgcn_readfirstlane(y.x);
    y.y = __builtin_amdgcn_readfirstlane(y.y);
    y.z = __builtin_amdgcn_readfirstlane(y.z);
    y.w = __builtin_amdgcn_readfirstlane(y.w);
    if (unit.topo != guess) {
      x = td[2 * unit.topo];
      y = td[2 * unit.topo + 1];
    }
    nb = x.x;
    N = x.y;
    e0 = x.z;
    E = x.w;
    if (hasPrefixes) {
      p0 = y.x;
      P = y.y;
      a0 = y.z;
      A = y.w;
    }
  } else {
    nb = g.node_base[unit.topo];
    N = g.node_base[unit.topo + 1] - nb;
    e0 = g.row_ptr[nb];
    E = g.row_ptr[nb + N] - e0;
    if (hasPrefixes) {
      p0 = pt.pfx_base[unit.topo];
      P = pt.pfx_base[unit.topo + 1] - p0;
      a0 = pt.adv_off[p0];
      A = pt.adv_off[p0 + P] - a0;
    }
  }
#ifdef OGS_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tDesc = __builtin_amdgcn_s_memtime();
#endif
  const bool brs = flags & OGS_F_BEST_ROUTE_SELECTION;
  const WaveLayout L = WaveLayout::make(g.max_nodes, g.max_edges,
                                        hasPrefixes ? pt.max_prefixes : 0,
                                        hasPrefixes ? maxA : 0, brs);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* base = smem + uib * ldsPerUnit;
  uint64_t* dn = reinterpret_cast<uint64_t*>(base + L.dn);
  uint32_t* lrow = reinterpret_cast<uint32_t*>(base + L.row);
  uint64_t* ledg = reinterpret_cast<uint64_t*>(base + L.edges);

  // ---- staging: one batch of loads, then LDS writes -----------------------
  // With the per-position edge image (ogs_graph.slot_edges) each lane loads
  // its nodes' edges coalesced straight into registers and the CSR is not
  // staged at all.
  constexpr uint32_t P0 = NPL * 64;
  const bool img = perm && g.slot_edges && g.slot_degree == MAXD;
  uint32_t ie[NPL][MAXD];
  constexpr int KP = NPL + 1;  // prefixes per lane per pass (P <= 64*KP)
  // Node flags and the prefix tables are needed only by the route phase:
  // their loads are issued with the SPF inputs but waited on (and stored to
  // LDS) after the SPF rounds, so their latency hides behind the rounds.
  WStage<KP, uint32_t> sOff, sNode;
  WStage<KP, uint8_t> sPf;
  WStage<KP, int4> sMet;
  WStage<NPL, uint8_t> sFlag;
  const bool pfxFits = (P + 1 <= 64u * KP) && (A <= 64u * KP);
  {
    WStage<NPL + 1, uint32_t> sRow;
    WStage<NPL * MAXD, uint64_t> sEdge;  // E <= N * MAXD <= 64 * NPL * MAXD
    sRow.load(g.row_ptr + nb, img ? 0u : N + 1, lane);
    sEdge.load(g.edges + e0, img ? 0u : E, lane);
    if (img) {
      const uint32_t* ib = g.slot_edges + size_t(unit.topo) * (MAXD * P0);
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
#pragma unroll
        for (int k = 0; k < NPL; ++k) ie[k][j] = ib[j * P0 + k * 64 + lane];
      }
    } else {
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
#pragma unroll
        for (int k = 0; k < NPL; ++k) ie[k][j] = 0u;
      }
    }
    sFlag.load(g.node_flags + nb, N, lane);
    // unconditional (identity table without slot_node): no branch, so
    // nothing waits on these loads before the whole batch is issued
    const uint16_t* so = perm ? g.slot_node + size_t(unit.topo) * (NPL * 64)
                              : kIdentitySlots.v;
    uint32_t rawSlot[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) rawSlot[k] = so[k * 64 + lane];
    if (hasPrefixes && pfxFits) {
      sOff.load(pt.adv_off + p0, P + 1, lane);
      sNode.load(pt.adv_node + a0, A, lane);
      sMet.load(reinterpret_cast<const int4*>(pt.adv_metrics) + a0, brs ? A : 0u, lane);
      sPf.load(pt.pfx_flags + p0, P, lane);
    }
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      vk[k] = rawSlot[k] == 0xFFFFu ? 0xFFFFFFFFu : rawSlot[k];
    }
    sRow.store(lrow, img ? 0u : N + 1, lane);
    sEdge.store(ledg, img ? 0u : E, lane);
  }
  wave_sync();
#ifdef OGS_STAMPS
  tStaged = __builtin_amdgcn_s_memtime();
#endif

  // ---- registers: per-edge constants of the lane's node slots -------------
  // During SPF the LDS words are indexed by POSITION (slot*64 + lane), not
  // by node id: under the 2-colour order the neighbours of consecutive lanes
  // sit at consecutive positions of the other slot, so the gathers are
  // (nearly) bank-conflict free. Extra words after the P0 = 64*NPL
  // positions remove every branch and special case from the relaxation:
  //  * word P0 (dummy) = "unreachable": target of unusable edges;
  //  * word P0+1+r = {dist 0, next hops {r}}: the source seen through its
  //    link slot r. An edge v -> src reads the word of its own slot instead
  //    of the source's, so the tight contribution of every edge is just the
  //    word's next-hop part (LinkState.cpp:808-811: NH(v) gets the source's
  //    link to v).
  const bool hop = flags & OGS_F_HOP_METRIC;
  uint32_t ea[NPL][MAXD], ew[NPL][MAXD];  // word position, weight (0 if unusable)
  uint32_t wmax = 0;
  uint32_t posS = P0;  // the source's position (uniform; P0: not placed)
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(vk[k] == s);
    if (m) posS = uint32_t(k * 64) + uint32_t(__builtin_ctzll(m));
  }
  if (img) {
    wmax = wave_edges_from_image<NPL, MAXD>(ie, posS, hop, ea, ew);
  } else {
    {
      uint32_t* posOf = reinterpret_cast<uint32_t*>(base + L.dn32);  // scratch
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        if (vk[k] < N) posOf[vk[k]] = uint32_t(k * 64 + lane);
      }
    }
    wave_sync();
    const uint32_t* posOf = reinterpret_cast<const uint32_t*>(base + L.dn32);
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const uint32_t v = vk[k];
      const bool own = v < N;
      const uint32_t e = own ? lrow[v] - e0 : 0u;
      const uint32_t deg = own ? lrow[v + 1] - lrow[v] : 0u;
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        const uint64_t x = (uint32_t(j) < deg) ? ledg[e + j] : uint64_t(OGS_EDGE_DOWN);
        const uint32_t lo = static_cast<uint32_t>(x);
        const uint32_t u = edge_dst(lo);
        const bool ok = !(lo & OGS_EDGE_DOWN) &&
            !((lo & OGS_EDGE_DST_OVERLOADED) && u != s);
        const uint32_t w = hop ? 1u : static_cast<uint32_t>(x >> 32);
        ea[k][j] = !ok ? P0 : (u == s ? P0 + 1 + edge_rslot(lo) : posOf[u]);
        ew[k][j] = ok ? w : 0u;
        wmax = ew[k][j] > wmax ? ew[k][j] : wmax;
      }
    }
  }
  wmax = wave_max(wmax);
  uint64_t actMask[NPL];  // lanes holding a non-source node (uniform)
  uint32_t dcur[NPL], ncur[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    actMask[k] = __builtin_amdgcn_ballot_w64(vk[k] < N && vk[k] != s);
  }
  // Two-slot units whose slots are separated (every edge between two nodes
  // joins slot 0 and slot 1, true for the 2-colour order on bipartite
  // graphs) converge at the first slot evaluation after the first one that
  // changes nothing: slot X unchanged means slot Y's inputs are those of its
  // previous evaluation. Used by the register-resident (ds_bpermute) form
  // only; the LDS forms test once per round (cheaper than a test per slot).
  bool sep = false;
  if (NPL == 2 && (wopt & OGS_WAVE_OPT_BPERMUTE)) {
    bool bad = false;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        bad |= ((actMask[k] >> lane) & 1ull) && ea[k][j] < P0 &&
            (ea[k][j] >> 6) == uint32_t(k);
      }
    }
    sep = __builtin_amdgcn_ballot_w64(bad) == 0ull;
  }
  // register-resident relaxation (ds_bpermute gathers, no LDS words):
  // one slot (Jacobi), or two separated slots whose source edges cross
  // slots too (each slot reads only the other slot's register)
  bool regSpf = (wopt & OGS_WAVE_OPT_BPERMUTE) && posS < P0 && (NPL == 1 || (NPL == 2 && sep));
  if (NPL == 2 && regSpf) {
    bool bad = false;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        bad |= ((actMask[k] >> lane) & 1ull) && ea[k][j] > P0 && (posS >> 6) == uint32_t(k);
      }
    }
    regSpf = __builtin_amdgcn_ballot_w64(bad) == 0ull;
  }
  wave_sync();  // posOf scratch is overwritten below

  // ---- SPF: pull rounds to the fixpoint -------------------------------------
  const bool narrow = uint64_t(wmax) * (N > 0 ? N - 1 : 0) < 0x7FFFFFull;
  if (narrow && regSpf) {
    // Words as in the narrow form (wave_spf), held in registers: slot k's
    // lane gathers its neighbours' words from the other slot's register with
    // ds_bpermute (no LDS traffic, no bank conflicts). Per edge a lane
    // address and an addend: unusable edges add kUnr (saturating, so the
    // candidate is >= kUnr and never below a reachable word); edges into
    // the source read the source lane (word 0, kept there by the active
    // mask) and add w << 8 | the source's link-slot bit.
    constexpr uint32_t kUnr = 0x80000000u;
    uint32_t ba[NPL][MAXD], wb[NPL][MAXD], cur[NPL];
    bool act[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      act[k] = (actMask[k] >> lane) & 1ull;
      cur[k] = vk[k] == s ? 0u : kUnr;
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        const uint32_t e = ea[k][j];
        ba[k][j] = (e < P0 ? (e & 63u) : e == P0 ? uint32_t(lane) : (posS & 63u)) << 2;
        wb[k][j] = e == P0 ? kUnr
                           : (ew[k][j] << 8) | (e > P0 ? 1u << (e - P0 - 1) : 0u);
      }
    }
    auto relax = [&](int k, uint32_t other) {
      uint32_t cand[MAXD];
      uint32_t best = kUnr;
#pragma unroll
      for (int j = 0; j < MAXD; ++j) {
        const uint32_t x = uint32_t(__builtin_amdgcn_ds_bpermute(int(ba[k][j]), int(other)));
        cand[j] = __builtin_elementwise_add_sat(x, wb[k][j]);
        best = cand[j] < best ? cand[j] : best;
      }
      const uint32_t hiB = best | 0xFFu;
      uint32_t word = best & kUnr;
#pragma unroll
      for (int j = 0; j < MAXD; ++j) word |= cand[j] <= hiB ? cand[j] : 0u;
      return act[k] ? word : cur[k];
    };
    if (NPL == 1) {
      for (;;) {
        const uint32_t w = relax(0, cur[0]);
        const bool ch = __builtin_amdgcn_ballot_w64(w != cur[0]) != 0ull;
        cur[0] = w;
#ifdef OGS_STAMPS
        ++rounds;
#endif
        if (!ch) break;
      }
    } else {
      // Gauss-Seidel over the two slots; after the first sub-step, one
      // that changes nothing means the other slot's inputs are unchanged
      for (int step = 0;; ++step) {
        const uint32_t w0 = relax(0, cur[NPL - 1]);
        const bool ch0 = __builtin_amdgcn_ballot_w64(w0 != cur[0]) != 0ull;
        cur[0] = w0;
#ifdef OGS_STAMPS
        ++rounds;
#endif
        if (step > 0 && !ch0) break;
        const uint32_t w1 = relax(NPL - 1, cur[0]);
        const bool ch1 = __builtin_amdgcn_ballot_w64(w1 != cur[NPL - 1]) != 0ull;
        cur[NPL - 1] = w1;
        if (!ch1) break;
      }
    }
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      dcur[k] = cur[k] >= kUnr ? kInf : cur[k] >> 8;
      ncur[k] = cur[k] >= kUnr ? 0u : cur[k] & 0xFFu;
    }
  } else {
    wave_spf<NPL, MAXD>(base, L, narrow, vk, ea, ew, s, lane, dcur, ncur, rounds);
  }
  // final {dist, nh} words, now by NODE ID, for the route phase (ABI
  // "unreachable" = all ones); the source lane's registers hold its unused
  // evaluation. All position-indexed reads precede these writes in program
  // order.
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const uint32_t v = vk[k];
    if (v == s) {
      dcur[k] = 0u;
      ncur[k] = 0u;
    }
    if (v < N) dn[v] = uint64_t(dcur[k]) | (uint64_t(ncur[k]) << 32);
  }
  const bool ident = wave_stage_tables<NPL, KP>(pt, hasPrefixes, pfxFits, brs, wopt, N, P, A,
                                                p0, a0, sOff, sNode, sPf, sMet, sFlag, base, L,
                                                lane);
  wave_sync();
#ifdef OGS_STAMPS
  tSpf = __builtin_amdgcn_s_memtime();
#endif
  wave_outputs<NPL, KP>(g, pt, hasPrefixes, flags, out, size_t(uidx), s, N, P, a0, ident, vk,
                        dcur, ncur, sNode, sPf, base, L, lane);
#ifdef OGS_STAMPS
  wave_sync();
  if (lane == 0 && out.sel) {
    const uint64_t tEnd = __builtin_amdgcn_s_memtime();
    uint32_t* d = out.sel + size_t(uidx) * pt.max_prefixes;
    d[0] = uint32_t(tStaged - tStart);
    d[1] = uint32_t(tSpf - tStaged);
    d[2] = uint32_t(tEnd - tSpf);
    d[3] = rounds;
    d[4] = uint32_t(tDesc - tStart);
    d[5] = uint32_t(rtStart);
    d[6] = uint32_t(__builtin_amdgcn_s_memrealtime());
  }
#endif
}

// ---- two units per wavefront: 16-bit packed words ---------------------------
// "wave_wg_lds" option: minimum LDS bytes per workgroup (occupancy probe for
// A/B measurements; 0 = just what the units need)
// EngineOptions::waveWgLds (engine.h), default 0
// "wave_upb" option: units (wavefronts) per workgroup, 4, 8 or 16
// EngineOptions::waveUpb (engine.h), default 4
// "wave_opt" option: OGS_WAVE_OPT_* bits (A/B of the register paths); the
// ds_bpermute SPF measured no faster than the LDS words (latency-bound
// rounds), so only the register route path is on by default. (Two units per
// wavefront with 16-bit packed words measured slower in round 3 -- C2 11.1
// vs 10.0 us per launch, profiles/r03_ab_wave_pair.log: every wave is
// resident from the start, so a launch lasts one wave's dependent chain --
// and was removed in round 4.)
// EngineOptions::waveOpt (engine.h), default OGS_WAVE_OPT_REG_ROUTES

template <int NPL, int MAXD, int UPB>
hipError_t launch_wave_upb(const ogs_graph& g, const ogs_prefix_table& pt,
                           int hasPrefixes, const ogs_unit* units, int nUnits,
                           uint32_t flags, const ogs_spf_out& out, uint32_t lds,
                           uint32_t maxA, hipStream_t stream) {
  const int grid = (nUnits + UPB - 1) / UPB;
  size_t bytes = size_t(lds) * UPB;
  if (bytes < size_t(opts().waveWgLds)) bytes = size_t(opts().waveWgLds);
  auto k = spf_route_wave_kernel<NPL, MAXD, UPB>;
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(k),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
    if (e != hipSuccess) return e;
  }
  if (opts().routeStoreNt & 2) flags |= kFlagNtStores;
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * UPB), bytes, stream, g, pt,
                     hasPrefixes, units, nUnits, flags, out, lds, maxA, uint32_t(opts().waveOpt));
  return hipGetLastError();
}

template <int NPL, int MAXD>
hipError_t launch_wave(const ogs_graph& g, const ogs_prefix_table& pt,
                       int hasPrefixes, const ogs_unit* units, int nUnits,
                       uint32_t flags, const ogs_spf_out& out, uint32_t lds,
                       uint32_t maxA, hipStream_t stream) {
  if (opts().waveUpb == 16 && uint64_t(lds) * 16 <= 160 * 1024) {
    return launch_wave_upb<NPL, MAXD, 16>(g, pt, hasPrefixes, units, nUnits, flags,
                                          out, lds, maxA, stream);
  }
  if (opts().waveUpb == 8 && uint64_t(lds) * 8 <= 160 * 1024) {
    return launch_wave_upb<NPL, MAXD, 8>(g, pt, hasPrefixes, units, nUnits, flags,
                                         out, lds, maxA, stream);
  }
  return launch_wave_upb<NPL, MAXD, 4>(g, pt, hasPrefixes, units, nUnits, flags,
                                       out, lds, maxA, stream);
}

bool try_wave(const ogs_graph& g, const ogs_prefix_table& pt, int hasPrefixes,
              const ogs_unit* units, int nUnits, uint32_t flags,
              const ogs_spf_out& out, uint32_t maxA, hipStream_t stream,
              hipError_t* err) {
  if (flags & OGS_F_WIDE_METRIC) return false;
  if (g.max_nodes > 256 || g.max_degree > 8 || g.max_degree < 0) return false;
  const uint32_t P = hasPrefixes ? pt.max_prefixes : 0;
  const uint32_t A = hasPrefixes ? maxA : 0;
  const uint32_t lds = WaveLayout::make(g.max_nodes, g.max_edges, P, A,
                                        flags & OGS_F_BEST_ROUTE_SELECTION).total;
  if (uint64_t(lds) * 4 > 160 * 1024) return false;
  const int N = g.max_nodes;
  const bool d4 = g.max_degree <= 4;
#define OGS_WAVE(NPL_, MAXD_)                                             \
  *err = launch_wave<NPL_, MAXD_>(g, pt, hasPrefixes, units, nUnits, flags, \
                                  out, lds, A, stream);                   \
  return true;
  if (N <= 64) { if (d4) { OGS_WAVE(1, 4) } OGS_WAVE(1, 8) }
  if (N <= 128) { if (d4) { OGS_WAVE(2, 4) } OGS_WAVE(2, 8) }
  if (d4) { OGS_WAVE(4, 4) }
  OGS_WAVE(4, 8)
#undef OGS_WAVE
}

}  // namespace ogs
