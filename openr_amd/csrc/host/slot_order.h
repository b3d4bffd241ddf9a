// slot_order.h — relaxation order for the wave-per-unit SPF kernel
// (ogs_graph.slot_node / slot_stride).
//
// The wave kernel relaxes a topology's nodes in 64-lane "slots"; within a
// slot all lanes read their neighbours' values of the previous slot write
// (Jacobi), across slots it is Gauss-Seidel. Putting the two colour classes
// of a BFS 2-colouring into different slots means that, on a bipartite graph
// (grids, Clos fabrics), class-1 nodes already see the class-0 values of the
// same round, so one round advances the frontier by two hops instead of
// one. The order is a pure permutation and source-independent: results are
// identical for every order, only the round count changes.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

#include "openr_gpu.h"

namespace openr_amd {

// Stride (positions per topology) the wave kernel is instantiated for, or 0
// when topologies are too large for it.
inline int slotStrideFor(int maxNodes) {
  if (maxNodes <= 64) return 64;
  if (maxNodes <= 128) return 128;
  if (maxNodes <= 256) return 256;
  return 0;
}

// BFS parity colouring over the CSR (edges in both directions present); an
// odd cycle just leaves some same-colour neighbours, which is still exact.
inline std::vector<uint8_t> colorNodes(const uint32_t* rowPtr,
                                       const uint64_t* edges, uint32_t N) {
  std::vector<uint8_t> color(N, 0xFF);
  std::vector<uint32_t> q;
  q.reserve(N);
  for (uint32_t r = 0; r < N; ++r) {
    if (color[r] != 0xFF) continue;
    color[r] = 0;
    q.assign(1, r);
    for (size_t h = 0; h < q.size(); ++h) {
      const uint32_t v = q[h];
      for (uint32_t e = rowPtr[v]; e < rowPtr[v + 1]; ++e) {
        const uint32_t u = uint32_t(edges[e]) & OGS_EDGE_DST_MASK;
        if (u < N && color[u] == 0xFF) {
          color[u] = color[v] ^ 1u;
          q.push_back(u);
        }
      }
    }
  }
  return color;
}

// Writes `stride` positions: class 0 (by id), then class 1 starting on the
// next slot boundary when that still fits, else right after class 0;
// unused positions hold 0xFFFF.
inline void placeSlots(const std::vector<uint8_t>& color, int stride,
                       uint16_t* out) {
  const uint32_t N = uint32_t(color.size());
  std::fill(out, out + stride, uint16_t(0xFFFF));
  uint32_t c0 = 0;
  for (uint8_t c : color) c0 += c == 0;
  uint32_t o1 = (c0 + 63) / 64 * 64;
  if (o1 + (N - c0) > uint32_t(stride)) o1 = c0;
  uint32_t i0 = 0, i1 = o1;
  for (uint32_t v = 0; v < N; ++v) out[color[v] ? i1++ : i0++] = uint16_t(v);
}

// Degree of the per-position edge image (ogs_graph.slot_edges), or 0 when
// the batch does not qualify (degree > 8 or a metric > 65535).
inline int slotDegreeFor(int maxDegree, uint64_t maxMetric, int stride) {
  if (!stride || maxDegree > 8 || maxMetric > 0xFFFFu) return 0;
  return maxDegree <= 4 ? 4 : 8;
}

// Per-position edge image of one topology: out[j * stride + p] describes
// edge j of the node at position p (layout in include/openr_gpu.h).
// rowPtr[v] indexes `edges` directly (global or topology-local offsets).
inline void placeSlotEdges(const uint16_t* slots, int stride,
                           const uint32_t* rowPtr, const uint64_t* edges,
                           uint32_t N, int degree, uint32_t* out) {
  std::vector<uint16_t> pos(N, 0);
  for (int p = 0; p < stride; ++p) {
    if (slots[p] != 0xFFFF) pos[slots[p]] = uint16_t(p);
  }
  std::fill(out, out + size_t(degree) * stride, OGS_SLOT_EDGE_DOWN);
  for (int p = 0; p < stride; ++p) {
    const uint32_t v = slots[p];
    if (v == 0xFFFF) continue;
    for (uint32_t e = rowPtr[v], j = 0; e < rowPtr[v + 1]; ++e, ++j) {
      const uint32_t lo = uint32_t(edges[e]);
      const uint32_t w = uint32_t(edges[e] >> 32);
      const uint32_t u = lo & OGS_EDGE_DST_MASK;
      const uint32_t rslot = (lo >> OGS_EDGE_RSLOT_SHIFT) & OGS_EDGE_RSLOT_MASK;
      out[size_t(j) * stride + p] = uint32_t(pos[u]) |
          ((lo & OGS_EDGE_DOWN) ? OGS_SLOT_EDGE_DOWN : 0u) |
          ((lo & OGS_EDGE_DST_OVERLOADED) ? OGS_SLOT_EDGE_DST_OVERLOADED : 0u) |
          (rslot << OGS_SLOT_EDGE_RSLOT_SHIFT) | (w << 16);
    }
  }
}

}  // namespace openr_amd
