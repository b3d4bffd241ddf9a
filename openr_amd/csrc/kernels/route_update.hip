// route_update.hip — changed-route extraction for incremental route updates
// (SURVEY.md §8(f) f1).
//
// Reference: Decision::rebuildRoutes' incremental branch (Decision.cpp:
// 929-951) computes the new RouteDb and hands Fib the DecisionRouteUpdate of
// DecisionRouteDb::calculateUpdate (SpfSolver.cpp:21-56): every new or changed
// route, every deleted prefix. The variant kernels already mark those
// prefixes in a per-unit bitmap (route_stream.h: route_changed). This kernel
// gathers the records of exactly the marked prefixes into one compact,
// unit-major, prefix-ascending list, so the host materialises routes for the
// changes only and the D2H copy is proportional to the update, not to
// units x prefixes.
//
// One wavefront per unit (4 per workgroup): 64 bitmap words per step, a wave
// prefix scan of their popcounts gives each lane its output position, every
// lane then writes its word's records. Byte-bound; reads the bitmap once and
// only the changed records.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "spf_core.h"

namespace ogs {

template <int W>
__global__ __launch_bounds__(kBlock) void route_changes_kernel(
    const uint32_t* __restrict__ changed, uint32_t nUnits, uint32_t Sp,
    const uint32_t* __restrict__ meta, const uint32_t* __restrict__ metric,
    const uint32_t* __restrict__ mask, ogs_route_changes out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t u = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (u >= nUnits) return;  // whole wave leaves together
  const uint32_t words = (Sp + 31u) / 32u;
  const uint32_t* row = changed + size_t(u) * words;
  uint32_t pos = out.offsets[u];
  const uint32_t end = out.offsets[u + 1];
  const size_t total = out.total;
  for (uint32_t w0 = 0; w0 < words; w0 += 64u) {
    const uint32_t w = w0 + lane;
    uint32_t bits = w < words ? row[w] : 0u;
    if (w == words - 1u && (Sp & 31u)) bits &= (1u << (Sp & 31u)) - 1u;
    const uint32_t c = uint32_t(__popc(bits));
    uint32_t incl = c;  // inclusive wave scan of the popcounts
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= uint32_t(d)) incl += y;
    }
    uint32_t o = pos + incl - c;
    for (; bits; bits &= bits - 1u) {
      const uint32_t p = w * 32u + uint32_t(__builtin_ctz(bits));
      if (o < end) {  // never past the unit's slice, even on a bad scan
        const size_t r = size_t(u) * Sp + p;
        out.prefix[o] = p;
        out.meta[o] = meta[r];
        out.metric[o] = metric[r];
#pragma unroll
        for (int k = 0; k < W; ++k) {
          out.mask[size_t(k) * total + o] = mask[(size_t(u) * W + k) * Sp + p];
        }
      }
      ++o;
    }
    pos += __shfl(incl, 63, 64);
  }
}

hipError_t launch_route_changes(const uint32_t* changed, int nUnits, int Sp, int W,
                                const uint32_t* meta, const uint32_t* metric,
                                const uint32_t* mask, const ogs_route_changes& out,
                                hipStream_t stream) {
  const dim3 grid(unsigned((nUnits + kBlock / 64 - 1) / (kBlock / 64)));
  const uint32_t U = uint32_t(nUnits), P = uint32_t(Sp);
  switch (W) {
    case 1: hipLaunchKernelGGL(route_changes_kernel<1>, grid, dim3(kBlock), 0, stream, changed, U, P, meta, metric, mask, out); break;
    case 2: hipLaunchKernelGGL(route_changes_kernel<2>, grid, dim3(kBlock), 0, stream, changed, U, P, meta, metric, mask, out); break;
    default: hipLaunchKernelGGL(route_changes_kernel<4>, grid, dim3(kBlock), 0, stream, changed, U, P, meta, metric, mask, out); break;
  }
  return hipGetLastError();
}

}  // namespace ogs
