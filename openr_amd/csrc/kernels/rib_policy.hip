// rib_policy.hip — RibPolicy (UCMP next-hop weights) over the RouteDb records
// of a launch, one thread per (unit, prefix): SURVEY.md §8(a) row a16.
//
// Reference: RibPolicy::applyPolicy (RibPolicy.cpp:231-249) -> applyAction
// (221-229): statements in order, the first whose action keeps at least one
// next hop wins. RibPolicyStatement::match (74-107): no matcher -> never;
// tag matcher: the best entry's tags meet the statement's tags; prefix
// matcher: the route's prefix is in the set. RibPolicyStatement::applyAction
// (109-161): counterID is assigned on every matching statement (even one
// whose weights then drop every next hop); per next hop weight = neighbor
// weight, else area weight, else default; weight 0 drops the next hop; all
// dropped -> route unchanged, next statement.
// The host compiles the string matchers into bitsets over the prefix table
// (pfx_match, adv_tag_match) and the weights into per-source link-slot
// nonzero masks, so the device work is a bitwise segmented reduction.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "spf_core.h"

namespace ogs {

// W == 0: next-hop masks of runtime width Wr (sources of 512+ links)
template <int W>
__global__ __launch_bounds__(kBlock) void rib_policy_kernel(
    ogs_prefix_table pt, ogs_rib_policy pol, uint32_t A,
    const uint32_t* __restrict__ meta, uint32_t* __restrict__ mask,
    uint16_t* __restrict__ applied, uint16_t* __restrict__ counter, int Wr) {
  const int WW = W > 0 ? W : Wr;
  const uint32_t u = blockIdx.y;
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t p0 = pt.pfx_base[0];
  const uint32_t P = pt.pfx_base[1] - p0;
  if (p >= P) return;
  const uint32_t Sp = uint32_t(pt.max_prefixes);
  const uint32_t K = uint32_t(pol.num_statements);
  const size_t o = size_t(u) * Sp + p;
  const uint32_t m = meta[o];
  const uint32_t base = uint32_t(pol.statement_base);
  uint32_t app = OGS_POLICY_NONE, cnt = OGS_POLICY_NONE;
  if (base) {  // a later chunk: keep what earlier statements decided
    app = applied[o];
    cnt = counter[o];
    if (app != OGS_POLICY_NONE) return;
  }
  if (m & OGS_ROUTE_VALID) {
    const uint32_t gp = p0 + p;
    const uint32_t best = pt.adv_off[gp] + (m >> OGS_ROUTE_BEST_SHIFT);
    uint32_t cand = pol.pfx_match[gp] & pol.adv_tag_match[best] & pol.active;
    const uint32_t* nz = pol.slot_nonzero + size_t(u) * K * A * WW;
    for (; cand; cand &= cand - 1) {
      const uint32_t k = __builtin_ctz(cand);
      cnt = base + k;  // counterID set by every matching statement
      bool any = false;
      for (uint32_t a = 0; a < A; ++a) {
        for (int w = 0; w < WW; ++w) {
          any |= (mask[((size_t(u) * A + a) * WW + w) * Sp + p] &
                  nz[(size_t(k) * A + a) * WW + w]) != 0u;
        }
      }
      if (!any) continue;  // every next hop weighted 0: route unchanged
      app = base + k;
      for (uint32_t a = 0; a < A; ++a) {
        for (int w = 0; w < WW; ++w) {
          mask[((size_t(u) * A + a) * WW + w) * Sp + p] &= nz[(size_t(k) * A + a) * WW + w];
        }
      }
      break;
    }
  }
  if (applied) applied[o] = uint16_t(app);
  if (counter) counter[o] = uint16_t(cnt);
}

hipError_t launch_rib_policy(const ogs_prefix_table& pt, const ogs_rib_policy& pol,
                             int A, int nUnits, int W, const uint32_t* meta,
                             uint32_t* mask, uint16_t* applied, uint16_t* counter,
                             hipStream_t stream) {
  if (pt.max_prefixes <= 0) return hipSuccess;
  const dim3 grid(unsigned((pt.max_prefixes + kBlock - 1) / kBlock), unsigned(nUnits));
  switch (W) {
    case 1: hipLaunchKernelGGL(rib_policy_kernel<1>, grid, dim3(kBlock), 0, stream, pt, pol, uint32_t(A), meta, mask, applied, counter, 0); break;
    case 2: hipLaunchKernelGGL(rib_policy_kernel<2>, grid, dim3(kBlock), 0, stream, pt, pol, uint32_t(A), meta, mask, applied, counter, 0); break;
    case 4: hipLaunchKernelGGL(rib_policy_kernel<4>, grid, dim3(kBlock), 0, stream, pt, pol, uint32_t(A), meta, mask, applied, counter, 0); break;
    case 8: hipLaunchKernelGGL(rib_policy_kernel<8>, grid, dim3(kBlock), 0, stream, pt, pol, uint32_t(A), meta, mask, applied, counter, 0); break;
    case 16: hipLaunchKernelGGL(rib_policy_kernel<16>, grid, dim3(kBlock), 0, stream, pt, pol, uint32_t(A), meta, mask, applied, counter, 0); break;
    default: hipLaunchKernelGGL(rib_policy_kernel<0>, grid, dim3(kBlock), 0, stream, pt, pol, uint32_t(A), meta, mask, applied, counter, W); break;
  }
  return hipGetLastError();
}

}  // namespace ogs
