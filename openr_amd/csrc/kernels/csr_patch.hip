// csr_patch.hip — in-place update of a device-resident CSR after a link or
// node attribute change.
//
// Reference: LinkState::updateAdjacencyDatabase (LinkState.cpp:440-640)
// changes link metrics, overload bits, usability and node overload/drain in
// place; the topology (node set, link set) stays. The host patches the edge
// words of exactly the touched links (both directions) and of the edges into
// a node whose overload bit flipped, and this kernel scatters them into the
// HBM copy, instead of re-flattening and re-uploading the whole CSR.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "openr_gpu.h"
#include "spf_core.h"

namespace ogs {

__global__ __launch_bounds__(kBlock) void csr_patch_kernel(
    uint64_t* __restrict__ edges, const uint32_t* __restrict__ idx,
    const uint64_t* __restrict__ val, uint32_t n) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) edges[idx[i]] = val[i];
}

hipError_t launch_csr_patch(uint64_t* edges, const uint32_t* idx, const uint64_t* val,
                            int n, hipStream_t stream) {
  const dim3 grid(unsigned((n + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(csr_patch_kernel, grid, dim3(kBlock), 0, stream, edges, idx, val,
                     uint32_t(n));
  return hipGetLastError();
}

}  // namespace ogs
