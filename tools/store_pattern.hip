// store_pattern.hip — HBM write ceiling of the C3 RouteDb stream's store
// pattern without its SPF / gathers (diagnostic, not part of the product).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/store_pattern tools/store_pattern.hip
// Run:   tools/store_pattern [units=2080] [prefixes=208000]  (sweeps LDS per workgroup)
//
// Forms (same 3 x 4 B per (unit, prefix) output volume as one C3 W = 1 build):
//   flat      one grid-stride 16-B store stream over the whole volume
//   rows_nt   one workgroup per unit, three rows (meta, metric, mask), four
//             prefixes per lane, 16-B non-temporal stores (the C3 stream)
//   rows      the same with ordinary stores
//   rows_seq  one workgroup per unit, the three rows written one after the
//             other (one store stream per workgroup at a time)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

__global__ __launch_bounds__(256) void flat_kernel(uint32_t* p, size_t n4) {
  const size_t stride = size_t(gridDim.x) * 256;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += stride) {
    u32x4 v = {uint32_t(i), 1u, 2u, 3u};
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p) + i);
  }
}

template <bool NT, int X>
__global__ __launch_bounds__(256) void rows_kernel(uint32_t* meta, uint32_t* metric,
                                                   uint32_t* mask, uint32_t Sp) {
  extern __shared__ char smem[];
  if (threadIdx.x == 0) smem[0] = 0;
  const size_t u = blockIdx.x;
  uint32_t* a = meta + u * Sp;
  uint32_t* b = metric + u * Sp;
  uint32_t* c = mask + u * Sp;
  for (uint32_t q = threadIdx.x * 4u * X; q < Sp; q += 256u * 4u * X) {
#pragma unroll
    for (int x = 0; x < X; ++x) {
      const uint32_t r = q + 4u * x;
      if (r >= Sp) break;
      u32x4 v = {r, r + 1, r + 2, r + 3};
      if (NT) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(a + r));
        __builtin_nontemporal_store(v + 1u, reinterpret_cast<u32x4*>(b + r));
        __builtin_nontemporal_store(v + 2u, reinterpret_cast<u32x4*>(c + r));
      } else {
        *reinterpret_cast<u32x4*>(a + r) = v;
        *reinterpret_cast<u32x4*>(b + r) = v + 1u;
        *reinterpret_cast<u32x4*>(c + r) = v + 2u;
      }
    }
  }
}

__global__ __launch_bounds__(256) void rows_seq_kernel(uint32_t* meta, uint32_t* metric,
                                                       uint32_t* mask, uint32_t Sp) {
  extern __shared__ char smem[];
  if (threadIdx.x == 0) smem[0] = 0;
  const size_t u = blockIdx.x;
  uint32_t* rows[3] = {meta + u * Sp, metric + u * Sp, mask + u * Sp};
  for (int k = 0; k < 3; ++k) {
    for (uint32_t q = threadIdx.x * 4u; q < Sp; q += 1024u) {
      u32x4 v = {q, q + 1, q + 2, uint32_t(k)};
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(rows[k] + q));
    }
  }
}

template <typename F>
float timed(F launch) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int i = 0; i < 6; ++i) {
    CHECK(hipEventRecord(e0, 0));
    launch();
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (i) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
  const uint32_t U = argc > 1 ? uint32_t(std::atoi(argv[1])) : 2080u;
  const uint32_t Sp = argc > 2 ? uint32_t(std::atoi(argv[2])) : 208000u;
  if (Sp % 4 || U == 0) {
    std::fprintf(stderr, "prefixes must be a multiple of 4, units > 0\n");
    return 1;
  }
  const size_t row = size_t(U) * Sp;
  const size_t bytes = 3 * row * 4;
  uint32_t* buf = nullptr;
  CHECK(hipMalloc(&buf, bytes));
  uint32_t *meta = buf, *metric = buf + row, *mask = buf + 2 * row;
  auto tbps = [&](float ms) { return double(bytes) / (ms * 1e-3) / 1e12; };
  const void* ks[] = {reinterpret_cast<const void*>(rows_kernel<true, 1>),
                      reinterpret_cast<const void*>(rows_kernel<false, 1>),
                      reinterpret_cast<const void*>(rows_seq_kernel)};
  for (const void* k : ks) {
    CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  }
  std::printf("units %u prefixes %u: %.3f GB per pass (median of 5; 3 sweeps)\n", U, Sp,
              bytes / 1e9);
  const uint32_t ldsSweep[] = {0, 21000, 27000, 33000, 40000, 54000, 81000};
  for (int sweep = 0; sweep < 3; ++sweep) {
    float ms = timed([&] {
      hipLaunchKernelGGL(flat_kernel, dim3(256 * 32), dim3(256), 0, 0, buf, bytes / 16);
    });
    std::printf("sweep %d flat %.3f ms %.2f TB/s\n", sweep, ms, tbps(ms));
    for (uint32_t lds : ldsSweep) {
      const float a = timed([&] {
        hipLaunchKernelGGL((rows_kernel<true, 1>), dim3(U), dim3(256), lds, 0, meta, metric,
                           mask, Sp);
      });
      const float b = timed([&] {
        hipLaunchKernelGGL((rows_kernel<false, 1>), dim3(U), dim3(256), lds, 0, meta, metric,
                           mask, Sp);
      });
      const float c = timed([&] {
        hipLaunchKernelGGL(rows_seq_kernel, dim3(U), dim3(256), lds, 0, meta, metric, mask, Sp);
      });
      std::printf("sweep %d lds %6u  rows_nt %.2f  rows %.2f  rows_seq_nt %.2f TB/s\n", sweep,
                  lds, tbps(a), tbps(b), tbps(c));
    }
  }
  CHECK(hipFree(buf));
  return 0;
}
