// Probe library for bench/probes/prefetch_probe.py: a streaming read of a buffer (results
// folded into one word that is stored only under an impossible condition) to pull it into
// the Infinity Cache ahead of a kernel that consumes it. NT = 1: non-temporal loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void prefetch_kernel(const u32x4* __restrict__ p, long n16,
                                                       unsigned* sink) {
  unsigned acc = 0;
  const long stride = (long)gridDim.x * 256 * 4;
  for (long i = (long)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long j = i + u * 256;
      if (j < n16) v[u] = NT ? __builtin_nontemporal_load(p + j) : p[j];
      else v[u] = u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x9E3779B9u) *sink = acc;  // data-dependent: keeps the loads, (practically) never stores
}

extern "C" int prefetch_launch(const void* p, long bytes, int blocks, int nt, unsigned* sink,
                               hipStream_t s) {
  const long n16 = bytes / 16;
  if (nt)
    hipLaunchKernelGGL(prefetch_kernel<true>, dim3(blocks), dim3(256), 0, s, (const u32x4*)p, n16, sink);
  else
    hipLaunchKernelGGL(prefetch_kernel<false>, dim3(blocks), dim3(256), 0, s, (const u32x4*)p, n16, sink);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}
