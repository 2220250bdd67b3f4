// Does hipExtAnyOrderLaunch let a kernel start before the previous kernel on the SAME stream
// has finished (AQL barrier bit clear)? Kernel A: one workgroup records its start, spins
// ~100 us of wall clock, records its end. Kernel B (launched right after A on the same stream,
// with or without the flag): records its start. Prints A start/end and B start (wall-clock
// ticks, 100 MHz) for both launch forms.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void spin_kernel(unsigned long long* t, unsigned long long ticks) {
  if (threadIdx.x) return;
  const unsigned long long t0 = wall_clock64();
  t[0] = t0;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  t[1] = wall_clock64();
}

__global__ void stamp_kernel(unsigned long long* t) {
  if (threadIdx.x == 0 && blockIdx.x == 0) t[2] = wall_clock64();
}

int main() {
  unsigned long long* d;
  unsigned long long h[3];
  if (hipMalloc(&d, 64) != hipSuccess) return 1;
  hipStream_t s;
  hipStreamCreate(&s);
  for (int flag = 0; flag < 2; ++flag) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemsetAsync(d, 0, 64, s);
      hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, d, 10000ull);
      hipExtLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, s, nullptr, nullptr,
                            flag ? hipExtAnyOrderLaunch : 0u, d);
      hipStreamSynchronize(s);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("{\"anyorder\": %d, \"a_us\": %.1f, \"b_start_minus_a_end_us\": %.1f}\n", flag,
             (h[1] - h[0]) / 100.0, ((long long)h[2] - (long long)h[1]) / 100.0);
    }
  }
  printf("%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
