// LDS-DMA intake rate per CU versus bytes in flight (bench/probes/ldsdma_rate.py).
//
// Every workgroup streams `steps` tiles of TILE bytes from a source buffer into an LDS ring of
// NS slots with LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction), keeping NS - 1
// tiles in flight (counted vmcnt waits, one s_barrier per tile, nothing else) -- the load
// pattern of the GEMM main loops without their MFMAs. The source is either a small buffer all
// workgroups re-read (L2-resident) or a large one each workgroup sweeps once (HBM). The probe
// answers: is a k-step of the wgrad / forward loops bound by latency (rate grows with the
// bytes in flight) or by a per-CU intake ceiling (rate flat)?
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LDS_AS __attribute__((address_space(3)))

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
template <int NS, int TILE_KB, int NW>
__global__ __launch_bounds__(NW * 64) void ldsdma_stream(const char* __restrict__ src,
                                                         long src_bytes, int steps, int sweep,
                                                         unsigned long long* out) {
  __shared__ __attribute__((aligned(16))) char lds[NS * TILE_KB * 1024];
  constexpr int PIECES = TILE_KB / NW;  // 1 KiB wave-instructions per wave per tile
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // each workgroup's tile sequence: sweep = its own contiguous range of a large buffer (HBM),
  // else all workgroups read the same small window (L2-resident)
  const long wg_base = sweep ? (long)blockIdx.x * steps * TILE_KB * 1024L : 0;
  const long wrap = sweep ? src_bytes : (long)TILE_KB * 1024 * 32;  // 32-tile window
  auto issue = [&](int t, int slot) {
    const long tb = (wg_base + (long)t * TILE_KB * 1024) % wrap;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int piece = i * NW + wave;
      const char* a = src + tb + piece * 1024 + lane * 16;
      const unsigned m0v = __builtin_amdgcn_readfirstlane(
          (unsigned)(size_t)(lds + slot * TILE_KB * 1024 + piece * 1024));
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(a), "s"(m0v)
                   : "memory", "m0");
    }
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s, s);
  for (int t = 0; t < steps; ++t) {
    wait_vmcnt<(NS - 2) * PIECES>();  // own pieces of tile t landed
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(t + NS - 1, (t + NS - 1) % NS);  // past the end: re-reads, never waited for
  }
  wait_vmcnt<0>();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  // keep the LDS live: one read per lane into a discarded sum
  if (lds[threadIdx.x] == 127 && lane == 63) out[blockIdx.x] |= 1ull << 63;
}
#pragma clang diagnostic pop

typedef void (*fn_t)(const char*, long, int, int, unsigned long long*);

template <int NS, int KB, int NW>
static int run(const char* src, long bytes, int steps, int sweep, unsigned long long* out,
               int wgs, hipStream_t s) {
  hipLaunchKernelGGL((ldsdma_stream<NS, KB, NW>), dim3(wgs), dim3(NW * 64), 0, s, src, bytes,
                     steps, sweep, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// code = NS * 1000 + tile KiB * 10 + waves / 4 (4 or 8 waves)
extern "C" int ldsdma_probe(int code, const void* src, long bytes, int steps, int sweep,
                            void* out, int wgs, void* stream) {
  const char* p = (const char*)src;
  auto* o = (unsigned long long*)out;
  hipStream_t s = (hipStream_t)stream;
  switch (code) {
#define C(NS, KB, NW) \
  case NS * 1000 + KB * 10 + NW / 4: return run<NS, KB, NW>(p, bytes, steps, sweep, o, wgs, s);
    C(2, 16, 4) C(3, 16, 4) C(4, 16, 4) C(6, 16, 4) C(8, 16, 4)
    C(2, 32, 4) C(3, 32, 4) C(4, 32, 4)
    C(2, 32, 8) C(3, 32, 8) C(4, 32, 8) C(2, 64, 8) C(2, 48, 8) C(3, 48, 8)
    C(5, 32, 8) C(10, 16, 8)
#undef C
    default: return -2;
  }
}
