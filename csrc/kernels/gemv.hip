// Skinny forward layer for serving (batch 1..8): y[m][n] = act(sum_k x[m][k] W[n][k] + b[n]).
//
// The MFMA GEMM tiles rows by 64; a batch-1 request padded to 64 rows through a 1024-wide
// layer launches 16 workgroups that each stream K serially -- ~16 us per layer. Here one WAVE
// owns one output neuron: W is stored [N][K] (nn.Linear layout), so its row is contiguous and
// the wave reads it with 16-byte loads (all issued before any is used), multiplies with the
// <= 8 input rows (L2-resident, shared by every wave), reduces across the wave and applies
// bias + activation. A 1024-wide layer is 1024 waves -- the whole chip -- at ~2 L2/HBM round
// trips. Replaces the per-stage np.dot of /root/reference/src/grpc_node.py:75-97 on the
// latency path (BASELINE config 5: 8-stage chain, batch 1).
#include "common.hpp"
#include "gemv.hpp"

namespace dnn {

constexpr int GEMV_WAVES = 4;  // waves (= output neurons) per 256-thread block

// M = compile-time row capacity (1, 2, 4, 8); rows = actual rows (<= M): rows beyond `rows`
// are never read or written.
template <int M, bool OUT_F32>
__global__ __launch_bounds__(256) void gemv_kernel(const u16* __restrict__ x, long ldx,
                                                   const u16* __restrict__ w, long ldw,
                                                   const float* __restrict__ bias,
                                                   void* __restrict__ y, long ldy, int rows, int N,
                                                   int K, int act) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * GEMV_WAVES + (threadIdx.x >> 6);
  if (n >= N) return;  // whole wave exits together
  const u16* wr = w + (long)n * ldw;
  float acc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) acc[m] = 0.f;
  // K is a multiple of 8; chunks of 512 elements = 64 lanes x 8. Up to 4 chunks (K <= 2048)
  // are loaded before use; longer rows loop.
  constexpr int U = 4;
  for (int k0 = 0; k0 < K; k0 += 512 * U) {
    bf16x8_t wv[U], xv[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * 512 + lane * 8;
      if (k < K) {
        wv[u] = *(const bf16x8_t*)(wr + k);
#pragma unroll
        for (int m = 0; m < M; ++m)
          xv[u][m] = m < rows ? *(const bf16x8_t*)(x + m * ldx + k) : bf16x8_t{};
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * 512 + lane * 8;
      if (k < K) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float we = bf2f((u16)wv[u][e]);
#pragma unroll
          for (int m = 0; m < M; ++m) acc[m] += we * bf2f((u16)xv[u][m][e]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m) acc[m] = wave_sum(acc[m]);
  if (lane < rows) {
    float v = 0.f;
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (m == lane) v = acc[m];
    v += bias ? bias[n] : 0.f;
    v = act_fwd(v, act);
    if constexpr (OUT_F32)
      ((float*)y)[(long)lane * ldy + n] = v;
    else
      ((u16*)y)[(long)lane * ldy + n] = f2bf(v);
  }
}

int gemv_bf16(const uint16_t* x, long ldx, const uint16_t* w, long ldw, const float* bias,
              void* y, long ldy, int M, int N, int K, int act, int out_f32, hipStream_t stream) {
  if (M < 1 || M > GEMV_MAX_ROWS || N < 1 || K < 8 || K % 8) return -1;
  if (ldx < K || ldw < K || ldy < N || ldx % 8 || ldw % 8) return -2;
  if ((((uintptr_t)x) | ((uintptr_t)w)) & 15) return -5;
  const dim3 grid((N + GEMV_WAVES - 1) / GEMV_WAVES), block(256);
#define DNN_GEMV(MM)                                                                         \
  if (out_f32)                                                                               \
    hipLaunchKernelGGL((gemv_kernel<MM, true>), grid, block, 0, stream, x, ldx, w, ldw, bias, \
                       y, ldy, M, N, K, act);                                                \
  else                                                                                       \
    hipLaunchKernelGGL((gemv_kernel<MM, false>), grid, block, 0, stream, x, ldx, w, ldw,     \
                       bias, y, ldy, M, N, K, act);
  switch (M) {
    case 1: DNN_GEMV(1) break;
    case 2: DNN_GEMV(2) break;
    case 3:  // rows 3..4 on the 4-row kernel, 5..8 on the 8-row one (guarded by `rows`)
    case 4: DNN_GEMV(4) break;
    default: DNN_GEMV(8) break;
  }
#undef DNN_GEMV
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

}  // namespace dnn
