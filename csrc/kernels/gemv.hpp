// Skinny forward layer for serving batches of 1..GEMV_MAX_ROWS rows (csrc/kernels/gemv.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dnn {

constexpr int GEMV_MAX_ROWS = 8;

// y[m][n] = act(sum_k x[m][k] * w[n][k] + bias[n]) for m < M; x [M][ldx] bf16, w [N][ldw]
// bf16 (nn.Linear layout), y bf16 or fp32 (out_f32). K % 8 == 0, x and w 16-byte aligned.
int gemv_bf16(const uint16_t* x, long ldx, const uint16_t* w, long ldw, const float* bias,
              void* y, long ldy, int M, int N, int K, int act, int out_f32, hipStream_t stream);

}  // namespace dnn
