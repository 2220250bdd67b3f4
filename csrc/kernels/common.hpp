// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of docker_dist_nn_amd.
//
// Everything here is written for wave64 + MFMA; there is no other target.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define LDS_AS __attribute__((address_space(3)))

namespace dnn {

constexpr int kWave = 64;

// Activation codes shared with the host (docker_dist_nn_amd/ops/native.py keeps the same table).
enum Act : int { ACT_LINEAR = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_SOFTMAX = 3 };

__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((unsigned)h) << 16); }

// Round-to-nearest-even f32 -> bf16 through the native conversion (v_cvt_pk_bf16_f32 at -O3,
// NaN-preserving; see MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ u16 f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(u16, b);
}

__device__ __forceinline__ float act_fwd(float v, int act) {
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_SIGMOID) return 1.f / (1.f + __expf(-v));
  return v;
}

// d(act)/dz expressed through the stored activation output y.
__device__ __forceinline__ float act_bwd(float g, float y, int act) {
  if (act == ACT_RELU) return y > 0.f ? g : 0.f;
  if (act == ACT_SIGMOID) return g * y * (1.f - y);
  return g;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// One SGD step on 4 elements (weight decay, optional momentum, optional bf16 shadow): shared
// by sgd_kernel, the fused reduction (reduce_multi) and the fused-update weight-gradient
// epilogue (gemm_tile.hpp), so every path produces the same bits.
__device__ __forceinline__ f32x4_t sgd4(float* __restrict__ p, f32x4_t gv,
                                        float* __restrict__ mom, u16* __restrict__ shadow,
                                        float lr, float mu, float wd) {
  f32x4_t pv = *(const f32x4_t*)p;
  gv += wd * pv;
  if (mom) {
    f32x4_t m = *(const f32x4_t*)mom;
    m = mu * m + gv;
    *(f32x4_t*)mom = m;
    gv = m;
  }
  pv -= lr * gv;
  *(f32x4_t*)p = pv;
  if (shadow) {
    bf16x4_t o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(pv[e]);
    *(bf16x4_t*)shadow = o;
  }
  return pv;  // the updated weights
}

}  // namespace dnn
