// Library GEMM path: hipBLASLt for the plain large products where its assembly-scheduled
// kernels beat the hand-written ones (docs/DESIGN.md "Large GEMMs": 4-wave 128x128-per-wave
// tiles with software pipelining that HIP source does not control).
//
// Row-major problem:  D[M][N] (=|+=) epi( op(A) . op(B) ), bf16 A/B, fp32 accumulation,
// D bf16 or fp32. The three training products of a Linear layer map onto it as
//   fwd    Y  = X . W^T    (bias [+ ReLU] in hipBLASLt's epilogue)
//   dgrad  dX = dZ . W     (no epilogue; the activation derivative + bias-gradient partials
//                           run as dact_colsum in elementwise.hip)
//   wgrad  dW = dZ^T . X   (fp32 output, beta = 1 accumulates)
// Descriptors, layouts and the heuristic's algorithm are built once per problem signature and
// cached; a call only patches the pointers. Calls are stream-ordered; each stream gets its own
// workspace.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dnn {

struct BlasGemm {
  int trans_a, trans_b;  // row-major operands: A is [M][K] (0) or [K][M] (1); B is [K][N] (0)
                         // or [N][K] (1)
  int M, N, K;
  const uint16_t* A;
  long lda;
  const uint16_t* B;
  long ldb;
  void* D;
  long ldd;
  int d_f32;           // D fp32 (else bf16)
  const float* bias;   // [N] fp32 or null
  int relu;            // ReLU after the bias (fwd)
  int accumulate;      // D += result (fp32 D only)
  int algo;            // index into the heuristic's candidate list (0 = its first choice;
                       // the in-step tuner stores the measured best per GEMM)
};

// 0 on success; < 0: -1 bad arguments, -2 library error, -3 no algorithm for the problem.
int blas_gemm(const BlasGemm& g, hipStream_t stream);
const char* blas_error(int code);
// Whether the library initialises at all, and whether it has an algorithm for a problem
// signature (pointers are ignored; the plan is cached for the later calls).
int blas_available();
int blas_supported(const BlasGemm& g);

}  // namespace dnn
