// Host-visible interface of the fused classifier-tail kernel (csrc/kernels/mlp_tail.hip).
//
// For the last two layers of a stage whose hidden widths are narrow (K3 <= 256 inputs,
// N3 <= 128 hidden units, <= 16 classes), ONE launch runs, per 16-row block and entirely out
// of registers + a small per-wave LDS scratch:
//   h3  = act3(X . W3^T + b3)                         forward of layer L-2   -> H3
//   dz4 = (softmax(h3 . W4^T + b4) - onehot) * scale  forward + CE of L-1    -> DZ4, loss, correct
//   dz3 = (dz4 . W4) * act3'(h3)                      dgrad of layer L-1     -> DZ3
//   dz2 = (dz3 . W3) * act2'(X)                       dgrad of layer L-2     -> DZ2
// plus the bias-gradient partials (column sums of the stored dz4 / dz3 / dz2) per workgroup.
// These are the four kernels fwd3 / fwd4+xent / dgrad4 / dgrad3 of the unfused step, each
// latency-bound at 2-20 % MFMA on the headline model (profiles/r1_final/pmc_step_kernels.txt).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dnn {

struct TailParams {
  const uint16_t* X;  // [M][K3] input of layer L-2 (and the activation act2 differentiates)
  long ldx;
  const uint16_t* W3;  // [N3][K3]
  long ldw3;
  const float* b3;     // [N3]
  const uint16_t* W4;  // [N4][N3], N4 = padded classes (64 or 128), rows >= n_cls zero
  long ldw4;
  const float* b4;     // [N4]
  const int* labels;   // [M], < 0 = padding row
  uint16_t* H3;        // [M][N3]
  long ldh3;
  uint16_t* DZ4;       // [M][N4]: columns 0..15 written; 16..N4-1 must already be zero (never
                       // written: the caller zero-initialises the buffer once)
  long lddz4;
  uint16_t* DZ3;       // [M][N3]
  long lddz3;
  uint16_t* DZ2;       // [M][K3]
  long lddz2;
  float* loss_part;    // [nwg]
  int* correct;        // [nwg]
  float* cs4;          // [nwg][ld_cs4] (N4 columns written)
  long ld_cs4;
  float* cs3;          // [nwg][ld_cs3] (N3 columns)
  long ld_cs3;
  float* cs2;          // [nwg][ld_cs2] (K3 columns)
  long ld_cs2;
  int M, K3, N3, N4, n_cls;
  float scale;
  int act3, act2;  // Act codes
};

// Workgroups (= partials per output) the tail launch uses for M rows.
int mlp_tail_blocks(int M);
// 0, or < 0 on an unsupported geometry / launch failure (see mlp_tail_error).
int mlp_tail(const TailParams& p, hipStream_t stream);
// The forward of the layer before the tail (g: A [M][K] . W [256][K]^T + bias, ReLU, C == the
// tail's X) fused in front of the tail: one workgroup per 256-row tile, M / 256 partials, which
// must equal mlp_tail_blocks(M). -2 = unsupported geometry (the caller keeps two launches).
struct GemmParams;
const char* mlp_tail_error(int code);

}  // namespace dnn
