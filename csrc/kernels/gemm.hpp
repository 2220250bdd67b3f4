// Host-visible interface of the bf16 MFMA GEMM family (csrc/kernels/gemm.hip).
//
// C[M,N] (+)= epilogue( sum_k A[m,k] * B[k,n] ), bf16 inputs, fp32 accumulation.
// Each operand is stored either contraction-contiguous (KMAJ: [MN][K]) or
// output-dim-contiguous (MNMAJ: [K][MN]); the three training GEMMs of a Linear layer are
//   forward  Y  = X  . W^T : A = X  KMAJ , B = W  KMAJ   (W stored nn.Linear-style [out][in])
//   dgrad    dX = dZ . W   : A = dZ KMAJ , B = W  MNMAJ
//   wgrad    dW = dZ^T . X : A = dZ MNMAJ, B = X  MNMAJ  (contraction over the batch)
// so no transposed copy of any tensor is ever materialised: MNMAJ tiles are read with the
// gfx950 transposing LDS read (ds_read_b64_tr_b16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dnn {

enum Layout : int { KMAJ = 0, MNMAJ = 1 };

struct GemmParams {
  const uint16_t* A;  // bf16
  long lda;           // elements between consecutive storage rows of A
  const uint16_t* B;  // bf16
  long ldb;
  void* C;              // bf16 or f32
  long ldc;
  long c_split_stride;  // elements between split-K output slabs (f32 output only)
  const float* bias;    // optional, [N] fp32, added in the epilogue
  const uint16_t* aux;  // optional, bf16 activation output used for the backward mask
  long ld_aux;
  int M, N, K;     // K = contraction length handled by ONE split (uniform split-K)
  int k_total;     // > 0: uneven split-K over k_total (split s: k-steps [s*KS/S, (s+1)*KS/S))
  int act;         // Act code: forward activation, or (with aux) the activation to differentiate
  int accumulate;  // f32 output: C += result (split slab accumulation across micro-batches)
  float* colsum;   // optional (bf16 output only): colsum[tile_m][n] = sum over the tile's rows
  long ld_colsum;  //   of the stored (bf16-rounded) output -> bias-gradient partials of dgrad
  // Fused softmax cross-entropy epilogue (bf16 output, N == bn: a row is one tile). When
  // xent_labels is set the kernel computes logits = acc + bias, and stores
  // dz = (softmax(logits[:n_cls]) - onehot(label)) * xent_scale instead of the logits;
  // loss_part[tile_m] = sum of -log p[label] over the tile's rows, correct[tile_m] = #argmax==label
  // (per-tile partials, written not accumulated: no per-step zeroing, fixed-order host sum).
  const int* xent_labels;
  int n_cls;
  float xent_scale;
  float* loss_part;
  int* correct;
  // raster order: row-tiles per group (<= 0: launcher default, 1 = row-major tiles)
  int group_m;
  // 1-bit ReLU masks, ceil(M/16) x ld_mask x 16 bytes, row-block-major (gemm_tile.hpp
  // mask_index: byte of row r, chunk c at ((r/16) * ld_mask + c) * 16 + r % 16); bit e of the
  // byte of chunk c = column 8c + e (bf16 output only):
  // mask_out (forward, act = relu): bit = stored bf16 output > 0; mask_in (dgrad, act = relu,
  // replaces aux): the derivative reads 1 bit per element instead of the 16-bit activation.
  // ld_mask < 0: FRAGMENT order instead (gemm_tile.hpp frag_mask_offset; register-direct
  // epilogue only, forward and dgrad on the same tile / wave layout).
  unsigned char* mask_out;
  const unsigned char* mask_in;
  long ld_mask;
  // optional second bf16 output, TRANSPOSED: ct[n][m] = the stored C[m][n] (bf16 output, the
  // one-tile form). A forward writes the next weight gradient's X^T, a dgrad its dZ^T, so that
  // wgrad reads both operands contraction-contiguous (ds_read_b128, no per-tile transpose).
  uint16_t* ct;
  long ld_ct;
  // Optional fused SGD update (f32 output, one split, no accumulation): instead of storing the
  // weight gradient C[m][n], the epilogue applies sgd4 to the fp32 master weights at the same
  // [m][n] (row stride ldc), momentum, and the bf16 shadow, and (with ct) writes the new bf16
  // weights transposed: W^T for the dgrad. lr from device memory.
  float* upd_master;
  float* upd_mom;
  uint16_t* upd_shadow;
  const float* upd_lr;
  float upd_mu, upd_wd;
  // optional per-workgroup phase timestamps (one-tile kernels; bench/probes/gemm_timeline.py):
  // timeline[4 * blockIdx.x + i] = s_memrealtime (100 MHz) at kernel entry (i = 0), after the
  // ring prologue (1), after the main loop (2) and at the end of the epilogue (3).
  unsigned long long* timeline;
  // Diagnosis only (bench/probes/gemm_timeline.py --epi-probe; results are WRONG when set):
  // bit 0 = the register-direct epilogue stores nothing, bit 1 = it loads no bias (zeros);
  // bit 2 (results correct) = the activation read per element, as before round 4 (A/B).
  int epi_probe;
};

// Returns 0 on success, a negative code when a shape/alignment precondition fails
// (nothing is launched then).
// stages: LDS pipeline depth 2..4 (0 = default_stages(bm, bn)).
// persist: 0 = one tile per workgroup (gemm.hip); != 0 = persistent workgroups walking tile
// runs with a register-direct epilogue (gemm_persist.hip): > 0 workgroup count, < 0 one round
// of resident workgroups. The fused cross-entropy always runs the one-tile form.
// Several problems with one 4-wave tile configuration (64|128 x 64|128, 2 stages) in ONE
// launch (each validated like gemm_bf16; splits per problem).
constexpr int GEMM_GROUP_MAX = 8;
struct GemmGroup {
  GemmParams p[GEMM_GROUP_MAX];
  int tiles_n[GEMM_GROUP_MAX], tiles_m[GEMM_GROUP_MAX], nwg[GEMM_GROUP_MAX];
  int start[GEMM_GROUP_MAX + 1];
  int n;
};
int gemm_bf16_group(const GemmParams* ps, const int* splits, int n, int layout_a, int layout_b,
                    int out_f32, int bm, int bn, int stages, hipStream_t stream);
// The argument checks of gemm_bf16 (0 or its error code).
int gemm_check(const GemmParams& p, int layout_a, int layout_b, int out_f32, int bm, int bn,
               int splits);
int gemm_bf16(const GemmParams& p, int layout_a, int layout_b, int out_f32, int bm, int bn,
              int splits, hipStream_t stream, int stages = 0, int persist = 0);
// stages == 8 with 256x256 tiles: the ping-pong, half-tile-streamed main loop (gemm_pp.hip).
int gemm_pp_launch(const GemmParams& q, int la, int lb, int out_f32, int splits,
                   hipStream_t stream);
// stages == 6 / 9 / 11: the register-prefetched main loop (gemm_rp.hip).
int gemm_rp_launch(const GemmParams& q, int la, int lb, int out_f32, int bm, int bn, int splits,
                   int ns, hipStream_t stream);
int gemm_persist_launch(const GemmParams& q, int la, int lb, int out_f32, int bm, int bn,
                        int splits, int ns, int persist, hipStream_t stream);
int default_stages(int bm, int bn);
// Tiles: 64|128 x 64|128 (4 waves, 256 threads) and 256 x 64|128|256, 128 x 256 (8 waves).
bool gemm_tile_supported(int bm, int bn);
int gemm_tile_threads(int bm, int bn);

// Stream-K form for batch-contraction (wgrad) GEMMs with few output tiles: `nwg` workgroups take
// equal shares of the (tile, k-step) space, write fp32 partial tiles to `part`
// (nwg * 2 * bm * bn floats), and a reduction kernel sums them in a fixed order into the fp32 C
// (C += when p.accumulate). p.K is the FULL contraction length.
int gemm_bf16_streamk(const GemmParams& p, int layout_a, int layout_b, int bm, int bn, int nwg,
                      float* part, hipStream_t stream);

const char* gemm_error_string(int code);

}  // namespace dnn
