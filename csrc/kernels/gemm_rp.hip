// build-flags: -mllvm -amdgpu-mfma-vgpr-form=1
// Register-prefetched main-loop variants of the one-tile GEMM (stage codes 6, 9, 11; Cfg RP,
// mma_tile_rp in gemm_tile.hpp), in a translation unit of their own so the build compiles
// them in parallel with gemm.hip.
#include "gemm_kernel.hpp"

namespace dnn {

// Stage code 6: the register-prefetched main loop (Cfg RP, mma_tile_rp) over a 2-deep ring with
// the staged epilogue (the form that supports the transposed copy and the fused update).
// Code 9: the same loop with swapped MFMA operands and the register-direct epilogue (RP_ = 2):
// bias / activation / aux derivative / colsum / split-K f32, ReLU bit masks (both layouts,
// fragment order only here), no transposed copy, fused update or cross-entropy.
// Code 11: register-direct epilogue over the asymmetric ring (A 3 deep, B 2 deep: two k-steps
// for the streamed A panel to land), 256x256 / 256x128 / 128x128.
// (Round 5 removed the variants the tuned table never selects -- 3-deep RP rings (codes 7 /
// 10), 32-deep k-steps (12-14), the L2 touch-prefetch (15-17); the patch that restores them is
// profiles/r5_lean/removed_variants.patch.)
static gemm_fn pick_rp(int bm, int bn, int code, int la, int lb, int f32) {
  if (code == 11) {  // asymmetric A3/B2 ring, register-direct epilogue
#define DNN_RPA(BM, BN, WM, WN) pick_layout<Cfg<BM, BN, WM, WN, 3, 2, 64, 2>>(la, lb, f32)
    if (bm == 256 && bn == 256) return DNN_RPA(256, 256, 4, 2);
    if (bm == 256 && bn == 128) return DNN_RPA(256, 128, 4, 2);
    if (bm == 128 && bn == 128) return DNN_RPA(128, 128, 2, 2);
#undef DNN_RPA
    return nullptr;
  }
  if (code != 6 && code != 9) return nullptr;
  const int rpv = code == 9 ? 2 : 1;
#define DNN_RP(BM, BN, WM, WN)                                                            \
  (rpv == 2 ? pick_layout<Cfg<BM, BN, WM, WN, 2, 2, 64, 2>>(la, lb, f32)                \
            : pick_layout<Cfg<BM, BN, WM, WN, 2, 2, 64, 1>>(la, lb, f32))
  if (bm == 256 && bn == 256) return DNN_RP(256, 256, 4, 2);
  if (bm == 256 && bn == 128) return DNN_RP(256, 128, 4, 2);
  if (bm == 128 && bn == 128) return DNN_RP(128, 128, 2, 2);
  if (bm == 128 && bn == 64) return DNN_RP(128, 64, 2, 2);
  if (bm == 64 && bn == 64) return DNN_RP(64, 64, 2, 2);
#undef DNN_RP
  return nullptr;
}

int gemm_rp_launch(const GemmParams& q, int la, int lb, int out_f32, int bm, int bn, int splits,
                   int ns, hipStream_t stream) {
  gemm_fn f = pick_rp(bm, bn, ns, la, lb, out_f32);
  if (!f) return -12;
  const int tiles_n = (q.N + bn - 1) / bn, tiles_m = (q.M + bm - 1) / bm;
  const int nwg = tiles_n * tiles_m * splits;
  const int nt = gemm_tile_threads(bm, bn);
  hipLaunchKernelGGL(f, dim3(nwg), dim3(nt), 0, stream, q, tiles_n, tiles_m, nwg);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

}  // namespace dnn
