// Register-prefetched main-loop variants of the one-tile GEMM (stage codes 6 / 7; Cfg RP,
// mma_tile_rp in gemm_tile.hpp), in a translation unit of their own so the build compiles
// them in parallel with gemm.hip.
#include "gemm_kernel.hpp"

namespace dnn {

// Stage codes 6 / 7: the register-prefetched main loop (Cfg RP, mma_tile_rp) with a 2- / 3-deep
// ring; 3 deep only where three 64-deep stages fit (not 256x256).
// Code 11: register-direct epilogue over the asymmetric ring (A 3 deep, B 2 deep: two k-steps
// for the streamed A panel to land), 256x256 / 256x128 / 128x128.
// Codes 9 / 10: the same loop with swapped MFMA operands and the register-direct epilogue
// (RP_ = 2): bias / activation / aux derivative / colsum / split-K f32, ReLU bit masks (both
// layouts, fragment order only here), no
// transposed copy, fused update or cross-entropy.
// Codes 15 / 16: code 9 (2-deep ring, register-direct epilogue) with the L2 touch-prefetch
// (Cfg TOUCH, touch_tiles) one / two k-steps beyond the ring; code 17: code 11 (A3/B2 ring)
// with touch distance 1 (256x128, 128x128).
static gemm_fn pick_rp(int bm, int bn, int code, int la, int lb, int f32) {
  if (code == 15 || code == 16 || code == 17) {
    constexpr int T1 = 2 | (1 << 4), T2 = 2 | (2 << 4);
#define DNN_RPT(BM, BN, WM, WN, NS, NSB, RPV) pick_layout<Cfg<BM, BN, WM, WN, NS, NSB, 64, RPV>>(la, lb, f32)
    if (code == 17) {
      // (256x256 A3/B2 fills all 160 KiB: no room for the touch scratch)
      if (bm == 256 && bn == 128) return DNN_RPT(256, 128, 4, 2, 3, 2, T1);
      if (bm == 128 && bn == 128) return DNN_RPT(128, 128, 2, 2, 3, 2, T1);
      return nullptr;
    }
    if (bm == 256 && bn == 256) return code == 15 ? DNN_RPT(256, 256, 4, 2, 2, 2, T1) : DNN_RPT(256, 256, 4, 2, 2, 2, T2);
    if (bm == 256 && bn == 128) return code == 15 ? DNN_RPT(256, 128, 4, 2, 2, 2, T1) : DNN_RPT(256, 128, 4, 2, 2, 2, T2);
    if (bm == 128 && bn == 128) return code == 15 ? DNN_RPT(128, 128, 2, 2, 2, 2, T1) : DNN_RPT(128, 128, 2, 2, 2, 2, T2);
    if (bm == 64 && bn == 64) return code == 15 ? DNN_RPT(64, 64, 2, 2, 2, 2, T1) : DNN_RPT(64, 64, 2, 2, 2, 2, T2);
#undef DNN_RPT
    return nullptr;
  }
  if (code == 11) {  // asymmetric A3/B2 ring, register-direct epilogue
#define DNN_RPA(BM, BN, WM, WN) pick_layout<Cfg<BM, BN, WM, WN, 3, 2, 64, 2>>(la, lb, f32)
    if (bm == 256 && bn == 256) return DNN_RPA(256, 256, 4, 2);
    if (bm == 256 && bn == 128) return DNN_RPA(256, 128, 4, 2);
    if (bm == 128 && bn == 128) return DNN_RPA(128, 128, 2, 2);
#undef DNN_RPA
    return nullptr;
  }
  const int ns = code == 6 || code == 9 ? 6 : 7;
  if (code == 9 || code == 10) {
#define DNN_RP(BM, BN, WM, WN, NS) pick_layout<Cfg<BM, BN, WM, WN, NS, NS, 64, 2>>(la, lb, f32)
    if (bm == 256 && bn == 256) return ns == 6 ? DNN_RP(256, 256, 4, 2, 2) : nullptr;
    if (bm == 256 && bn == 128) return ns == 6 ? DNN_RP(256, 128, 4, 2, 2) : DNN_RP(256, 128, 4, 2, 3);
    if (bm == 128 && bn == 128) return ns == 6 ? DNN_RP(128, 128, 2, 2, 2) : DNN_RP(128, 128, 2, 2, 3);
    if (bm == 128 && bn == 64) return ns == 6 ? DNN_RP(128, 64, 2, 2, 2) : DNN_RP(128, 64, 2, 2, 3);
    if (bm == 64 && bn == 64) return ns == 6 ? DNN_RP(64, 64, 2, 2, 2) : DNN_RP(64, 64, 2, 2, 3);
#undef DNN_RP
    return nullptr;
  }
#define DNN_RP(BM, BN, WM, WN, NS) pick_layout<Cfg<BM, BN, WM, WN, NS, NS, 64, 1>>(la, lb, f32)
  if (bm == 256 && bn == 256) return ns == 6 ? DNN_RP(256, 256, 4, 2, 2) : nullptr;
  if (bm == 256 && bn == 128) return ns == 6 ? DNN_RP(256, 128, 4, 2, 2) : DNN_RP(256, 128, 4, 2, 3);
  if (bm == 128 && bn == 128) return ns == 6 ? DNN_RP(128, 128, 2, 2, 2) : DNN_RP(128, 128, 2, 2, 3);
  if (bm == 128 && bn == 64) return ns == 6 ? DNN_RP(128, 64, 2, 2, 2) : DNN_RP(128, 64, 2, 2, 3);
  if (bm == 64 && bn == 64) return ns == 6 ? DNN_RP(64, 64, 2, 2, 2) : DNN_RP(64, 64, 2, 2, 3);
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
