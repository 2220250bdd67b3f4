// One-tile GEMM kernel template (gemm_tile_wg / gemm_bf16_kernel) and its layout dispatch,
// shared by the translation units that instantiate main-loop variants (gemm.hip, gemm_rp.hip).
#pragma once
#include "gemm_tile.hpp"

namespace dnn {

// One output tile (workgroup `bid` of a launch of nwg = tiles * splits workgroups).
template <class C, int LA, int LB, bool OUT_F32>
__device__ __forceinline__ void gemm_tile_wg(const GemmParams& p, int tiles_n, int tiles_m,
                                             int nwg, int bid, char LDS_AS* lds) {
  constexpr int BM = C::BM, BN = C::BN;

  // XCD-aware bijective remap: hardware deals block b to XCD group b%8; give each group a
  // contiguous run of logical tiles. Within a split, tiles are walked in groups of
  // group_m row-tiles (column-major inside a group), so the ~32 workgroups an XCD holds at
  // once cover e.g. 4 row x 8 column tiles: 12 operand k-slices shared through its L2
  // instead of 33 for a 1 x 32 strip (guide §5.5 T1 + grouped raster order).
  const int wgid = xcd_remap(bid, nwg);
  const int per_split = tiles_n * tiles_m;
  const int split = wgid / per_split;
  const int t = wgid - split * per_split;
  const int gm_full = p.group_m > 1 ? p.group_m : 1;
  const int per_group = gm_full * tiles_n;
  const int grp = t / per_group, first_m = grp * gm_full;
  const int gm = min(tiles_m - first_m, gm_full);
  const int tin = t - grp * per_group;
  const int tm = first_m + tin % gm;
  const int tn = tin / gm;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m0 = tm * BM, n0 = tn * BN;
  int kbase, nk;  // nk in k-steps of C::BK (split ranges stay in 64-deep units)
  if (p.k_total > 0) {  // uneven split-K: split s takes k-steps [s*KS/S, (s+1)*KS/S)
    const int KS = p.k_total >> 6, S = nwg / (tiles_n * tiles_m);
    const int a = (int)((long)split * KS / S), b = (int)((long)(split + 1) * KS / S);
    kbase = a * 64;
    nk = (b - a) * (64 / C::BK);
  } else {
    kbase = split * p.K;
    nk = p.K / C::BK;
  }

  tl_mark(p, 0);
  f32x4_t acc[C::FM][C::FN];
  mma_tile<C, LA, LB>(p, m0, n0, kbase, nk, lds, acc, wave, lane);
  tl_mark(p, 2);

  if constexpr (C::DIRECT) {  // register-direct stores (colsum partials in ring slot 0)
    epilogue_direct<C::FM, C::FN, BN, C::SN, C::WM, C::NS, C::STAGE, OUT_F32>(
        p, acc, lds, 1, tm, tn, split, wave / C::WN, wave % C::WN, lane, true);
  } else {
    epilogue_staged<C, OUT_F32>(p, acc, lds, m0, n0, tm, split, wave, lane);
  }
  tl_mark(p, 3);
}

template <class C, int LA, int LB, bool OUT_F32>
__global__ __launch_bounds__(C::NT) void gemm_bf16_kernel(GemmParams p, int tiles_n, int tiles_m,
                                                          int nwg) {
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  gemm_tile_wg<C, LA, LB, OUT_F32>(p, tiles_n, tiles_m, nwg, blockIdx.x, (char LDS_AS*)smem);
}

typedef void (*gemm_fn)(GemmParams, int, int, int);

template <class C>
static gemm_fn pick_layout(int la, int lb, int f32) {
#define DNN_G(LA, LB, F) gemm_bf16_kernel<C, LA, LB, F>
  if (la == KMAJ && lb == KMAJ) return f32 ? DNN_G(KMAJ, KMAJ, true) : DNN_G(KMAJ, KMAJ, false);
  if (la == KMAJ && lb == MNMAJ) return f32 ? DNN_G(KMAJ, MNMAJ, true) : DNN_G(KMAJ, MNMAJ, false);
  if (la == MNMAJ && lb == KMAJ) return f32 ? DNN_G(MNMAJ, KMAJ, true) : DNN_G(MNMAJ, KMAJ, false);
  return f32 ? DNN_G(MNMAJ, MNMAJ, true) : DNN_G(MNMAJ, MNMAJ, false);
#undef DNN_G
}

}  // namespace dnn
