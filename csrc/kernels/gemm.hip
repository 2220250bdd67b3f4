// bf16 MFMA GEMM for gfx950 (MI355X) with fused training epilogues.
//
// Structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop"):
//   * 256 threads = 4 waves in a 2x2 grid, each wave owns a (BM/2)x(BN/2) output sub-tile built
//     from v_mfma_f32_16x16x32_bf16 fragments;
//   * BK = 64; A and B tiles are staged global->LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB
//     per wave-instruction) into two LDS buffers so the load of tile k+1 overlaps compute of k;
//   * LDS images are XOR-swizzled so fragment reads are bank-conflict free; because the LDS-DMA
//     destination is lane-linear, the swizzle is applied to the per-lane GLOBAL source address
//     and the same involution is applied on the read (guide §5.4 rule 21);
//   * contraction-contiguous tiles are read with ds_read_b128, output-dim-contiguous tiles with
//     the transposing ds_read_b64_tr_b16 (guide §5.5 T10) -- this is what lets dgrad and wgrad
//     consume W, dZ and X in their natural row-major layouts;
//   * the epilogue stages the fp32 accumulators through LDS and stores whole 16-byte row chunks,
//     fusing bias + activation (forward), activation-derivative masking from the stored
//     activation output (dgrad), or fp32 split-K slab accumulation (wgrad);
//   * workgroup ids are remapped so consecutive output tiles (sharing an A panel) land on the
//     same XCD / L2 (guide §5.5 T1, bijective form).
//
// Reference parity: replaces the per-stage NumPy `np.dot(x, W) + b` + activation of
// /root/reference/src/grpc_node.py:75-97 (forward) and adds the backward the reference only had
// centrally (/root/reference/scripts/generate_mnist_pytorch.py:41-52).
#include "gemm_kernel.hpp"

namespace dnn {

// Grouped launch: up to GEMM_GROUP_MAX independent problems with one tile configuration (e.g.
// every layer's weight gradient of a step) in ONE launch; problem j owns the workgroups
// [start[j], start[j] + nwg[j]) (start rounded to multiples of 8 so each problem keeps its
// XCD-aware raster). Small, latency-bound problems then fill each other's idle CUs.
template <class C, int LA, int LB, bool OUT_F32>
__global__ __launch_bounds__(C::NT) void gemm_group_kernel(GemmGroup g) {
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  int j = 0;
  while (j + 1 < g.n && (int)blockIdx.x >= g.start[j + 1]) ++j;
  const int bid = blockIdx.x - g.start[j];
  if (bid >= g.nwg[j]) return;  // padding to the next multiple of 8 (uniform per workgroup)
  gemm_tile_wg<C, LA, LB, OUT_F32>(g.p[j], g.tiles_n[j], g.tiles_m[j], g.nwg[j], bid,
                                   (char LDS_AS*)smem);
}

// ---- stream-K (balanced split-K) for batch-contraction GEMMs ---------------------------------
// The wgrad GEMMs have few output tiles (e.g. 52 for a 512x832 weight) and a huge contraction
// (the batch). Classic split-K leaves the chip unevenly loaded (416 workgroups = 2 on 160 CUs,
// 1 on 96). Here the flattened (tile, k-step) space of `total` iterations is cut into `nwg`
// contiguous, equal shares; a workgroup walks its share, emitting one fp32 partial tile per
// tile segment it touches (at most 2 when ipw <= k-steps per tile) into
// part[(wg * 2 + seg)][BM][BN]. streamk_reduce then sums each tile's contributors in
// workgroup order (deterministic) into C.
template <int BM, int BN, int LA, int LB>
__global__ __launch_bounds__(256) void gemm_bf16_streamk_kernel(GemmParams p, int tiles_n,
                                                                int ksteps, int ipw, int total,
                                                                int nwg, float* part) {
  using TC = Cfg<BM, BN, 2, 2, 2>;
  constexpr int FM = TC::FM, FN = TC::FN, CS_LD = TC::CS_LD;
  __shared__ __attribute__((aligned(16))) char smem[TC::SMEM];
  char LDS_AS* lds = (char LDS_AS*)smem;
  const int w = xcd_remap(blockIdx.x, nwg);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int it = w * ipw;
  const int it_end = min(total, it + ipw);
  for (int seg = 0; it < it_end; ++seg) {
    const int tile = it / ksteps, k0 = it % ksteps;
    const int k1 = min(ksteps, k0 + (it_end - it));
    const int tn = tile % tiles_n, tm = tile / tiles_n;
    f32x4_t acc[FM][FN];
    mma_tile<TC, LA, LB>(p, tm * BM, tn * BN, k0 * 64, k1 - k0, lds, acc, wave, lane);
    float LDS_AS* cs = (float LDS_AS*)lds;
    acc_to_lds<TC>(acc, cs, 0, wave, lane);
    __syncthreads();
    float* dst = part + ((long)w * 2 + seg) * (BM * BN);
    constexpr int C4 = BN / 4;
#pragma unroll 4
    for (int idx = threadIdx.x; idx < BM * C4; idx += 256) {
      const int row = idx / C4, col = (idx % C4) * 4;
      *(f32x4_t*)(dst + row * BN + col) = *(const f32x4_t LDS_AS*)(cs + row * CS_LD + col);
    }
    __syncthreads();  // LDS is re-staged by the next segment
    it += k1 - k0;
  }
}

// C[tile] (+)= sum of the tile's partials; one block per (tile, 1024-float chunk).
__global__ __launch_bounds__(256) void streamk_reduce_kernel(const float* __restrict__ part,
                                                             float* __restrict__ C, long ldc,
                                                             int bm, int bn, int tiles_n,
                                                             int ksteps, int ipw,
                                                             int accumulate) {
  const int tile = blockIdx.y;
  const int tn = tile % tiles_n, tm = tile / tiles_n;
  const int tile_elems = bm * bn;
  const int e = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (e >= tile_elems) return;
  const long first_it = (long)tile * ksteps, last_it = first_it + ksteps - 1;
  const int w0 = (int)(first_it / ipw), w1 = (int)(last_it / ipw);
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  for (int w = w0; w <= w1; ++w) {
    const int seg = ((long)w * ipw / ksteps == tile) ? 0 : 1;  // tile w started in -> seg 0
    s += *(const f32x4_t*)(part + ((long)w * 2 + seg) * tile_elems + e);
  }
  const int row = e / bn, col = e % bn;
  float* c = C + (long)(tm * bm + row) * ldc + tn * bn + col;
  if (accumulate) s += *(const f32x4_t*)c;
  *(f32x4_t*)c = s;
}

int gemm_bf16_streamk(const GemmParams& p, int layout_a, int layout_b, int bm, int bn, int nwg,
                      float* part, hipStream_t stream) {
  if (!((bm == 64 || bm == 128) && (bn == 64 || bn == 128))) return -1;
  if (p.M <= 0 || p.N <= 0 || p.M % bm || p.N % bn) return -2;
  if (p.K <= 0 || p.K % 64) return -3;
  if ((p.lda | p.ldb | p.ldc) % 4 || p.lda % 8 || p.ldb % 8) return -4;
  auto mis = [](const void* q) { return ((uintptr_t)q) & 15; };
  if (mis(p.A) || mis(p.B) || mis(p.C) || mis(part)) return -5;
  if ((layout_a != KMAJ && layout_a != MNMAJ) || (layout_b != KMAJ && layout_b != MNMAJ)) return -6;
  const int tiles_n = p.N / bn, tiles = tiles_n * (p.M / bm), ksteps = p.K / 64;
  const long total = (long)tiles * ksteps;
  if (nwg < tiles) nwg = tiles;  // guarantees ipw <= ksteps -> at most 2 segments per wg
  if (total > 0x7fffffff) return -3;
  const int ipw = (int)((total + nwg - 1) / nwg);
  nwg = (int)((total + ipw - 1) / ipw);
  typedef void (*fn_t)(GemmParams, int, int, int, int, int, float*);
  fn_t fn;
#define DNN_SK(BM_, BN_)                                                                     \
  fn = (layout_a == KMAJ ? (layout_b == KMAJ ? gemm_bf16_streamk_kernel<BM_, BN_, KMAJ, KMAJ>   \
                                             : gemm_bf16_streamk_kernel<BM_, BN_, KMAJ, MNMAJ>) \
                         : (layout_b == KMAJ ? gemm_bf16_streamk_kernel<BM_, BN_, MNMAJ, KMAJ>  \
                                             : gemm_bf16_streamk_kernel<BM_, BN_, MNMAJ, MNMAJ>))
  if (bm == 128 && bn == 128) DNN_SK(128, 128);
  else if (bm == 128) DNN_SK(128, 64);
  else if (bn == 128) DNN_SK(64, 128);
  else DNN_SK(64, 64);
#undef DNN_SK
  hipLaunchKernelGGL(fn, dim3(nwg), dim3(256), 0, stream, p, tiles_n, ksteps, ipw, (int)total,
                     nwg, part);
  if (hipGetLastError() != hipSuccess) return -9;
  const int chunks = (bm * bn / 4 + 255) / 256;
  hipLaunchKernelGGL(streamk_reduce_kernel, dim3(chunks, tiles), dim3(256), 0, stream, part,
                     (float*)p.C, p.ldc, bm, bn, tiles_n, ksteps, ipw, p.accumulate);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// 4-wave tiles: any NS in 2..4, or 5 = the asymmetric ring (A 3 deep, B 2 deep); 8-wave tiles:
// NS = 2, 3 where it fits, or 5 (256x256: 3 x 32 KiB A + 2 x 32 KiB B = all 160 KiB of LDS)
template <int BM, int BN>
static gemm_fn pick4(int ns, int la, int lb, int f32) {
  return ns == 2   ? pick_layout<Cfg<BM, BN, 2, 2, 2>>(la, lb, f32)
         : ns == 3 ? pick_layout<Cfg<BM, BN, 2, 2, 3>>(la, lb, f32)
         : ns == 5 ? pick_layout<Cfg<BM, BN, 2, 2, 3, 2>>(la, lb, f32)
                   : pick_layout<Cfg<BM, BN, 2, 2, 4>>(la, lb, f32);
}

bool gemm_tile_supported(int bm, int bn) {
  const bool small = (bm == 64 || bm == 128) && (bn == 64 || bn == 128);
  const bool big = (bm == 256 && (bn == 64 || bn == 128 || bn == 256)) || (bm == 128 && bn == 256);
  return small || big;
}

int gemm_tile_threads(int bm, int bn) { return bm == 256 || bn == 256 ? 512 : 256; }

const char* gemm_error_string(int code) {
  switch (code) {
    case 0: return "ok";
    case -1: return "unsupported tile (64|128 x 64|128, 256 x 64|128|256, 128 x 256)";
    case -2: return "M and N must be positive multiples of 8 (edge tiles are partial)";
    case -3: return "per-split K must be a positive multiple of 64";
    case -4: return "leading dimensions must be multiples of 8 elements (16-byte rows)";
    case -5: return "pointers must be 16-byte aligned";
    case -6: return "bad layout code";
    case -7: return "split-K > 1 requires fp32 output";
    case -8: return "leading dimension smaller than the row it stores";
    case -9: return "hip launch failed";
    case -10: return "colsum needs bf16 output and ld_colsum >= N";
    case -11: return "fused cross-entropy needs bf16 output, N == bn <= 128, a bias and 0 < n_cls <= N";
    case -13: return "relu bit masks need bf16 output, act = relu, ld_mask >= N/8 (or < 0: fragment order, stage codes 9 / 11), no aux/xent, one-tile form";
    case -12: return "pipeline stages must be 2..4, 5 = A3/B2 ring, 6 = register-prefetched 2-deep ring (staged epilogue), 9 = the same with the register-direct epilogue (no ct / fused update), 11 = register-direct epilogue on the A3/B2 ring (256x256, 256x128, 128x128) (8-wave tiles: 2, 3, 5; 256x256: 2, 5 or 8 = ping-pong; 5: one-tile form, no fused xent)";
    case -14: return "transposed output ct needs bf16 output (or the fused update), no xent, one split, one-tile form, ld_ct >= M, 16-byte alignment";
    case -15: return "fused SGD epilogue needs f32 output, one split, no accumulate/bias/xent, a device lr, 16-byte aligned buffers, N % 8 == 0, one-tile form";
    default: return "unknown gemm error";
  }
}

int default_stages(int bm, int bn) {
  (void)bm;
  (void)bn;
  return 2;
}

int gemm_check(const GemmParams& p, int la, int lb, int out_f32, int bm, int bn, int splits) {
  if (!gemm_tile_supported(bm, bn)) return -1;
  // partial edge tiles: M and N need only be multiples of 8 (16-byte rows / chunks)
  if (p.M <= 0 || p.N <= 0 || p.M % 8 || p.N % 8) return -2;
  if (splits < 1) return -3;
  if (p.k_total > 0) {  // uneven split-K ranges are cut in 64-deep units
    if (p.k_total % 64 || splits > p.k_total / 64) return -3;
  } else if (p.K <= 0 || p.K % 64) {
    return -3;
  }
  const long ktot = p.k_total > 0 ? (long)p.k_total : (long)p.K * splits;
  if ((p.lda | p.ldb | p.ldc) % 8 || (p.aux && p.ld_aux % 8)) return -4;
  auto mis = [](const void* q) { return ((uintptr_t)q) & 15; };
  if (mis(p.A) || mis(p.B) || mis(p.C) || (p.aux && mis(p.aux)) || (p.bias && mis(p.bias)))
    return -5;
  if ((la != KMAJ && la != MNMAJ) || (lb != KMAJ && lb != MNMAJ)) return -6;
  if (splits > 1 && !out_f32) return -7;
  if (p.colsum && (out_f32 || p.ld_colsum < p.N)) return -10;
  if (p.xent_labels && (out_f32 || p.N != bn || bn > 128 || bm > 128 || p.M % bm || !p.bias ||
                        p.n_cls <= 0 || p.n_cls > p.N || splits != 1 || p.aux))
    return -11;
  const long a_row = la == KMAJ ? ktot : p.M;
  const long b_row = lb == KMAJ ? ktot : p.N;
  if (p.lda < a_row || p.ldb < b_row || p.ldc < p.N || (p.aux && p.ld_aux < p.N)) return -8;
  if (p.ct && ((out_f32 && !p.upd_master) || p.xent_labels || splits != 1 || p.ld_ct < p.M ||
               p.ld_ct % 8 || ((uintptr_t)p.ct & 15)))
    return -14;
  // fused SGD epilogue: the f32 weight gradient of ONE split is consumed in place
  if (p.upd_master && (!out_f32 || splits != 1 || p.accumulate || p.bias || p.xent_labels ||
                       !p.upd_lr || mis(p.upd_master) || (p.upd_mom && mis(p.upd_mom)) ||
                       (p.upd_shadow && ((uintptr_t)p.upd_shadow & 15)) || p.N % 8))
    return -15;
  if ((p.mask_out || p.mask_in) &&
      (out_f32 || p.act != ACT_RELU || (p.mask_in && p.aux) || (p.mask_out && p.mask_in) ||
       p.xent_labels || (p.ld_mask >= 0 && p.ld_mask < (p.N + 7) / 8)))
    return -13;
  return 0;
}

int gemm_bf16(const GemmParams& p, int la, int lb, int out_f32, int bm, int bn, int splits,
              hipStream_t stream, int stages, int persist) {
  const int rc = gemm_check(p, la, lb, out_f32, bm, bn, splits);
  if (rc) return rc;
  if ((p.mask_out || p.mask_in) && persist) return -13;
  // fragment-order masks (ld_mask < 0) exist only in the register-direct epilogue
  const bool direct = stages == 9 || stages == 11;
  if ((p.mask_out || p.mask_in) && p.ld_mask < 0 && !direct) return -13;
  if (p.ct && persist) return -14;
  if (p.upd_master && persist) return -15;

  // (A 4-wave 256x256 form -- 128x128 per wave, one wave per SIMD, accumulators in AGPRs,
  // hipBLASLt's MT256x256 MIWT8_8 shape -- was built and measured: 7 % slower on 8192^3 fwd,
  // 20 % on K = 832, 3-4x on dgrad (spills); without hand-scheduled intra-wave pipelining one
  // wave per SIMD cannot hide LDS latency, so the 8-wave form is the 256x256 tile. Round 5
  // re-measured it on the register-prefetched loop (stage code 13, bitwise equal to code 11):
  // 6-43 % slower on every BASELINE GEMM, wgrad included, whose loop compiles clean; the
  // K-major loops also shuffle accumulators between VGPRs and AGPRs -- 256 AGPRs of
  // accumulators leave the allocator no spare. profiles/r5_blas/code13_*.)
  if (stages == 8) {  // ping-pong half-tile-streamed form (gemm_pp.hip)
    if (bm != 256 || bn != 256) return -12;
    if (p.xent_labels) return -11;
    GemmParams q = p;
    if (q.group_m <= 0) q.group_m = ((p.N + 255) / 256) >= 8 ? 4 : 1;
    return gemm_pp_launch(q, la, lb, out_f32, splits, stream);
  }
  const int nt = gemm_tile_threads(bm, bn);
  const int ns = stages ? stages : default_stages(bm, bn);
  if (ns == 6 || ns == 9 || ns == 11) {  // register-prefetched loop
    if (persist || p.xent_labels) return -12;
    if (ns >= 9) {  // register-direct epilogue (9, 11): no transposed copy / fused update
      if (p.ct) return -14;
      if (p.upd_master) return -15;
    }
    GemmParams q = p;
    if (q.group_m <= 0) q.group_m = ((p.N + bn - 1) / bn) >= 8 ? 4 : 1;
    return gemm_rp_launch(q, la, lb, out_f32, bm, bn, splits, ns, stream);
  }
  // 8-wave tiles: NS = 3 where three stages fit (not 256x256); 5 = asymmetric A3/B2 ring
  if (ns < 2 || ns > 5 || (nt == 512 && (ns == 4 || (ns == 3 && bm == 256 && bn == 256))))
    return -12;
  if (ns == 5 && (persist || p.xent_labels)) return -12;
  if (persist && !p.xent_labels) {  // persistent form (gemm_persist.hip); NS <= 3
    if (ns > 3) return -12;
    GemmParams q = p;
    if (q.group_m <= 0) q.group_m = ((p.N + bn - 1) / bn) >= 8 ? 4 : 1;
    return gemm_persist_launch(q, la, lb, out_f32, bm, bn, splits, ns, persist, stream);
  }
  gemm_fn fn;
  if (bm == 128 && bn == 128) fn = pick4<128, 128>(ns, la, lb, out_f32);
  else if (bm == 128 && bn == 64) fn = pick4<128, 64>(ns, la, lb, out_f32);
  else if (bm == 64 && bn == 128) fn = pick4<64, 128>(ns, la, lb, out_f32);
  else if (bm == 64 && bn == 64) fn = pick4<64, 64>(ns, la, lb, out_f32);
  else if (bm == 256 && bn == 256)
    fn = ns == 5 ? pick_layout<Cfg<256, 256, 4, 2, 3, 2>>(la, lb, out_f32)
                 : pick_layout<Cfg<256, 256, 4, 2, 2>>(la, lb, out_f32);
  else if (bm == 256 && bn == 128)
    fn = ns == 2   ? pick_layout<Cfg<256, 128, 4, 2, 2>>(la, lb, out_f32)
         : ns == 5 ? pick_layout<Cfg<256, 128, 4, 2, 3, 2>>(la, lb, out_f32)
                   : pick_layout<Cfg<256, 128, 4, 2, 3>>(la, lb, out_f32);
  else if (bm == 256 && bn == 64)
    fn = ns == 2   ? pick_layout<Cfg<256, 64, 4, 2, 2>>(la, lb, out_f32)
         : ns == 5 ? pick_layout<Cfg<256, 64, 4, 2, 3, 2>>(la, lb, out_f32)
                   : pick_layout<Cfg<256, 64, 4, 2, 3>>(la, lb, out_f32);
  else
    fn = ns == 2   ? pick_layout<Cfg<128, 256, 2, 4, 2>>(la, lb, out_f32)
         : ns == 5 ? pick_layout<Cfg<128, 256, 2, 4, 3, 2>>(la, lb, out_f32)
                   : pick_layout<Cfg<128, 256, 2, 4, 3>>(la, lb, out_f32);

  const int tiles_n = (p.N + bn - 1) / bn, tiles_m = (p.M + bm - 1) / bm;
  const int nwg = tiles_n * tiles_m * splits;
  GemmParams q = p;
  // grouped raster (see the kernel): worth it once a row of column tiles outgrows what one
  // XCD holds at a time; a caller-provided group_m wins
  if (q.group_m <= 0) q.group_m = tiles_n >= 8 ? 4 : 1;
  hipLaunchKernelGGL(fn, dim3(nwg), dim3(nt), 0, stream, q, tiles_n, tiles_m, nwg);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int gemm_bf16_group(const GemmParams* ps, const int* splits, int n, int la, int lb, int out_f32,
                    int bm, int bn, int stages, hipStream_t stream) {
  if (n <= 0 || n > GEMM_GROUP_MAX) return -1;
  if (gemm_tile_threads(bm, bn) != 256 || (stages && stages != 2)) return -12;
  GemmGroup g{};
  g.n = n;
  int blocks = 0;
  for (int j = 0; j < n; ++j) {
    // the one-problem validation (shapes, alignment, layouts, epilogue combinations)
    const int rc = gemm_check(ps[j], la, lb, out_f32, bm, bn, splits[j]);
    if (rc) return rc;
    if ((ps[j].mask_out || ps[j].mask_in) && ps[j].ld_mask < 0) return -13;
    g.p[j] = ps[j];
    g.tiles_n[j] = (ps[j].N + bn - 1) / bn;
    g.tiles_m[j] = (ps[j].M + bm - 1) / bm;
    g.nwg[j] = g.tiles_n[j] * g.tiles_m[j] * splits[j];
    if (g.p[j].group_m <= 0) g.p[j].group_m = g.tiles_n[j] >= 8 ? 4 : 1;
    g.start[j] = blocks;
    blocks += (g.nwg[j] + 7) / 8 * 8;
  }
  g.start[n] = blocks;
  typedef void (*fn_t)(GemmGroup);
  fn_t fn = nullptr;
#define DNN_GG(BM, BN)                                                                     \
  if (bm == BM && bn == BN) {                                                              \
    using C = Cfg<BM, BN, 2, 2, 2>;                                                        \
    if (la == KMAJ && lb == KMAJ)                                                          \
      fn = out_f32 ? gemm_group_kernel<C, KMAJ, KMAJ, true> : gemm_group_kernel<C, KMAJ, KMAJ, false>; \
    else if (la == KMAJ && lb == MNMAJ)                                                    \
      fn = out_f32 ? gemm_group_kernel<C, KMAJ, MNMAJ, true> : gemm_group_kernel<C, KMAJ, MNMAJ, false>; \
    else if (la == MNMAJ && lb == MNMAJ && out_f32)                                        \
      fn = gemm_group_kernel<C, MNMAJ, MNMAJ, true>;                                       \
  }
  DNN_GG(64, 64)
  DNN_GG(64, 128)
  DNN_GG(128, 64)
  DNN_GG(128, 128)
#undef DNN_GG
  if (!fn) return -6;
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, stream, g);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

}  // namespace dnn
