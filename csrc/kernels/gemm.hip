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
#include "gemm_tile.hpp"

namespace dnn {

// Accumulator fragments of the waves in epilogue chunk `chunk` -> fp32 [EPI_ROWS][CS_LD] LDS
// tile (C/D map: col = lane&15, row = 4*(lane>>4) + r).
template <class C>
__device__ __forceinline__ void acc_to_lds(const f32x4_t (&acc)[C::FM][C::FN],
                                           float LDS_AS* cs, int chunk, int wave, int lane) {
  const int wm = wave / C::WN, wn = wave % C::WN;
  if (wm / C::WPC != chunk) return;
  const int rbase = (wm % C::WPC) * C::SM;
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + i * 16 + (lane >> 4) * 4 + r;
        const int col = wn * C::SN + j * 16 + (lane & 15);
        cs[row * C::CS_LD + col] = acc[i][j][r];
      }
}

// Fused softmax cross-entropy over the fp32 logits tile in LDS (the whole padded row lives in
// this tile: N == BN; 4-wave tiles, one epilogue chunk). Thread r < BM owns row r: adds the
// bias, finds max / argmax (lowest index, np.argmax rule) / log-sum-exp over the n_cls valid
// columns, and overwrites the row with dz = (p - onehot) * scale (0 in padding columns and for
// label < 0 padding rows). Block loss and correct-count go to loss_part[tile_m] /
// correct[tile_m].
template <class C>
__device__ __forceinline__ void xent_rows(const GemmParams& p, float LDS_AS* cs, int m0) {
  static_assert(C::NW == 4 && C::CHUNKS == 1, "fused cross-entropy runs on 4-wave tiles");
  constexpr int BM = C::BM, BN = C::BN, CS_LD = C::CS_LD;
  // scratch after the staging tile (all LDS lives in the kernel's single __shared__ array)
  float LDS_AS* s_loss = cs + BM * CS_LD;
  int LDS_AS* s_corr = (int LDS_AS*)(s_loss + 4);
  const int r = threadIdx.x;
  float loss = 0.f;
  int corr = 0;
  if (r < BM) {
    float LDS_AS* row = cs + r * CS_LD;
    const int label = p.xent_labels[m0 + r];
    const int nc = p.n_cls;
    float mx = -INFINITY;
    int amax = 0;
    for (int c = 0; c < nc; ++c) {
      const float v = row[c] + p.bias[c];
      row[c] = v;
      if (v > mx) {
        mx = v;
        amax = c;
      }
    }
    float se = 0.f;
    for (int c = 0; c < nc; ++c) se += __expf(row[c] - mx);
    const float inv = 1.f / se;
    if (label >= 0) {
      loss = -(row[label] - mx - __logf(se));
      corr = amax == label;
      for (int c = 0; c < nc; ++c)
        row[c] = (__expf(row[c] - mx) * inv - (c == label ? 1.f : 0.f)) * p.xent_scale;
    } else {
      for (int c = 0; c < nc; ++c) row[c] = 0.f;
    }
    for (int c = nc; c < BN; ++c) row[c] = 0.f;
  }
  // block reduction of loss / correct (fixed order -> reproducible)
  loss = wave_sum(loss);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) corr += __shfl_xor(corr, o, 64);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_loss[wave] = loss;
    s_corr[wave] = corr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (p.loss_part) p.loss_part[m0 / BM] = (s_loss[0] + s_loss[1]) + (s_loss[2] + s_loss[3]);
    const int cc = s_corr[0] + s_corr[1] + s_corr[2] + s_corr[3];
    if (p.correct) p.correct[m0 / BM] = cc;
  }
}

template <class C, int LA, int LB, bool OUT_F32>
__global__ __launch_bounds__(C::NT) void gemm_bf16_kernel(GemmParams p, int tiles_n, int tiles_m,
                                                          int nwg) {
  constexpr int BM = C::BM, BN = C::BN, NT = C::NT, CS_LD = C::CS_LD;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  char LDS_AS* lds = (char LDS_AS*)smem;

  // XCD-aware bijective remap: hardware deals block b to XCD group b%8; give each group a
  // contiguous run of logical tiles. Within a split, tiles are walked in groups of
  // group_m row-tiles (column-major inside a group), so the ~32 workgroups an XCD holds at
  // once cover e.g. 4 row x 8 column tiles: 12 operand k-slices shared through its L2
  // instead of 33 for a 1 x 32 strip (guide §5.5 T1 + grouped raster order).
  const int wgid = xcd_remap(blockIdx.x, nwg);
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
  int kbase, nk;
  if (p.k_total > 0) {  // uneven split-K: split s takes k-steps [s*KS/S, (s+1)*KS/S)
    const int KS = p.k_total >> 6, S = nwg / (tiles_n * tiles_m);
    const int a = (int)((long)split * KS / S), b = (int)((long)(split + 1) * KS / S);
    kbase = a * 64;
    nk = b - a;
  } else {
    kbase = split * p.K;
    nk = p.K >> 6;
  }

  f32x4_t acc[C::FM][C::FN];
  mma_tile<C, LA, LB>(p, m0, n0, kbase, nk, lds, acc, wave, lane);

  // ---- epilogue: accumulators -> LDS (fp32, EPI_ROWS at a time) -> 16-B row chunks -----------
  float LDS_AS* cs = (float LDS_AS*)lds;
  constexpr int CPR = BN / 8;
  constexpr int ITER = C::EPI_ROWS * CPR / NT;
  constexpr int RSTEP = NT / CPR;  // rows between a thread's consecutive iterations
  // A thread's 8-column chunk is the same in every iteration and chunk (NT % CPR == 0): its
  // bias is loaded ONCE, and the per-row global reads of a chunk (activation for the dgrad
  // mask, previous slab for split-K accumulation) are all issued before the first is used --
  // one L2 round trip per chunk instead of one per row (the per-row form serialised ~16
  // round trips per 256x256 tile: half the tile's time at K = 832).
  const int ccol = (threadIdx.x % CPR) * 8, crow = threadIdx.x / CPR;
  const long gn = n0 + ccol;
  bool xent = false;
  if constexpr (!OUT_F32 && C::NW == 4 && C::CHUNKS == 1)
    xent = p.xent_labels != nullptr;  // uniform
  const bool col_ok = gn < p.N;  // partial edge tile: this thread's columns may be past N
  float bias_r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (p.bias && !xent && col_ok) {
    const f32x4_t b0 = *(const f32x4_t*)(p.bias + gn);
    const f32x4_t b1 = *(const f32x4_t*)(p.bias + gn + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bias_r[e] = b0[e];
      bias_r[e + 4] = b1[e];
    }
  }
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int chunk = 0; chunk < C::CHUNKS; ++chunk) {
    if (chunk) __syncthreads();  // previous chunk's stores have read the staging tile
    acc_to_lds<C>(acc, cs, chunk, wave, lane);
    __syncthreads();
    if constexpr (!OUT_F32 && C::NW == 4 && C::CHUNKS == 1) {
      if (xent) {  // fused softmax-CE, one thread per row of the tile
        xent_rows<C>(p, cs, m0);
        __syncthreads();
      }
    }
    const long gm0 = m0 + chunk * C::EPI_ROWS + crow;
    [[maybe_unused]] bf16x8_t yv[ITER];
    [[maybe_unused]] f32x4_t cp0[ITER], cp1[ITER];
    if constexpr (OUT_F32) {
      if (p.accumulate) {
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
          if (!col_ok || gm0 + it * RSTEP >= p.M) continue;
          const float* c = (const float*)p.C + (long)split * p.c_split_stride +
                           (gm0 + it * RSTEP) * p.ldc + gn;
          cp0[it] = *(const f32x4_t*)c;
          cp1[it] = *(const f32x4_t*)(c + 4);
        }
      }
    } else {
      if (p.aux && !xent) {
#pragma unroll
        for (int it = 0; it < ITER; ++it)
          if (col_ok && gm0 + it * RSTEP < p.M)
            yv[it] = *(const bf16x8_t*)(p.aux + (gm0 + it * RSTEP) * p.ld_aux + gn);
      }
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int row = crow + it * RSTEP;
      const f32x4_t v0 = *(const f32x4_t LDS_AS*)(cs + row * CS_LD + ccol);
      const f32x4_t v1 = *(const f32x4_t LDS_AS*)(cs + row * CS_LD + ccol + 4);
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const long gm = gm0 + it * RSTEP;
      if (!col_ok || gm >= p.M) continue;  // outside a partial edge tile: not stored
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bias_r[e];
      if constexpr (OUT_F32) {
        float* c = (float*)p.C + (long)split * p.c_split_stride + gm * p.ldc + gn;
        if (!p.accumulate && p.act != ACT_LINEAR) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = act_fwd(v[e], p.act);
        }
        f32x4_t o0 = {v[0], v[1], v[2], v[3]}, o1 = {v[4], v[5], v[6], v[7]};
        if (p.accumulate) {
          o0 += cp0[it];
          o1 += cp1[it];
        }
        *(f32x4_t*)c = o0;
        *(f32x4_t*)(c + 4) = o1;
      } else {
        if (xent) {
          // dz already computed in LDS
        } else if (p.aux) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = act_bwd(v[e], bf2f((u16)yv[it][e]), p.act);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = act_fwd(v[e], p.act);
        }
        bf16x8_t o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const u16 h = f2bf(v[e]);
          o[e] = (short)h;
          csum[e] += bf2f(h);
        }
        *(bf16x8_t*)((u16*)p.C + gm * p.ldc + gn) = o;
      }
    }
  }
  if constexpr (!OUT_F32) {
    if (p.colsum) {  // uniform across the block
      __syncthreads();  // all reads of the staging tile are done
      f32x4_t LDS_AS* red = (f32x4_t LDS_AS*)lds;
      red[2 * threadIdx.x] = f32x4_t{csum[0], csum[1], csum[2], csum[3]};
      red[2 * threadIdx.x + 1] = f32x4_t{csum[4], csum[5], csum[6], csum[7]};
      __syncthreads();
      if ((int)threadIdx.x < BN) {
        const int col = threadIdx.x, cc = col >> 3, e = col & 7;
        const float LDS_AS* rf = (const float LDS_AS*)lds;
        float t = 0.f;
#pragma unroll 4
        for (int r = 0; r < NT / CPR; ++r) t += rf[(r * CPR + cc) * 8 + e];
        if (n0 + col < p.N) p.colsum[(long)tm * p.ld_colsum + n0 + col] = t;
      }
    }
  }
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

// 4-wave tiles: any NS in 2..4; 8-wave tiles: NS = 2 (a third 64-KiB stage does not fit)
template <int BM, int BN>
static gemm_fn pick4(int ns, int la, int lb, int f32) {
  return ns == 2   ? pick_layout<Cfg<BM, BN, 2, 2, 2>>(la, lb, f32)
         : ns == 3 ? pick_layout<Cfg<BM, BN, 2, 2, 3>>(la, lb, f32)
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
    case -12: return "pipeline stages must be 2..4 (8-wave tiles: 2..3, 256x256: 2)";
    default: return "unknown gemm error";
  }
}

int default_stages(int bm, int bn) {
  (void)bm;
  (void)bn;
  return 2;
}

int gemm_bf16(const GemmParams& p, int la, int lb, int out_f32, int bm, int bn, int splits,
              hipStream_t stream, int stages, int persist) {
  if (!gemm_tile_supported(bm, bn)) return -1;
  // partial edge tiles: M and N need only be multiples of 8 (16-byte rows / chunks)
  if (p.M <= 0 || p.N <= 0 || p.M % 8 || p.N % 8) return -2;
  if (splits < 1) return -3;
  if (p.k_total > 0) {
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

  // (A 4-wave 256x256 form -- 128x128 per wave, one wave per SIMD, accumulators in AGPRs,
  // hipBLASLt's MT256x256 MIWT8_8 shape -- was built and measured: 7 % slower on 8192^3 fwd,
  // 20 % on K = 832, 3-4x on dgrad (spills); without hand-scheduled intra-wave pipelining one
  // wave per SIMD cannot hide LDS latency, so the 8-wave form is the 256x256 tile.)
  const int nt = gemm_tile_threads(bm, bn);
  const int ns = stages ? stages : default_stages(bm, bn);
  // 8-wave tiles: NS = 3 where three stages fit (not 256x256)
  if (ns < 2 || ns > 4 || (nt == 512 && (ns > 3 || (ns == 3 && bm == 256 && bn == 256))))
    return -12;
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
  else if (bm == 256 && bn == 256) fn = pick_layout<Cfg<256, 256, 4, 2, 2>>(la, lb, out_f32);
  else if (bm == 256 && bn == 128)
    fn = ns == 2 ? pick_layout<Cfg<256, 128, 4, 2, 2>>(la, lb, out_f32)
                 : pick_layout<Cfg<256, 128, 4, 2, 3>>(la, lb, out_f32);
  else if (bm == 256 && bn == 64)
    fn = ns == 2 ? pick_layout<Cfg<256, 64, 4, 2, 2>>(la, lb, out_f32)
                 : pick_layout<Cfg<256, 64, 4, 2, 3>>(la, lb, out_f32);
  else
    fn = ns == 2 ? pick_layout<Cfg<128, 256, 2, 4, 2>>(la, lb, out_f32)
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

}  // namespace dnn
