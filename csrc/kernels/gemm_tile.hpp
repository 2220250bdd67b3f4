// Shared building blocks of the gfx950 bf16 MFMA GEMM kernels (gemm.hip: one tile per
// workgroup, LDS-staged epilogue; gemm_persist.hip: persistent workgroups, direct epilogue).
// See gemm.hip for the structure of the main loop.
#pragma once
#include "common.hpp"
#include "gemm.hpp"

namespace dnn {

// ---- LDS image swizzles -------------------------------------------------------------------
// KMAJ image: [rows = BM or BN][64 k] bf16, 128-B rows of 8 16-B chunks; chunk' = c ^ ((r>>1)&7).
// The 16 rows a ds_read_b128 lane group touches then cover all 16 slots of the 256-B bank row.
__device__ __forceinline__ int k_swz(int r) { return (r >> 1) & 7; }

// MNMAJ image: [64 k-rows][T cols] bf16 (T*2-byte rows). A transposed read by one 32-lane half
// touches 8 k-rows x 32 B; the XOR (always even, so 32-B column pairs stay together) spreads the
// 8 rows over distinct 32-B bank positions. For T >= 128 a row spans >= one 256-B bank row, so
// the T = 128 pattern serves T = 256 too (the XOR only flips chunk bits 1..3).
template <int T>
__device__ __forceinline__ int mn_swz(int r) {
  static_assert(T == 64 || T == 128 || T == 256, "MNMAJ tile width");
  if constexpr (T == 64) return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1;
  return ((r & 3) | (((r >> 3) & 1) << 2)) << 1;
}

// ---- tile configurations ----------------------------------------------------------------------
// BM x BN output tile computed by WM x WN waves (NT = 64*WM*WN threads), each wave owning an
// (BM/WM) x (BN/WN) sub-tile of 16x16 MFMA fragments; NS = LDS pipeline stages (NS-1 tiles in
// flight while one is consumed). 4-wave tiles (<= 128x128) run 2..4 per CU; the 8-wave 256-row
// /-column tiles halve the bytes staged into LDS per FLOP (the GEMMs of this engine are bound
// by the global->LDS fill rate, see profiles/) at one workgroup per CU.
template <int A, int B>
struct cmax {
  static constexpr int v = A > B ? A : B;
};

template <int BM_, int BN_, int WM_, int WN_, int NS_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NS = NS_;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int SM = BM / WM, SN = BN / WN, FM = SM / 16, FN = SN / 16;
  static constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  // LDS-DMA instructions one wave issues per stage (A + B): the vmcnt unit of the pipeline
  static constexpr int PER_STAGE = (BM + BN) / (8 * NW);
  // epilogue: fp32 staging of EPI_ROWS rows at a time (whole tile when it fits)
  static constexpr int CS_LD = BN + 4;
  static constexpr int EPI_ROWS = (NW == 4 && BM <= 128) ? BM : SM;
  static constexpr int CHUNKS = BM / EPI_ROWS, WPC = EPI_ROWS / SM;  // wave-rows per chunk
  static constexpr int CS_BYTES = EPI_ROWS * CS_LD * 4;
  static constexpr int RED_BYTES = NT * 32;  // colsum partial staging
  static constexpr int SMEM = cmax<cmax<NS * STAGE, CS_BYTES + 64>::v, RED_BYTES>::v;
  static_assert(FM >= 1 && FN >= 1 && SM % 16 == 0 && SN % 16 == 0, "wave sub-tile");
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "LDS-DMA pieces per wave");
  static_assert(NT % (BN / 8) == 0 && (EPI_ROWS * (BN / 8)) % NT == 0, "epilogue mapping");
  static_assert(SMEM <= 160 * 1024, "LDS budget");
};

// Stage one operand tile (T entries of the M/N dim x 64 of K) into LDS with LDS-DMA.
// Tile bytes = T*128 = T/8 KiB pieces; each of the NW waves issues T/(8*NW) of them.
// Rows / columns at or past `mn_lim` (a partial edge tile) are clamped onto the last valid
// row / 8-column chunk: the loads stay in bounds, and the outputs they feed are never stored.
template <int L, int T, int NW>
__device__ __forceinline__ void stage_tile(const u16* __restrict__ g, long ld, int mn0, int k0,
                                           char LDS_AS* dst, int wave, int lane, int mn_lim) {
  constexpr int NI = T / (8 * NW);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int piece = i * NW + wave;
    const int chunk = piece * 64 + lane;
    const u16* src;
    if constexpr (L == KMAJ) {
      const int r = chunk >> 3, ph = chunk & 7;
      const int c = ph ^ k_swz(r);
      src = g + (long)min(mn0 + r, mn_lim - 1) * ld + k0 + c * 8;
    } else {
      constexpr int CPR = T / 8;
      const int r = chunk / CPR, ph = chunk % CPR;
      const int c = ph ^ mn_swz<T>(r);
      src = g + (long)(k0 + r) * ld + min(mn0 + c * 8, mn_lim - 8);
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (void LDS_AS*)(dst + piece * 1024), 16, 0, 0);
  }
}

// Fragment of v_mfma_f32_16x16x32_bf16 for 16-wide block `blk` of the tile and k-step s (32 k):
// lane l holds X[idx = l&15][k = 8*(l>>4) + j], j = 0..7 (guide §3 operand maps). The same form
// serves A (idx = row m) and B (idx = column n).
template <int L, int T>
__device__ __forceinline__ bf16x8_t load_frag(const char LDS_AS* tile, int blk, int s, int lane) {
  if constexpr (L == KMAJ) {
    const int r = blk * 16 + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    return *(const bf16x8_t LDS_AS*)(tile + r * 128 + ((c ^ k_swz(r)) << 4));
  } else {
    constexpr int RB = T * 2;
    const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
    const int ch = 2 * blk + (p >> 1);
    const int r0 = 32 * s + 8 * g + q;
    const int r1 = r0 + 4;
    bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (bf16x4_t LDS_AS*)(tile + r0 * RB + ((ch ^ mn_swz<T>(r0)) << 4) + 8 * (p & 1)));
    bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (bf16x4_t LDS_AS*)(tile + r1 * RB + ((ch ^ mn_swz<T>(r1)) << 4) + 8 * (p & 1)));
    bf16x8_t f;
    f.lo = lo;
    f.hi = hi;
    return f;
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Workgroup barrier WITHOUT the release fence of __syncthreads(): that fence waits for
// vmcnt(0), i.e. for every LDS-DMA load in flight, which would serialise the pipeline. LDS
// hazards are handled explicitly instead: own ds_reads done (lgkmcnt(0)) + own LDS-DMA tile
// landed (wait_stage) before the barrier. The "memory" clobber keeps the compiler from moving
// LDS accesses across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Wait until at most `after` (0 .. NS-2, runtime) later stages are still in flight.
template <int NS, int PS>
__device__ __forceinline__ void wait_stage(int after) {
  if constexpr (NS >= 4) {
    if (after >= 2) {
      wait_vmcnt<2 * PS>();
      return;
    }
  }
  if constexpr (NS >= 3) {
    if (after >= 1) {
      wait_vmcnt<PS>();
      return;
    }
  }
  wait_vmcnt<0>();
}

// acc (+)= A[m0:m0+BM, k] . B[k, n0:n0+BN] over k-steps [kbase, kbase + 64*nk) with an
// NS-deep LDS-DMA ring and ONE barrier per 64-deep k-step:
//   top of step kt: own loads of tile kt landed (vmcnt) -> barrier (everyone's landed, and
//   everyone finished step kt-1, so its buffer is free) -> issue tile kt+NS-1 into that
//   buffer -> MFMA on tile kt.
// acc is zeroed first; ends with every wave past a barrier, so the caller may reuse the LDS.
template <class C, int LA, int LB>
__device__ __forceinline__ void mma_tile(const GemmParams& p, int m0, int n0, int kbase, int nk,
                                         char LDS_AS* lds, f32x4_t (&acc)[C::FM][C::FN],
                                         int wave, int lane) {
  constexpr int FM = C::FM, FN = C::FN, A_BYTES = C::A_BYTES, STAGE = C::STAGE, NS = C::NS;
  const int wm = wave / C::WN, wn = wave % C::WN;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    if (s < nk) {
      stage_tile<LA, C::BM, C::NW>(p.A, p.lda, m0, kbase + s * 64, lds + s * STAGE, wave, lane,
                                   p.M);
      stage_tile<LB, C::BN, C::NW>(p.B, p.ldb, n0, kbase + s * 64, lds + s * STAGE + A_BYTES,
                                   wave, lane, p.N);
    }
  }
  int rd = 0, wr = NS - 1;  // ring slots of tile kt and of tile kt + NS - 1
  for (int kt = 0; kt < nk; ++kt) {
    wait_stage<NS, C::PER_STAGE>(min(nk - 1 - kt, NS - 2));
    lds_barrier();
    if (kt + NS - 1 < nk) {
      char LDS_AS* nxt = lds + wr * STAGE;
      const int k0 = kbase + (kt + NS - 1) * 64;
      stage_tile<LA, C::BM, C::NW>(p.A, p.lda, m0, k0, nxt, wave, lane, p.M);
      stage_tile<LB, C::BN, C::NW>(p.B, p.ldb, n0, k0, nxt + A_BYTES, wave, lane, p.N);
    }
    const char LDS_AS* sa = lds + rd * STAGE;
    const char LDS_AS* sb = sa + A_BYTES;
    // (Reading both 32-deep halves' fragments up front behind a sched_barrier was measured:
    // +8 % on 128x128 big GEMMs, -35 % on 256x256 dgrad whose 40 transposed reads exceed what
    // lgkmcnt can count -- the compiler's own interleaving is kept.)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = load_frag<LA, C::BM>(sa, wm * FM + i, s, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = load_frag<LB, C::BN>(sb, wn * FN + j, s, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    rd = rd + 1 == NS ? 0 : rd + 1;
    wr = wr + 1 == NS ? 0 : wr + 1;
  }
  __syncthreads();
}

}  // namespace dnn
