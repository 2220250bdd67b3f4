// Shared building blocks of the gfx950 bf16 MFMA GEMM kernels (gemm.hip: one tile per
// workgroup, LDS-staged epilogue; gemm_persist.hip: persistent workgroups, direct epilogue).
// See gemm.hip for the structure of the main loop.
#pragma once
#include <type_traits>
#include "common.hpp"
#include "gemm.hpp"

namespace dnn {

// ---- LDS image swizzles -------------------------------------------------------------------
// KMAJ image: [rows = BM or BN][BK k] bf16. BK = 64: 128-B rows of 8 16-B chunks, chunk' =
// c ^ ((r>>1)&7); BK = 32: 64-B rows of 4 chunks, chunk' = c ^ ((r>>2)&3). Either way the 16
// rows a ds_read_b128 lane group touches cover all 16 slots of the 256-B bank row.
template <int BK = 64>
__device__ __forceinline__ int k_swz(int r) {
  static_assert(BK == 64 || BK == 32, "k-step depth");
  if constexpr (BK == 64) return (r >> 1) & 7;
  return (r >> 2) & 3;
}

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

//
// NSB_ (default NS_): a B ring of its own depth. NS = 3, NSB = 2 keeps TWO A tiles in flight
// behind the one being consumed and one B tile: the A operand of the forward / dgrad is the
// streamed activation panel (HBM), B the weights (L2-resident after the first tiles), and what
// limits those GEMMs is HBM bytes in flight per CU (profiles/r3_pmc: waves parked in vmcnt
// waits 47-63 % of their cycles), not LDS. Only that asymmetric pair is implemented.
//
// BK_ (default 64): contraction depth of one k-step / LDS stage. BK = 32 halves every stage, so a
// 2-stage 256x256 ring is 64 KiB and TWO such workgroups share a CU: one's prologue / epilogue
// runs beside the other's main loop, and 4 MFMA-issuing waves per SIMD instead of 2 hide the
// load latency -- at the price of a barrier per 32 k instead of per 64.
//
// RP_ (default 0): register-prefetched k-step (mma_tile_rp): fragments of the next 32-deep half
// are read while the MFMAs of the current one run, and the ring barrier sits between the two
// halves of a k-step instead of in front of a fragment read that every wave then waits for.
// RP_ = 2 also swaps the MFMA operands (a lane's accumulator fragment = 4 consecutive output
// columns of one row) so the tile is stored by the register-direct epilogue (epilogue_direct)
// instead of being staged through LDS: measured 11 us of a 256x256 bf16 tile's ~32 us was the
// staged epilogue (bench/probes/gemm_timeline.py), latency-bound even on an idle chip.
template <int BM_, int BN_, int WM_, int WN_, int NS_, int NSB_ = NS_, int BK_ = 64, int RP_ = 0>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NS = NS_, NSB = NSB_, BK = BK_;
  // RP_ bits 0-1: 1 = staged epilogue, 2 = register-direct; bits 2+: fragment-read placement
  // in each half (0 = one read per NM/NR MFMAs, 1 = two reads per MFMA up front, 2 = all reads
  // first)
  static constexpr bool RP = RP_ != 0, DIRECT = (RP_ & 3) == 2;
  static constexpr int RP_PATTERN = (RP_ >> 2) & 3;
  static_assert(!RP || (BK == 64 && NS <= 3), "register prefetch: BK 64, NS 2..3 (or A3/B2)");
  static_assert(NSB == NS || (NS == 3 && NSB == 2), "asymmetric ring: A 3 deep, B 2 deep only");
  static_assert(BK == 64 || BK == 32, "k-step depth 64 or 32");
  static constexpr bool ASYM = NSB != NS;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int SM = BM / WM, SN = BN / WN, FM = SM / 16, FN = SN / 16;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  // asymmetric ring layout: [NS A slots][NSB B slots]
  static constexpr int RING = ASYM ? NS * A_BYTES + NSB * B_BYTES : NS * STAGE;
  // LDS-DMA instructions one wave issues per stage (A + B): the vmcnt unit of the pipeline
  static constexpr int PER_STAGE = (BM + BN) * BK / (512 * NW);
  // epilogue: fp32 staging of EPI_ROWS rows at a time (whole tile when it fits)
  static constexpr int CS_LD = BN + 4;
  static constexpr int EPI_ROWS = (NW == 4 && BM <= 128) ? BM : SM;
  static constexpr int CHUNKS = BM / EPI_ROWS, WPC = EPI_ROWS / SM;  // wave-rows per chunk
  static constexpr int CS_BYTES = EPI_ROWS * CS_LD * 4;
  static constexpr int RED_BYTES = NT * 32;  // colsum partial staging
  static constexpr int SMEM = cmax<cmax<RING, CS_BYTES + 64>::v, RED_BYTES>::v;
  // per-wave LDS-DMA instructions of one A / one B tile (vmcnt units of the asymmetric ring)
  static constexpr int PER_A = BM * BK / (512 * NW), PER_B = BN * BK / (512 * NW);
  static_assert(FM >= 1 && FN >= 1 && SM % 16 == 0 && SN % 16 == 0, "wave sub-tile");
  static_assert((BM * BK) % (512 * NW) == 0 && (BN * BK) % (512 * NW) == 0,
                "LDS-DMA pieces per wave");
  static_assert(NT % (BN / 8) == 0 && (EPI_ROWS * (BN / 8)) % NT == 0, "epilogue mapping");
  static_assert(SMEM <= 160 * 1024, "LDS budget");
};

// Stage one operand tile (T entries of the M/N dim x BK of K) into LDS with LDS-DMA.
// Tile bytes = T*BK*2 = T*BK/512 KiB pieces; each of the NW waves issues T*BK/(512*NW) of them.
// Rows / columns at or past `mn_lim` (a partial edge tile) are clamped onto the last valid
// row / 8-column chunk: the loads stay in bounds, and the outputs they feed are never stored.
template <int L, int T, int NW, int BK = 64>
__device__ __forceinline__ void stage_tile(const u16* __restrict__ g, long ld, int mn0, int k0,
                                           char LDS_AS* dst, int wave, int lane, int mn_lim) {
  constexpr int NI = T * BK / (512 * NW);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int piece = i * NW + wave;
    const int chunk = piece * 64 + lane;
    const u16* src;
    if constexpr (L == KMAJ) {
      constexpr int CPR = BK / 8;  // 16-B chunks per row
      const int r = chunk / CPR, ph = chunk % CPR;
      const int c = ph ^ k_swz<BK>(r);
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

// LDS-DMA source of one operand for the register-prefetched loop, strength-reduced (round 5).
// The loads are issued from inline asm: the compiler's wait-count pass tracks LDS-DMA it emits
// itself and, finding no alias information, puts an s_waitcnt vmcnt(0) in front of every later
// ds_read_b64_tr_b16 -- each k-step of an MN-major operand would wait for the tile just issued
// for the NEXT k-step; issued from asm the loads are invisible to that pass and the pipeline's
// own counted vmcnt waits order them. Until round 5 every lane's source address was recomputed
// per k-step -- for an MN-major operand `(k0 + r) * ld` as a 64-bit multiply per piece (16
// quarter-rate v_mul_lo_u32 + 8 v_mad_u64_u32 per 64-deep k-step of the 128x128 wgrad: more
// VALU issue than its 32 MFMAs, docs/DESIGN.md section 7). Now every lane's byte offset inside
// the tile (edge clamp included) is computed ONCE and a k-step only moves a scalar base: the
// load is the SADDR form `global_load_lds_dwordx4 voff, s[base]` (address = base + voff), so
// the loop issues no vector ALU for its loads (profiles/r5_isa).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
template <int L, int T, int NW>
struct DmaSrc {
  static constexpr int NI = T * 64 / (512 * NW);
  unsigned voff[NI];  // per-lane byte offset of piece i from the tile's (k0, mn0) corner
  const char* base;   // operand + mn0 (row offset for K-major), bytes; uniform
  long kstride;       // bytes per unit of k: ld * 2 (MN-major) or 2 (K-major)

  __device__ __forceinline__ DmaSrc(const u16* __restrict__ g, long ld, int mn0, int wave,
                                    int lane, int mn_lim) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int chunk = (i * NW + wave) * 64 + lane;
      if constexpr (L == KMAJ) {
        const int r = chunk / 8, ph = chunk % 8;
        const int c = ph ^ k_swz<64>(r);
        voff[i] = (unsigned)((long)(min(mn0 + r, mn_lim - 1) - mn0) * ld * 2 + c * 16);
      } else {
        constexpr int CPR = T / 8;
        const int r = chunk / CPR, ph = chunk % CPR;
        const int c = ph ^ mn_swz<T>(r);
        voff[i] = (unsigned)((long)r * ld * 2 + (min(mn0 + c * 8, mn_lim - 8) - mn0) * 2);
      }
    }
    base = (const char*)(g + (L == KMAJ ? (long)mn0 * ld : (long)mn0));
    kstride = L == KMAJ ? 2 : ld * 2;
  }

  // the k-step starting at contraction index k0 -> LDS tile `dst` (T x 64 image)
  __device__ __forceinline__ void issue(int k0, char LDS_AS* dst, int wave) const {
    const char* b = base + (long)k0 * kstride;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const unsigned m0v =
          __builtin_amdgcn_readfirstlane((unsigned)(size_t)(dst + (i * NW + wave) * 1024));
      asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1"
                   :: "v"(voff[i]), "s"(b), "s"(m0v) : "memory", "m0");
    }
  }
};
#pragma clang diagnostic pop

// Fragment of v_mfma_f32_16x16x32_bf16 for 16-wide block `blk` of the tile and k-step s (32 k):
// lane l holds X[idx = l&15][k = 8*(l>>4) + j], j = 0..7 (guide §3 operand maps). The same form
// serves A (idx = row m) and B (idx = column n).
template <int L, int T, int BK = 64>
__device__ __forceinline__ bf16x8_t load_frag(const char LDS_AS* tile, int blk, int s, int lane) {
  if constexpr (L == KMAJ) {
    const int r = blk * 16 + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    return *(const bf16x8_t LDS_AS*)(tile + r * (BK * 2) + ((c ^ k_swz<BK>(r)) << 4));
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

// Byte of the 1-bit ReLU mask for row `row`, 8-column chunk `c` (GemmParams::mask_out/in):
// row-block-major, [M/16][ld_mask][16], so the 16 rows x 4 consecutive chunks a wave stores in
// the register-direct epilogue are 64 contiguous bytes (row-major bytes scattered one store
// over 16 rows).
__device__ __forceinline__ long mask_index(long row, long c, long ld) {
  return (((row >> 4) * ld + c) << 4) + (row & 15);
}

// Fragment-order ReLU masks (GemmParams::ld_mask < 0; register-direct epilogue only). The
// NB = FM * FN / 2 mask bytes one lane stores (forward) or reads (dgrad) -- byte jj * FM + i =
// row 16 i of the lane, the 8-column chunk it holds of fragment pair jj after the 16-lane swap
// -- are contiguous, lane-major within a wave and wave-major within a tile: one NB-byte access
// per lane moves a wave's whole mask, where the row-block-major layout takes NB one-byte
// accesses of 64 bytes per wave. Forward and dgrad must run the same tile / wave layout
// (ops.FragMask pins it). Buffer: tiles_m * tiles_n * BM * BN / 8 bytes.
template <int FM, int FN, int BN, int SN, int WM>
__device__ __forceinline__ long frag_mask_offset(const GemmParams& p, int tm, int tn, int wm,
                                                 int wn, int lane) {
  constexpr int WN = BN / SN, NB = FM * FN / 2;
  const long tiles_n = (p.N + BN - 1) / BN;
  return ((((long)tm * tiles_n + tn) * (WM * WN) + wm * WN + wn) * 64 + lane) * NB;
}
template <int NB>
__device__ __forceinline__ void frag_mask_store(unsigned char* dst, const unsigned* w) {
  if constexpr (NB == 16) *(uint4*)dst = make_uint4(w[0], w[1], w[2], w[3]);
  else if constexpr (NB == 8) *(uint2*)dst = make_uint2(w[0], w[1]);
  else *(unsigned*)dst = w[0];
}
template <int NB>
__device__ __forceinline__ void frag_mask_load(const unsigned char* src, unsigned* w) {
  if constexpr (NB == 16) {
    const uint4 v = *(const uint4*)src;
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else if constexpr (NB == 8) {
    const uint2 v = *(const uint2*)src;
    w[0] = v.x; w[1] = v.y;
  } else {
    w[0] = *(const unsigned*)src;
  }
}

// Phase timestamp of the workgroup (GemmParams::timeline); thread 0 stores it.
__device__ __forceinline__ void tl_mark(const GemmParams& p, int slot) {
  if (p.timeline && threadIdx.x == 0)
    p.timeline[4 * blockIdx.x + slot] = __builtin_amdgcn_s_memrealtime();
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
// The k-step body shared by both rings: fragments of one staged A / B tile -> MFMAs.
template <class C, int LA, int LB>
__device__ __forceinline__ void mma_kstep(const char LDS_AS* sa, const char LDS_AS* sb,
                                          f32x4_t (&acc)[C::FM][C::FN], int wm, int wn,
                                          int lane) {
  constexpr int FM = C::FM, FN = C::FN;
#pragma unroll
  for (int s = 0; s < C::BK / 32; ++s) {
    bf16x8_t a[FM], b[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) a[i] = load_frag<LA, C::BM, C::BK>(sa, wm * FM + i, s, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) b[j] = load_frag<LB, C::BN, C::BK>(sb, wn * FN + j, s, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// Asymmetric ring (Cfg NS = 3, NSB = 2): A slots kt % 3, B slots kt % 2. Issue order is
// A0 B0 A1 | step kt: B(kt+1) A(kt+2), so at the top of step kt the only loads younger than
// A(kt) and B(kt) are A(kt+1)'s: wait vmcnt(PER_A) (vmcnt(0) once A(kt+1) does not exist).
// Bytes in flight while step kt computes: A(kt+1), A(kt+2), B(kt+1) -- two A tiles instead of
// one. WAR: step kt restages A slot (kt+2)%3 and B slot (kt+1)%2, both last read in step kt-1,
// which every wave finished before the barrier at the top of kt.
template <class C, int LA, int LB>
__device__ __forceinline__ void mma_tile_asym(const GemmParams& p, int m0, int n0, int kbase,
                                              int nk, char LDS_AS* lds,
                                              f32x4_t (&acc)[C::FM][C::FN], int wm, int wn,
                                              int wave, int lane) {
  constexpr int A_BYTES = C::A_BYTES, B_BYTES = C::B_BYTES;
  char LDS_AS* ring_b = lds + 3 * A_BYTES;
  auto stage_a = [&](int k) {
    stage_tile<LA, C::BM, C::NW, C::BK>(p.A, p.lda, m0, kbase + k * C::BK,
                                        lds + (k % 3) * A_BYTES, wave, lane, p.M);
  };
  auto stage_b = [&](int k) {
    stage_tile<LB, C::BN, C::NW, C::BK>(p.B, p.ldb, n0, kbase + k * C::BK,
                                        ring_b + (k & 1) * B_BYTES, wave, lane, p.N);
  };
  stage_a(0);
  stage_b(0);
  if (nk > 1) stage_a(1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) wait_vmcnt<C::PER_A>();
    else wait_vmcnt<0>();
    lds_barrier();
    if (kt + 1 < nk) stage_b(kt + 1);
    if (kt + 2 < nk) stage_a(kt + 2);
    mma_kstep<C, LA, LB>(lds + (kt % 3) * A_BYTES, ring_b + (kt & 1) * B_BYTES, acc, wm, wn,
                         lane);
  }
  __syncthreads();
}

// Register-prefetched ring (Cfg RP): per 64-deep k-step kt, with the k 0..31 fragments of tile
// kt already in registers:
//   read k 32..63 fragments of kt | MFMAs on k 0..31
//   -> own loads of tile kt+1 landed, lds_barrier (every wave's reads of tile kt are done and
//      everyone's tile kt+1 landed) -> LDS-DMA tile kt+NS into tile kt's slot
//   read k 0..31 fragments of kt+1 | MFMAs on k 32..63 of kt
// so every fragment read overlaps MFMAs of the same wave, and the barrier is followed by MFMAs
// that do not wait on LDS. NS tiles are staged up front (tile kt+NS reuses tile kt's slot).
template <class C, int LA, int LB>
__device__ __forceinline__ void read_half(const char LDS_AS* sa, const char LDS_AS* sb,
                                          bf16x8_t (&a)[C::FM], bf16x8_t (&b)[C::FN], int wm,
                                          int wn, int s, int lane) {
#pragma unroll
  for (int i = 0; i < C::FM; ++i) a[i] = load_frag<LA, C::BM>(sa, wm * C::FM + i, s, lane);
#pragma unroll
  for (int j = 0; j < C::FN; ++j) b[j] = load_frag<LB, C::BN>(sb, wn * C::FN + j, s, lane);
}

template <class C>
__device__ __forceinline__ void mfma_half(const bf16x8_t (&a)[C::FM], const bf16x8_t (&b)[C::FN],
                                          f32x4_t (&acc)[C::FM][C::FN]) {
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      if constexpr (C::DIRECT)  // swapped: the fragment is C^T's (epilogue_direct layout)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      else
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
}

// Placement of a half's NR fragment reads among its NM MFMAs (sched_group_barrier masks:
// 0x8 MFMA, 0x100 DS read), closed by a sched_barrier so nothing crosses into the wait /
// barrier that follows.
template <int PATTERN, int NR, int NM>
__device__ __forceinline__ void rp_interleave() {
  if constexpr (PATTERN == 0) {  // one read, then NM / NR MFMAs; the rest of the MFMAs last
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, NM / NR > 0 ? NM / NR : 1, 0);
    }
    if constexpr (NM > NR * (NM / NR))
      __builtin_amdgcn_sched_group_barrier(0x8, NM - NR * (NM / NR), 0);
  } else if constexpr (PATTERN == 1) {  // two reads per MFMA until the reads are out
    static_assert(NR % 2 == 0, "reads come in pairs");
#pragma unroll
    for (int i = 0; i < NR / 2; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
    }
    if constexpr (NM > NR / 2) __builtin_amdgcn_sched_group_barrier(0x8, NM - NR / 2, 0);
  } else {  // every read first
    __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
    __builtin_amdgcn_sched_group_barrier(0x8, NM, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <class C, int LA, int LB>
__device__ __forceinline__ void mma_tile_rp(const GemmParams& p, int m0, int n0, int kbase,
                                            int nk, char LDS_AS* lds,
                                            f32x4_t (&acc)[C::FM][C::FN], int wm, int wn,
                                            int wave, int lane) {
  // Ring slots: symmetric = NS x [A | B] stages; asymmetric (C::ASYM) = 3 A slots then 2 B
  // slots, so the A operand (the streamed activation panel, HBM) gets two k-steps to land
  // and the B operand (weights, L2-resident) one.
  constexpr int NA = C::NS, NB = C::NSB, A_BYTES = C::A_BYTES, B_BYTES = C::B_BYTES;
  auto a_at = [&](int slot) -> char LDS_AS* {
    return C::ASYM ? lds + slot * A_BYTES : lds + slot * C::STAGE;
  };
  auto b_at = [&](int slot) -> char LDS_AS* {
    return C::ASYM ? lds + NA * A_BYTES + slot * B_BYTES : lds + slot * C::STAGE + A_BYTES;
  };
  const DmaSrc<LA, C::BM, C::NW> src_a(p.A, p.lda, m0, wave, lane, p.M);
  const DmaSrc<LB, C::BN, C::NW> src_b(p.B, p.ldb, n0, wave, lane, p.N);
  auto st_a = [&](int k, int slot) { src_a.issue(kbase + k * 64, a_at(slot), wave); };
  auto st_b = [&](int k, int slot) { src_b.issue(kbase + k * 64, b_at(slot), wave); };
  // Prologue: every slot staged (tiles past the end clamp to the last one: same load counts
  // whatever nk is), then tile 0 landed.
  if constexpr (C::ASYM) {  // issue order A0 B0 A1 B1 A2
    st_a(0, 0);
    st_b(0, 0);
    st_a(min(1, nk - 1), 1);
    st_b(min(1, nk - 1), 1);
    st_a(min(2, nk - 1), 2);
    wait_vmcnt<2 * C::PER_A + C::PER_B>();
  } else {
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      st_a(min(s, nk - 1), s);
      st_b(min(s, nk - 1), s);
    }
    wait_vmcnt<(NA - 1) * C::PER_STAGE>();
  }
  lds_barrier();
  tl_mark(p, 1);
  bf16x8_t a0[C::FM], b0[C::FN], a1[C::FM], b1[C::FN];
  read_half<C, LA, LB>(a_at(0), b_at(0), a0, b0, wm, wn, 0, lane);
  // Wait counts the compiler's wait-count pass can see (a builtin, unlike inline asm): with no
  // LDS read pending at the loop head / after the barrier, it lets the MFMAs on registers that
  // have landed issue while the next half's reads are in flight. The loop body is branch-free
  // (the last k-step is peeled), so no control-flow merge forces a conservative lgkmcnt(0) in
  // front of an MFMA.
  __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt(63) expcnt(7) lgkmcnt(0)
  // Instruction interleave of both halves (sched_group_barrier masks: 0x8 MFMA, 0x100 DS read):
  // each fragment read is followed by NM / NR MFMAs, the rest of the MFMAs come last.
  constexpr int NR = (C::FM + C::FN) * (LA == KMAJ ? 1 : 2) / 2 +
                     (C::FM + C::FN) * (LB == KMAJ ? 1 : 2) / 2;  // DS reads per half
  constexpr int NM = C::FM * C::FN;                                // MFMAs per half
  int ra = 0, rb = 0;  // A / B slots of tile kt
  for (int kt = 0; kt + 1 < nk; ++kt) {
    read_half<C, LA, LB>(a_at(ra), b_at(rb), a1, b1, wm, wn, 1, lane);
    mfma_half<C>(a0, b0, acc);
    rp_interleave<C::RP_PATTERN, NR, NM>();
    // own loads of tile kt+1 landed: asymmetric -- only A(kt+2) was issued after B(kt+1);
    // symmetric -- tiles kt+2 .. kt+NS-1 may stay in flight
    if constexpr (C::ASYM) wait_vmcnt<C::PER_A>();
    else wait_vmcnt<(NA - 2) * C::PER_STAGE>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_barrier" ::: "memory");
    // Tile kt's slots are free: B(kt+NB) and A(kt+NA) into them; past the end the last tile is
    // restaged instead (an L2 hit into a slot nobody reads again), so the loop body has no
    // branch and every k-step leaves the same loads in flight.
    st_b(min(kt + NB, nk - 1), rb);
    st_a(min(kt + NA, nk - 1), ra);
    ra = ra + 1 == NA ? 0 : ra + 1;
    rb = rb + 1 == NB ? 0 : rb + 1;
    read_half<C, LA, LB>(a_at(ra), b_at(rb), a0, b0, wm, wn, 0, lane);
    mfma_half<C>(a1, b1, acc);
    rp_interleave<C::RP_PATTERN, NR, NM>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  read_half<C, LA, LB>(a_at(ra), b_at(rb), a1, b1, wm, wn, 1, lane);
  mfma_half<C>(a0, b0, acc);
  mfma_half<C>(a1, b1, acc);
  // the restaged tail tiles (nothing reads them) land before the epilogue reuses LDS; waited
  // here, after the last k-step, not in front of it
  wait_vmcnt<0>();
  __syncthreads();
}

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
  if constexpr (C::RP) {
    mma_tile_rp<C, LA, LB>(p, m0, n0, kbase, nk, lds, acc, wm, wn, wave, lane);
    return;
  }
  if constexpr (C::ASYM) {
    mma_tile_asym<C, LA, LB>(p, m0, n0, kbase, nk, lds, acc, wm, wn, wave, lane);
    return;
  }

#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    if (s < nk) {
      stage_tile<LA, C::BM, C::NW, C::BK>(p.A, p.lda, m0, kbase + s * C::BK, lds + s * STAGE,
                                          wave, lane, p.M);
      stage_tile<LB, C::BN, C::NW, C::BK>(p.B, p.ldb, n0, kbase + s * C::BK,
                                          lds + s * STAGE + A_BYTES, wave, lane, p.N);
    }
  }
  int rd = 0, wr = NS - 1;  // ring slots of tile kt and of tile kt + NS - 1
  for (int kt = 0; kt < nk; ++kt) {
    wait_stage<NS, C::PER_STAGE>(min(nk - 1 - kt, NS - 2));
    lds_barrier();
    if (kt == 0) tl_mark(p, 1);
    if (kt + NS - 1 < nk) {
      char LDS_AS* nxt = lds + wr * STAGE;
      const int k0 = kbase + (kt + NS - 1) * C::BK;
      stage_tile<LA, C::BM, C::NW, C::BK>(p.A, p.lda, m0, k0, nxt, wave, lane, p.M);
      stage_tile<LB, C::BN, C::NW, C::BK>(p.B, p.ldb, n0, k0, nxt + A_BYTES, wave, lane, p.N);
    }
    // (Reading both 32-deep halves' fragments up front behind a sched_barrier was measured:
    // +8 % on 128x128 big GEMMs, -35 % on 256x256 dgrad whose 40 transposed reads exceed what
    // lgkmcnt can count -- the compiler's own interleaving is kept.)
    mma_kstep<C, LA, LB>(lds + rd * STAGE, lds + rd * STAGE + A_BYTES, acc, wm, wn, lane);
    rd = rd + 1 == NS ? 0 : rd + 1;
    wr = wr + 1 == NS ? 0 : wr + 1;
  }
  __syncthreads();
}

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

// Staged epilogue shared by the one-tile-per-workgroup kernels (gemm.hip, gemm_pp.hip):
// accumulators (C/D map: col = lane&15, row = 4*(lane>>4) + r) -> fp32 LDS tile (EPI_ROWS rows at
// a time) -> 16-byte row chunks with the fused bias / activation / activation-derivative /
// split-K accumulation / colsum / softmax-CE work. The caller's LDS (>= C::CS_BYTES + 64) must be
// free: every wave is past the main loop's last barrier.
template <class C, bool OUT_F32>
__device__ __forceinline__ void epilogue_staged(const GemmParams& p,
                                                const f32x4_t (&acc)[C::FM][C::FN],
                                                char LDS_AS* lds, int m0, int n0, int tm,
                                                int split, int wave, int lane) {
  constexpr int BM = C::BM, BN = C::BN, NT = C::NT, CS_LD = C::CS_LD;
  (void)BM;
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
  // Activation rows of the dgrad's act' (aux) are read one chunk AHEAD: chunk c+1's loads are
  // in flight while chunk c is stored, so only chunk 0's round trip is exposed.
  [[maybe_unused]] bf16x8_t yv[ITER], yn[ITER];
  const bool aux_rows = !OUT_F32 && p.aux && !xent;  // uniform
  auto load_aux = [&](int ch, bf16x8_t (&dst)[ITER]) {
    const long r0 = m0 + ch * C::EPI_ROWS + crow;
#pragma unroll
    for (int it = 0; it < ITER; ++it)
      if (col_ok && r0 + it * RSTEP < p.M)
        dst[it] = *(const bf16x8_t*)(p.aux + (r0 + it * RSTEP) * p.ld_aux + gn);
  };
  if (aux_rows) load_aux(0, yv);
#pragma unroll 1
  for (int chunk = 0; chunk < C::CHUNKS; ++chunk) {
    // Epilogue barriers are LDS-only (lds_barrier): __syncthreads' release fence would wait
    // for every global store of the previous chunk (vmcnt(0)), serialising the chunks.
    if (chunk) lds_barrier();  // every thread has read the previous chunk's staging tile
    acc_to_lds<C>(acc, cs, chunk, wave, lane);
    lds_barrier();
    if constexpr (!OUT_F32 && C::NW == 4 && C::CHUNKS == 1) {
      if (xent) {  // fused softmax-CE, one thread per row of the tile
        xent_rows<C>(p, cs, m0);
        lds_barrier();
      }
    }
    const long gm0 = m0 + chunk * C::EPI_ROWS + crow;
    [[maybe_unused]] bf16x8_t ov[ITER];  // the stored values, for the transposed copy
    [[maybe_unused]] unsigned mk[ITER];
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
      if (aux_rows) {
        if (chunk + 1 < C::CHUNKS) load_aux(chunk + 1, yn);
      } else if (p.mask_in) {
#pragma unroll
        for (int it = 0; it < ITER; ++it)
          if (col_ok && gm0 + it * RSTEP < p.M)
            mk[it] = p.mask_in[mask_index(gm0 + it * RSTEP, gn >> 3, p.ld_mask)];
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
        if (p.upd_master) {  // uniform: fused SGD of the weights this gradient belongs to
          const long off = gm * p.ldc + gn;
          const float lr = *p.upd_lr;
          const f32x4_t w0 = sgd4(p.upd_master + off, f32x4_t{v[0], v[1], v[2], v[3]},
                                  p.upd_mom ? p.upd_mom + off : nullptr,
                                  p.upd_shadow ? p.upd_shadow + off : nullptr, lr, p.upd_mu,
                                  p.upd_wd);
          const f32x4_t w1 = sgd4(p.upd_master + off + 4, f32x4_t{v[4], v[5], v[6], v[7]},
                                  p.upd_mom ? p.upd_mom + off + 4 : nullptr,
                                  p.upd_shadow ? p.upd_shadow + off + 4 : nullptr, lr,
                                  p.upd_mu, p.upd_wd);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ov[it][e] = (short)f2bf(w0[e]);
            ov[it][e + 4] = (short)f2bf(w1[e]);
          }
          continue;
        }
        float* c = (float*)p.C + (long)split * p.c_split_stride + gm * p.ldc + gn;
        if (!p.accumulate && p.act != ACT_LINEAR) {  // (one uniform test per row, not per element)
          if (p.act == ACT_RELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = act_fwd(v[e], p.act);
          }
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
        } else if (p.aux) {  // activation tests hoisted out of the element loops (uniform)
          if (p.act == ACT_RELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = bf2f((u16)yv[it][e]) > 0.f ? v[e] : 0.f;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = act_bwd(v[e], bf2f((u16)yv[it][e]), p.act);
          }
        } else if (p.mask_in) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (mk[it] >> e) & 1u ? v[e] : 0.f;
        } else if (p.act == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        } else if (p.act != ACT_LINEAR) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = act_fwd(v[e], p.act);
        }
        bf16x8_t o;
        unsigned bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const u16 h = f2bf(v[e]);
          o[e] = (short)h;
          csum[e] += bf2f(h);
          bits |= (bf2f(h) > 0.f ? 1u : 0u) << e;
        }
        *(bf16x8_t*)((u16*)p.C + gm * p.ldc + gn) = o;
        ov[it] = o;
        if (p.mask_out) p.mask_out[mask_index(gm, gn >> 3, p.ld_mask)] = (unsigned char)bits;
      }
    }
    {
      if (p.ct) {  // uniform: transposed copy of this chunk through LDS (bf16 [BN][rows]):
                   // the stored bf16 output, or (fused update) the new bf16 weights
        // bf16 [BN][TLD] transposed tile. The 8-row block of a row index is XOR-swizzled by
        // the column's 8-column group (sw): together with the +8 pad, the 2-byte writes of a
        // half-wave (32 column groups, one row) spread over 16 banks instead of 2, and every
        // 8-row block stays a contiguous, aligned 16-byte read.
        constexpr int TLD = C::EPI_ROWS + 8;
        constexpr int RC = C::EPI_ROWS / 8;  // 16-byte chunks per transposed row
        static_assert(BN * TLD * 2 <= C::SMEM, "transposed chunk fits the staging LDS");
        static_assert((RC & (RC - 1)) == 0, "row blocks: power of two");
        u16 LDS_AS* tt = (u16 LDS_AS*)lds;
        lds_barrier();  // every thread is done reading the fp32 staging tile
        const int sw = ((ccol >> 3) & (RC - 1)) << 3;
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
          const int row = (crow + it * RSTEP) ^ sw;
#pragma unroll
          for (int e = 0; e < 8; ++e) tt[(ccol + e) * TLD + row] = (u16)ov[it][e];
        }
        lds_barrier();
        const long m_base = m0 + chunk * C::EPI_ROWS;
#pragma unroll 2
        for (int idx = threadIdx.x; idx < BN * RC; idx += NT) {
          const int col = idx / RC, r8 = (idx % RC) * 8;
          const long gcol = n0 + col, grow = m_base + r8;
          if (gcol >= p.N || grow >= p.M) continue;  // partial edge tile
          const int rs = r8 ^ (((col >> 3) & (RC - 1)) << 3);
          const bf16x8_t v = *(const bf16x8_t LDS_AS*)(tt + col * TLD + rs);
          *(bf16x8_t*)(p.ct + gcol * p.ld_ct + grow) = v;
        }
      }
    }
    if (aux_rows) {
#pragma unroll
      for (int it = 0; it < ITER; ++it) yv[it] = yn[it];
    }
  }
  if constexpr (!OUT_F32) {
    if (p.colsum) {  // uniform across the block
      lds_barrier();  // all reads of the staging tile are done
      f32x4_t LDS_AS* red = (f32x4_t LDS_AS*)lds;
      red[2 * threadIdx.x] = f32x4_t{csum[0], csum[1], csum[2], csum[3]};
      red[2 * threadIdx.x + 1] = f32x4_t{csum[4], csum[5], csum[6], csum[7]};
      lds_barrier();
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

// Sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15) in a fixed butterfly order.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}

// Register-direct epilogue for SWAPPED-operand accumulators (mfma(b, a): a lane's fragment
// holds 4 consecutive output columns of one row): acc[i][j][e] = C[row0 + 16 i][col0 + 16 j + e]
// with row0 = tile row + wave row offset + (lane & 15), col0 = ... + 4 * (lane >> 4). bf16
// output pairs fragments j, j+1 with v_permlane16_swap into one 16-byte chunk per lane; fp32
// output stores each fragment's 16 bytes. with_colsum: the bias-gradient column sums are
// reduced across the WM wave rows in the ring slot the last k-step consumed (`rd` is the ring
// read cursor after the loop) -- callers whose waves are not in lock step pass false.
// 16-byte stores every lane of a FULL tile issues in the bf16 form of epilogue_direct (before
// an optional column-sum store): a persistent kernel that issued its next stage before the
// epilogue may wait for it with vmcnt(this) instead of vmcnt(0) (stores retire in order).
template <int FM, int FN>
constexpr int epilogue_direct_stores() { return FM * FN / 2; }

template <int FM, int FN, int BN, int SN, int WM, int NS, int STAGE, bool OUT_F32>
__device__ __forceinline__ void epilogue_direct(const GemmParams& p, f32x4_t (&acc)[FM][FN],
                                                char LDS_AS* lds, int rd, int tm, int tn,
                                                int split, int wm, int wn, int lane,
                                                bool with_colsum) {
  static_assert(FN % 2 == 0, "fragment pairs for the 16-byte epilogue stores");
  const int frow = lane & 15, fg = lane >> 4;
    // ---- epilogue straight from the accumulators ------------------------------------------
    // acc[i][j][e] = C[row0 + 16 i][col0 + 16 j + e]
    const int row0 = tm * (WM * 16 * FM) + wm * 16 * FM + frow;
    const int col0 = tn * BN + wn * SN + 4 * fg;
    if constexpr (OUT_F32) {
      float* cbase = (float*)p.C + (long)split * p.c_split_stride + col0;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = row0 + 16 * i;
        if (row >= p.M) continue;
        float* crow = cbase + (long)row * p.ldc;  // columns 16 j: immediate offsets
        f32x4_t v[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          v[j] = acc[i][j];
          if (p.accumulate && col0 + 16 * j < p.N) v[j] += *(const f32x4_t*)(crow + 16 * j);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if (col0 + 16 * j >= p.N) continue;
          if (p.bias) v[j] += *(const f32x4_t*)(p.bias + col0 + 16 * j);
          if (!p.accumulate && p.act != ACT_LINEAR) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              v[j][e] = p.act == ACT_RELU ? (v[j][e] > 0.f ? v[j][e] : 0.f) : act_fwd(v[j][e], p.act);
          }
          *(f32x4_t*)(crow + 16 * j) = v[j];
        }
      }
    } else {
      const bool want_sum = with_colsum && p.colsum != nullptr;  // uniform
      // store column after the 16-lane swap: even groups keep an 8-column half of fragment j,
      // odd groups take one of fragment j+1 (see below)
      const int scol0 = tn * BN + wn * SN + 16 * (fg & 1) + 8 * (fg >> 1);
      // [WM][BN] colsum partials in the slot of the last consumed stage: no DMA targets it
      // before the next k-step's barrier; wait until every wave has finished reading it
      float LDS_AS* red = (float LDS_AS*)(lds + (rd == 0 ? NS - 1 : rd - 1) * STAGE);
      if (want_sum) lds_barrier();
      // Every global READ of the epilogue (bias, activation values for the derivative) is
      // issued before its first store: loads and stores share vmcnt and retire in order, so a
      // load issued after a store would make its wait drain that store too. With the reads up
      // front the stores stream out unwaited, and a persistent caller only waits for its next
      // stage (issued before them) with vmcnt(#stores) -- see epilogue_direct_stores.
      // Two instantiations of the store loop (activation derivative from `aux`, or bias +
      // activation), so only one kind of hoisted operand is live at a time.
      // ReLU dgrad: the derivative is a mask, and masking commutes with the bf16 rounding, so
      // it is applied AFTER the 16-lane swap, to the 8 consecutive columns a lane stores: the
      // activation rows are then read as 16-byte chunks (64 contiguous bytes per row and
      // instruction) instead of 8-byte ones. Column sums of the stored values are taken in the
      // same layout; per column they add the same rows in the same order (the swap keeps a
      // lane's row), so the result is bitwise that of the generic path.
      // from_mask: the derivative comes from the forward's 1-bit ReLU mask (mask_in: one byte
      // per row and 8-column chunk -- exactly the chunk a lane stores) instead of the activation
      constexpr int NB = FM * FN / 2;  // fragment-order mask bytes per lane
      const bool frag = p.ld_mask < 0;  // uniform
      // FULL: the whole tile is inside C (uniform, tested once below), so the per-row /
      // per-column bounds tests -- divergent exec-mask regions around every store and
      // column-sum update -- compile away
      auto relu_body = [&](auto from_mask, auto full_t) {
      constexpr bool MASK = decltype(from_mask)::value;
      constexpr bool FULL = decltype(full_t)::value;
      [[maybe_unused]] uint4 yv[MASK ? 1 : FN / 2][FM];
      [[maybe_unused]] unsigned mv[MASK ? FN / 2 : 1][FM];
      [[maybe_unused]] unsigned fw[MASK && NB >= 4 ? NB / 4 : 1];
      if constexpr (MASK && NB >= 4 && NB <= 16) {
        if (frag)
          frag_mask_load<NB>(p.mask_in + frag_mask_offset<FM, FN, BN, SN, WM>(p, tm, tn, wm, wn,
                                                                             lane), fw);
      }
#pragma unroll
      for (int jj = 0; jj < FN / 2; ++jj) {
        const int c = min(scol0 + 32 * jj, p.N - 8);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const long r = min(row0 + 16 * i, p.M - 1);
          if constexpr (MASK) {
            if constexpr (NB >= 4 && NB <= 16) {
              const int b = jj * FM + i;
              mv[jj][i] = frag ? (fw[b >> 2] >> (8 * (b & 3))) & 0xffu
                               : p.mask_in[mask_index(r, c >> 3, p.ld_mask)];
            } else {
              mv[jj][i] = p.mask_in[mask_index(r, c >> 3, p.ld_mask)];
            }
          } else {
            yv[jj][i] = *(const uint4*)(p.aux + r * p.ld_aux + c);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
        f32x4_t b0 = {0.f, 0.f, 0.f, 0.f}, b1 = {0.f, 0.f, 0.f, 0.f};
        if (p.bias) {  // (no caller combines bias and aux; kept correct, not hoisted)
          const int c0 = col0 + 16 * j;
          if (c0 < p.N) b0 = *(const f32x4_t*)(p.bias + c0);
          if (c0 + 16 < p.N) b1 = *(const f32x4_t*)(p.bias + c0 + 16);
        }
        float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const int scol = scol0 + 16 * j;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = row0 + 16 * i;
          const unsigned x0 = pack_bf16x2(acc[i][j][0] + b0[0], acc[i][j][1] + b0[1]);
          const unsigned x1 = pack_bf16x2(acc[i][j][2] + b0[2], acc[i][j][3] + b0[3]);
          const unsigned z0 = pack_bf16x2(acc[i][j + 1][0] + b1[0], acc[i][j + 1][1] + b1[1]);
          const unsigned z1 = pack_bf16x2(acc[i][j + 1][2] + b1[2], acc[i][j + 1][3] + b1[3]);
          const auto s0 = __builtin_amdgcn_permlane16_swap(x0, z0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(x1, z1, false, false);
          unsigned w[4] = {s0[0], s1[0], s0[1], s1[1]};
          if constexpr (MASK) {
            const unsigned m = mv[j / 2][i];
#pragma unroll
            for (int q = 0; q < 4; ++q)  // bit e of the byte = column e of the chunk
              w[q] &= ((m >> (2 * q)) & 1u ? 0x0000ffffu : 0u) |
                      ((m >> (2 * q + 1)) & 1u ? 0xffff0000u : 0u);
          } else {
            const uint4 y = yv[j / 2][i];
            const unsigned ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // keep a bf16 where its activation is > 0
              const unsigned lo = ys[q] & 0xffffu, hi = ys[q] >> 16;
              const unsigned keep = ((lo & 0x8000u) == 0u && lo != 0u ? 0x0000ffffu : 0u) |
                                    ((hi & 0x8000u) == 0u && hi != 0u ? 0xffff0000u : 0u);
              w[q] &= keep;
            }
          }
          if (want_sum && (FULL || row < p.M)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              cs[2 * q] += __uint_as_float(w[q] << 16);
              cs[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
            }
          }
          if ((FULL || (row < p.M && scol < p.N)) && !(p.epi_probe & 1))
            *(uint4*)((u16*)p.C + (long)row * p.ldc + scol) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        if (want_sum) {  // the 8 columns this lane stores, summed over the wave's rows
          f32x4_t r0, r1;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            r0[e] = row16_sum(cs[e]);
            r1[e] = row16_sum(cs[4 + e]);
          }
          if (frow == 0) {
            float LDS_AS* d = red + wm * BN + (scol - tn * BN);
            *(f32x4_t LDS_AS*)d = r0;
            *(f32x4_t LDS_AS*)(d + 4) = r1;
          }
        }
      }
      };
      // `act_c`: the forward activation as a compile-time constant (ACT_RELU / ACT_LINEAR), or
      // -1 = read p.act per element. A runtime activation costs two scalar compare + branch
      // pairs per ELEMENT (128 per lane of a 256x256 tile): the ISA of the bias + ReLU
      // epilogue was mostly those branches (profiles/r4_timeline: 5.9 of its 6.2 us per round
      // remained with no stores and no bias loads)
      auto body = [&](auto has_aux, auto act_c, auto full_t) {
      constexpr bool AUX = decltype(has_aux)::value;
      constexpr int ACTC = decltype(act_c)::value;
      constexpr bool FULL = decltype(full_t)::value;
      [[maybe_unused]] unsigned fw[NB >= 4 ? NB / 4 : 1] = {};  // fragment-order mask_out
      [[maybe_unused]] f32x4_t bv[AUX ? 1 : FN];
      [[maybe_unused]] uint2 yv[AUX ? FN : 1][FM];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = col0 + 16 * j;
        if constexpr (AUX) {
          const u16* ya = p.aux + min(c, p.N - 4);
#pragma unroll
          for (int i = 0; i < FM; ++i)
            yv[j][i] = *(const uint2*)(ya + min(row0 + 16 * i, p.M - 1) * p.ld_aux);
        } else {
          bv[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          if (p.bias && (FULL || c < p.N) && !(p.epi_probe & 2))
            bv[j] = *(const f32x4_t*)(p.bias + c);
        }
      }
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
        f32x4_t b0 = {0.f, 0.f, 0.f, 0.f}, b1 = {0.f, 0.f, 0.f, 0.f};
        [[maybe_unused]] const uint2* y0 = nullptr;
        [[maybe_unused]] const uint2* y1 = nullptr;
        if constexpr (AUX) {
          y0 = yv[j];
          y1 = yv[j + 1];
          if (p.bias) {  // (no caller combines bias and aux; kept correct, not hoisted)
            const int c0 = col0 + 16 * j;
            if (c0 < p.N) b0 = *(const f32x4_t*)(p.bias + c0);
            if (c0 + 16 < p.N) b1 = *(const f32x4_t*)(p.bias + c0 + 16);
          }
        } else {
          b0 = bv[j];
          b1 = bv[j + 1];
        }
        float cs0[4] = {0.f, 0.f, 0.f, 0.f}, cs1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = row0 + 16 * i;
          float v0[4], v1[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v0[e] = acc[i][j][e] + b0[e];
            v1[e] = acc[i][j + 1][e] + b1[e];
          }
          if constexpr (AUX) {
            const unsigned ya[2] = {y0[i].x, y0[i].y}, yb[2] = {y1[i].x, y1[i].y};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const unsigned sh = (e & 1) ? 0u : 16u;
              v0[e] = act_bwd(v0[e], __uint_as_float((ya[e >> 1] << sh) & 0xffff0000u), p.act);
              v1[e] = act_bwd(v1[e], __uint_as_float((yb[e >> 1] << sh) & 0xffff0000u), p.act);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v0[e] = act_fwd(v0[e], ACTC >= 0 ? ACTC : p.act);
              v1[e] = act_fwd(v1[e], ACTC >= 0 ? ACTC : p.act);
            }
          }
          const unsigned x0 = pack_bf16x2(v0[0], v0[1]), x1 = pack_bf16x2(v0[2], v0[3]);
          const unsigned z0 = pack_bf16x2(v1[0], v1[1]), z1 = pack_bf16x2(v1[2], v1[3]);
          if (want_sum && (FULL || row < p.M)) {  // sums of the STORED (bf16-rounded) values
            cs0[0] += __uint_as_float(x0 << 16);
            cs0[1] += __uint_as_float(x0 & 0xffff0000u);
            cs0[2] += __uint_as_float(x1 << 16);
            cs0[3] += __uint_as_float(x1 & 0xffff0000u);
            cs1[0] += __uint_as_float(z0 << 16);
            cs1[1] += __uint_as_float(z0 & 0xffff0000u);
            cs1[2] += __uint_as_float(z1 << 16);
            cs1[3] += __uint_as_float(z1 & 0xffff0000u);
          }
          // 16-lane half exchange (odd DPP rows of x <-> even rows of z). Afterwards group 0
          // holds cols 0..7 of fragment j, group 1 cols 0..7 of j+1, group 2 cols 8..15 of j,
          // group 3 cols 8..15 of j+1; in every group [0] = the chunk's low 4 columns.
          const auto s0 = __builtin_amdgcn_permlane16_swap(x0, z0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(x1, z1, false, false);
          const int scol = scol0 + 16 * j;
          if ((FULL || (row < p.M && scol < p.N)) && !(p.epi_probe & 1)) {
            *(uint4*)((u16*)p.C + (long)row * p.ldc + scol) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
            if (!AUX && p.mask_out) {  // forward ReLU mask: bit e = stored bf16 of column e > 0
              const unsigned w[4] = {s0[0], s1[0], s0[1], s1[1]};
              unsigned bits = 0;
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const unsigned lo = w[q] & 0xffffu, hi = w[q] >> 16;
                bits |= ((lo & 0x8000u) == 0u && lo != 0u ? 1u : 0u) << (2 * q);
                bits |= ((hi & 0x8000u) == 0u && hi != 0u ? 1u : 0u) << (2 * q + 1);
              }
              if constexpr (NB >= 4 && NB <= 16) {
                const int b = (j / 2) * FM + i;
                if (frag) fw[b >> 2] |= bits << (8 * (b & 3));
                else p.mask_out[mask_index(row, scol >> 3, p.ld_mask)] = (unsigned char)bits;
              } else {
                p.mask_out[mask_index(row, scol >> 3, p.ld_mask)] = (unsigned char)bits;
              }
            }
          }
        }
        if (want_sum) {  // this pair's column sums over the wave's rows -> LDS [wm][col]
          f32x4_t r0, r1;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            r0[e] = row16_sum(cs0[e]);
            r1[e] = row16_sum(cs1[e]);
          }
          if (frow == 0) {
            float LDS_AS* d = red + wm * BN + wn * SN + 16 * j + 4 * fg;
            *(f32x4_t LDS_AS*)d = r0;
            *(f32x4_t LDS_AS*)(d + 16) = r1;
          }
        }
      }
      if constexpr (!AUX && NB >= 4 && NB <= 16) {
        if (frag && p.mask_out)  // the whole tile's bits, one NB-byte store per lane
          frag_mask_store<NB>(p.mask_out + frag_mask_offset<FM, FN, BN, SN, WM>(p, tm, tn, wm,
                                                                               wn, lane), fw);
      }
      };
      const bool full = (tm + 1) * (WM * 16 * FM) <= p.M && (tn + 1) * BN <= p.N &&
                        !(p.epi_probe & 4);  // uniform
      auto dispatch = [&](auto full_t) {
        if (p.aux && p.act == ACT_RELU) relu_body(std::false_type{}, full_t);
        else if (p.mask_in) relu_body(std::true_type{}, full_t);
        else if (p.aux) body(std::true_type{}, std::integral_constant<int, -1>{}, full_t);
        else if (p.act == ACT_RELU && !(p.epi_probe & 4))
          body(std::false_type{}, std::integral_constant<int, ACT_RELU>{}, full_t);
        else if (p.act == ACT_LINEAR && !(p.epi_probe & 4))
          body(std::false_type{}, std::integral_constant<int, ACT_LINEAR>{}, full_t);
        else body(std::false_type{}, std::integral_constant<int, -1>{}, full_t);
      };
      if (full) dispatch(std::true_type{});
      else dispatch(std::false_type{});
      if (want_sum) {
        lds_barrier();
        if ((int)threadIdx.x < BN) {
          const int col = threadIdx.x;
          float tsum = 0.f;
#pragma unroll
          for (int r = 0; r < WM; ++r) tsum += red[r * BN + col];
          if (tn * BN + col < p.N) p.colsum[(long)tm * p.ld_colsum + tn * BN + col] = tsum;
        }
        // the slot is restaged only after the next k-step's barrier
      }
    }
}

}  // namespace dnn
