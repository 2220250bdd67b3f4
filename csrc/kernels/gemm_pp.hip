// 256x256 bf16 MFMA GEMM for gfx950 with a ping-pong, half-tile-streamed main loop.
//
// The one-tile kernel of gemm.hip (8 waves, one barrier per 64-deep k-step) keeps one 64-KiB
// stage in flight and runs every wave's LDS reads and MFMAs in lock step, so each SIMD's matrix
// core idles while both of its waves read fragments: 54-56 % MFMA busy on 16384x8192x8192
// (profiles/r1_pmc/big_gemm_counters.json). This form follows the 8-phase template of the
// CDNA4 guide (cdna_hip_programming.md §5, "The 256² 8-phase template"):
//   * waves 2 (M) x 4 (N), each owning a 128x64 output (8x4 fragments of 16x16x32);
//   * the k-dimension is staged in 16-KiB HALF-tiles (A or B, 32 deep: [256][32] images for
//     contraction-contiguous operands, [32][256] for output-dim-contiguous ones) streamed
//     through a 10-slot ring that uses all 160 KiB of LDS, 8 half-tiles ahead of the phase
//     that reads them -- about 80 KiB in flight per CU instead of 64 KiB in lock step;
//   * a 64-deep k-step is 4 phases (k-half x wave M-half), each {fragment reads + one half-tile
//     LDS-DMA issue -> barrier -> 16 MFMAs -> barrier};
//   * the two wave groups (waves 0-3 / 4-7: one of each on every SIMD) run one barrier apart,
//     so on every SIMD one wave's MFMA cluster overlaps the other's LDS reads and loads;
//   * counted vmcnt only (never 0 in the loop): after the MFMAs of even phases a wave waits
//     for its share of the half-tiles read two phases later (5 newer half-tiles = 10 loads
//     may stay in flight); restaging a slot happens 2 phases after its last read.
// Epilogue: the staged epilogue of gemm.hip (all fused epilogue work), after the ring drains.
//
// Reference parity: the forward is /root/reference/src/grpc_node.py:87 (z = x.W + b); the
// backward GEMMs replace the centralised autograd of
// /root/reference/scripts/generate_mnist_pytorch.py:41-52.
#include "gemm_tile.hpp"

namespace dnn {
namespace pp {

constexpr int R = 10;          // ring slots (half-tiles)
constexpr int D = 8;           // half-tiles issued ahead of the phase that first reads them
constexpr int HALF = 16384;    // bytes per half-tile image
static_assert(R * HALF == 160 * 1024, "the ring is all of LDS");
static_assert(R >= D + 2, "a slot is restaged >= 2 phases after its last read");

// [256][32] bf16 image (64-B rows): 16-B chunk c of row r lives at chunk c ^ swz(r). With the
// ds_read_b128 lane groups of the microarch guide's LDS table, the 16 lanes of each group
// (rows i and chunks 0..3 of a fragment read) then hit 16 distinct 16-B bank slots.
__device__ __forceinline__ int kh_swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

// Stage one half-tile (16 pieces of 1 KiB, two per wave) of operand tile rows/cols
// [mn0, mn0 + 256) x k [k0, k0 + 32). Partial edge tiles clamp to the last valid row/chunk.
template <int L>
__device__ __forceinline__ void stage_half(const u16* __restrict__ g, long ld, int mn0, int k0,
                                           char LDS_AS* dst, int wave, int lane, int mn_lim) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = i * 8 + wave;
    const int chunk = piece * 64 + lane;
    const u16* src;
    if constexpr (L == KMAJ) {
      const int r = chunk >> 2, ph = chunk & 3;
      const int c = ph ^ kh_swz(r);
      src = g + (long)min(mn0 + r, mn_lim - 1) * ld + k0 + c * 8;
    } else {  // [32 k-rows][256]: 32 chunks per 512-B row
      const int r = chunk >> 5, ph = chunk & 31;
      const int c = ph ^ mn_swz<256>(r);
      src = g + (long)(k0 + r) * ld + min(mn0 + c * 8, mn_lim - 8);
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (void LDS_AS*)(dst + piece * 1024), 16, 0,
                                     0);
  }
}

// 16x16x32 fragment of 16-wide block `blk` from a half-tile image (lane l: idx = l&15,
// k = 8*(l>>4) + j).
template <int L>
__device__ __forceinline__ bf16x8_t frag_half(const char LDS_AS* img, int blk, int lane) {
  if constexpr (L == KMAJ) {
    const int r = blk * 16 + (lane & 15), c = lane >> 4;
    return *(const bf16x8_t LDS_AS*)(img + r * 64 + ((c ^ kh_swz(r)) << 4));
  } else {
    return load_frag<MNMAJ, 256>(img, blk, 0, lane);  // k-rows 0..31 of a [32][256] image
  }
}

__device__ __forceinline__ void barrier_only() { asm volatile("s_barrier" ::: "memory"); }

}  // namespace pp

template <int LA, int LB, bool OUT_F32>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmParams p, int tiles_n, int tiles_m,
                                                      int nwg) {
  using C = Cfg<256, 256, 2, 4, 2>;  // epilogue geometry: waves 2 (M) x 4 (N), 128x64 each
  static_assert(C::CS_BYTES + 64 <= pp::R * pp::HALF, "epilogue staging fits the ring");
  __shared__ __attribute__((aligned(16))) char smem[pp::R * pp::HALF];
  char LDS_AS* lds = (char LDS_AS*)smem;

  // tile decode: identical to gemm_bf16_kernel (XCD remap, grouped raster, uneven split-K)
  const int wgid = xcd_remap(blockIdx.x, nwg);
  const int per_split = tiles_n * tiles_m;
  const int split = wgid / per_split;
  const int t = wgid - split * per_split;
  const int gm_full = p.group_m > 1 ? p.group_m : 1;
  const int per_group = gm_full * tiles_n;
  const int grp_r = t / per_group, first_m = grp_r * gm_full;
  const int gm = min(tiles_m - first_m, gm_full);
  const int tin = t - grp_r * per_group;
  const int tm = first_m + tin % gm;
  const int tn = tin / gm;
  const int m0 = tm * 256, n0 = tn * 256;
  int kbase, nk;
  if (p.k_total > 0) {
    const int KS = p.k_total >> 6, S = nwg / (tiles_n * tiles_m);
    const int a = (int)((long)split * KS / S), b = (int)((long)(split + 1) * KS / S);
    kbase = a * 64;
    nk = b - a;
  } else {
    kbase = split * p.K;
    nk = p.K >> 6;
  }

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;  // wr is also the ping-pong group

  // half-tile stream: h = 4 * k-step + i, i = 0 B[k 0..31], 1 A[k 0..31], 2 B[k 32..63],
  // 3 A[k 32..63]; slot h % R. Phase q = 4 * k-step + r reads (r = 0) B-half and A-half of
  // k-half 0 (A rows of the wave's first 64), (r = 1) A-half 0 (rows 64..127), (r = 2, 3) the
  // same for k-half 1 -- so half h is last read in phase h and first read in phase
  // 4 * (h / 4) + (h & 2).
  const int H = 4 * nk;
  auto issue = [&](int h) {
    const int kt = h >> 2, i = h & 3;
    const int k0 = kbase + kt * 64 + ((i & 2) ? 32 : 0);
    char LDS_AS* dst = lds + (h % pp::R) * pp::HALF;
    if (i & 1) pp::stage_half<LA>(p.A, p.lda, m0, k0, dst, wave, lane, p.M);
    else pp::stage_half<LB>(p.B, p.ldb, n0, k0, dst, wave, lane, p.N);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int pro = min(pp::D, H);
  for (int h = 0; h < pro; ++h) issue(h);
  // halves 0 and 1 (phase 0) landed: D - 2 newer half-tiles may stay in flight
  if (H >= pp::D) wait_vmcnt<2 * (pp::D - 2)>();
  else wait_vmcnt<0>();
  pp::barrier_only();
  if (wr == 1) pp::barrier_only();  // group 1 runs one barrier behind group 0

  bf16x8_t a[4], b[4];
  for (int kt = 0; kt < nk; ++kt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 4 * kt + r, kh = r >> 1, mh = r & 1;
      // ---- load section: fragments of this phase, one half-tile of the stream ------------
      if (mh == 0) {
        const char LDS_AS* imgB = lds + ((4 * kt + 2 * kh) % pp::R) * pp::HALF;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = pp::frag_half<LB>(imgB, wc * 4 + j, lane);
      }
      const char LDS_AS* imgA = lds + ((4 * kt + 2 * kh + 1) % pp::R) * pp::HALF;
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = pp::frag_half<LA>(imgA, wr * 8 + mh * 4 + i, lane);
      if (q + pp::D < H) issue(q + pp::D);
      pp::barrier_only();
      // ---- MFMA section ------------------------------------------------------------------
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 * mh + i][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[4 * mh + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (mh == 0) {  // the halves phase q + 2 reads (newest: q + 3) have landed
        if (q + pp::D < H) wait_vmcnt<2 * (pp::D - 3)>();
        else wait_vmcnt<0>();
      }
      pp::barrier_only();
    }
  }
  if (wr == 0) pp::barrier_only();  // equal barrier counts for both groups
  __syncthreads();                  // ring drained; LDS becomes the epilogue staging tile

  epilogue_staged<C, OUT_F32>(p, acc, lds, m0, n0, tm, split, wave, lane);
}

// Called by gemm_bf16 for 256x256 tiles with stages == 8 (the ping-pong form), after its
// shape validation.
// Called by gemm_bf16 for 256x256 tiles with stages == 8, after its shape validation.
int gemm_pp_launch(const GemmParams& q, int la, int lb, int out_f32, int splits,
                   hipStream_t stream) {
  typedef void (*fn_t)(GemmParams, int, int, int);
  fn_t fn;
#define DNN_PP(LA, LB) (out_f32 ? gemm_pp_kernel<LA, LB, true> : gemm_pp_kernel<LA, LB, false>)
  if (la == KMAJ && lb == KMAJ) fn = DNN_PP(KMAJ, KMAJ);
  else if (la == KMAJ && lb == MNMAJ) fn = DNN_PP(KMAJ, MNMAJ);
  else if (la == MNMAJ && lb == KMAJ) fn = DNN_PP(MNMAJ, KMAJ);
  else fn = DNN_PP(MNMAJ, MNMAJ);
#undef DNN_PP
  const int tiles_n = (q.N + 255) / 256, tiles_m = (q.M + 255) / 256;
  const int nwg = tiles_n * tiles_m * splits;
  hipLaunchKernelGGL(fn, dim3(nwg), dim3(512), 0, stream, q, tiles_n, tiles_m, nwg);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

}  // namespace dnn
