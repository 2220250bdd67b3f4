// Persistent bf16 MFMA GEMM for gfx950 with a register-direct epilogue.
//
// Why (profiles/r1_tiles/k_fit_fwd.jsonl): the one-tile-per-workgroup kernel of gemm.hip pays a
// large fixed cost per tile -- at 65536x512x832 the 256x256 tile spends 38.6 of 74 us outside
// its main loop. All workgroups of a launch start together, so every CU issues its first LDS
// fill at the same moment, computes, and then writes its output through an LDS staging tile at
// the same moment: HBM sees a read burst, an idle stretch and a write burst per round, and
// nothing overlaps a tile's epilogue.
//
// This form keeps `nwg` workgroups resident (one round) and walks each one through every
// nwg-th output tile of the grouped, XCD-aware raster order of gemm.hip:
//   * the LDS-DMA ring is ONE stream across tiles: the last k-step of tile t already issues
//     the first stage of tile t+1, so its load latency hides behind the MFMAs of tile t and the
//     epilogue of tile t (no cold prologue per tile, no new-workgroup launch);
//   * the epilogue never touches the ring: MFMA operands are swapped (D = B^T.A^T), so a lane's
//     accumulator fragment holds 4 CONSECUTIVE output columns of one row; bias, activation /
//     activation-derivative (read straight from the stored activation) and the bf16 rounding
//     happen in registers, and v_permlane16_swap pairs two fragments into one 16-byte row
//     chunk per lane (guide T21, 16-lane form) -- stores go out while the next tile's first
//     stage is in flight;
//   * bias-gradient column sums (dgrad) are reduced over the tile's rows with DPP row
//     butterflies and across waves in the ring slot just consumed, in a fixed order (bitwise
//     reproducible); the kernel needs no LDS beyond the ring.
// The fused softmax cross-entropy needs whole rows in LDS and stays on gemm.hip.
//
// Reference parity: the forward is /root/reference/src/grpc_node.py:87 (z = x.W + b) with the
// activation of :62-73 fused; backward GEMMs have no reference counterpart (centralised
// training only: /root/reference/scripts/generate_mnist_pytorch.py:41-52).
#include <mutex>
#include <unordered_map>

#include "gemm_tile.hpp"

namespace dnn {

struct TileCoord {
  int tm, tn, split, kbase, nk;
};

// Logical tile t of the launch (split-major, grouped raster inside a split; same order as
// gemm_bf16_kernel) -> coordinates and k-range.
__device__ __forceinline__ TileCoord decode_tile(const GemmParams& p, int t, int tiles_n,
                                                 int tiles_m, int splits) {
  const int per_split = tiles_n * tiles_m;
  TileCoord c;
  c.split = t / per_split;
  const int r = t - c.split * per_split;
  const int gm_full = p.group_m > 1 ? p.group_m : 1;
  const int per_group = gm_full * tiles_n;
  const int grp = r / per_group, first_m = grp * gm_full;
  const int gm = min(tiles_m - first_m, gm_full);
  const int tin = r - grp * per_group;
  c.tm = first_m + tin % gm;
  c.tn = tin / gm;
  if (p.k_total > 0) {
    const int KS = p.k_total >> 6;
    const int a = (int)((long)c.split * KS / splits), b = (int)((long)(c.split + 1) * KS / splits);
    c.kbase = a * 64;
    c.nk = b - a;
  } else {
    c.kbase = c.split * p.K;
    c.nk = p.K >> 6;
  }
  return c;
}

template <class C, int LA, int LB, bool OUT_F32>
__global__ __launch_bounds__(C::NT) void gemm_persist_kernel(GemmParams p, int tiles_n,
                                                             int tiles_m, int splits, int nwg) {
  constexpr int BM = C::BM, BN = C::BN, NS = C::NS, FM = C::FM, FN = C::FN;
  constexpr int STAGE = C::STAGE, A_BYTES = C::A_BYTES, RING = NS * STAGE;
  static_assert(FN % 2 == 0, "fragment pairs for the 16-byte epilogue stores");
  static_assert(C::WM * BN * 4 <= STAGE, "colsum partials fit in one ring slot");
  // LDS = the ring only (as gemm.hip: e.g. two 80-KiB 256x64 workgroups share a CU); the
  // colsum cross-wave partials borrow the ring slot the tile's last k-step just consumed
  __shared__ __attribute__((aligned(16))) char smem[RING];
  char LDS_AS* lds = (char LDS_AS*)smem;

  // Round-robin tile assignment: in round r workgroup w takes tile r * nwg + w, so the tiles
  // in flight at any time are consecutive in the raster (the L2 sharing of gemm.hip's grouped
  // order is kept); the XCD remap gives each XCD a contiguous slice of every round.
  const int w = xcd_remap(blockIdx.x, nwg);
  const int total = tiles_n * tiles_m * splits;
  const int t_begin = w, t_end = total;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;

  // ---- load cursor: (tile lt, k-step lk) of the next stage to stage into the ring ----------
  int lt = t_begin, lk = 0;
  TileCoord lc = decode_tile(p, lt, tiles_n, tiles_m, splits);
  int issued = 0, consumed = 0;
  auto issue = [&](char LDS_AS* dst) {
    const int k0 = lc.kbase + lk * 64;
    stage_tile<LA, BM, C::NW>(p.A, p.lda, lc.tm * BM, k0, dst, wave, lane, p.M);
    stage_tile<LB, BN, C::NW>(p.B, p.ldb, lc.tn * BN, k0, dst + A_BYTES, wave, lane, p.N);
    ++issued;
    if (++lk == lc.nk) {
      lk = 0;
      if ((lt += nwg) < t_end) lc = decode_tile(p, lt, tiles_n, tiles_m, splits);
    }
  };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (lt < t_end) issue(lds + s * STAGE);
  int rd = 0, wr = NS - 1;

  // the previous tile's epilogue was a full bf16 tile: exactly epilogue_direct_stores() stores
  // per lane were issued after the next stage's DMA, so waiting for that stage need not drain
  // them (the stores of tile t overlap the first k-steps of tile t + 1)
  bool prev_full_bf16 = false;
  for (int t = t_begin; t < t_end; t += nwg) {
    const TileCoord cc = decode_tile(p, t, tiles_n, tiles_m, splits);
    f32x4_t acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < cc.nk; ++kt) {
      // the first step of a tile follows an epilogue whose stores also count in vmcnt
      if (kt == 0) {
        if (prev_full_bf16 && NS == 2) wait_vmcnt<epilogue_direct_stores<FM, FN>()>();
        else wait_vmcnt<0>();
      } else {
        wait_stage<NS, C::PER_STAGE>(min(issued - consumed - 1, NS - 2));
      }
      lds_barrier();
      if (lt < t_end) issue(lds + wr * STAGE);
      const char LDS_AS* sa = lds + rd * STAGE;
      const char LDS_AS* sb = sa + A_BYTES;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8_t a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = load_frag<LA, BM>(sa, wm * FM + i, s, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = load_frag<LB, BN>(sb, wn * FN + j, s, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)  // swapped operands: lane holds C[row][4 consecutive cols]
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      }
      ++consumed;
      rd = rd + 1 == NS ? 0 : rd + 1;
      wr = wr + 1 == NS ? 0 : wr + 1;
    }

    epilogue_direct<C::FM, C::FN, BN, C::SN, C::WM, NS, STAGE, OUT_F32>(
        p, acc, lds, rd, cc.tm, cc.tn, cc.split, wm, wn, lane, true);
    prev_full_bf16 = !OUT_F32 && (cc.tm + 1) * BM <= p.M && (cc.tn + 1) * BN <= p.N;
  }
}

typedef void (*persist_fn)(GemmParams, int, int, int, int);

template <class C>
static persist_fn pick_layout_p(int la, int lb, int f32) {
#define DNN_P(LA, LB, F) gemm_persist_kernel<C, LA, LB, F>
  if (la == KMAJ && lb == KMAJ) return f32 ? DNN_P(KMAJ, KMAJ, true) : DNN_P(KMAJ, KMAJ, false);
  if (la == KMAJ && lb == MNMAJ) return f32 ? DNN_P(KMAJ, MNMAJ, true) : DNN_P(KMAJ, MNMAJ, false);
  if (la == MNMAJ && lb == KMAJ) return f32 ? DNN_P(MNMAJ, KMAJ, true) : DNN_P(MNMAJ, KMAJ, false);
  return f32 ? DNN_P(MNMAJ, MNMAJ, true) : DNN_P(MNMAJ, MNMAJ, false);
#undef DNN_P
}

// Resident workgroups per CU of a kernel (registers + LDS), cached per kernel.
static int resident_per_cu(persist_fn fn, int nt) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find((const void*)fn);
  if (it != cache.end()) return it->second;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)fn, nt, 0) != hipSuccess ||
      occ < 1)
    occ = 1;
  cache[(const void*)fn] = occ;
  return occ;
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
  }
  return n;
}

// Called by gemm_bf16 after validation (persist != 0): persist > 0 = workgroup count,
// persist < 0 = one full round of resident workgroups (CUs x occupancy).
int gemm_persist_launch(const GemmParams& q, int la, int lb, int out_f32, int bm, int bn,
                        int splits, int ns, int persist, hipStream_t stream) {
  persist_fn fn;
  if (bm == 128 && bn == 128)
    fn = ns == 2 ? pick_layout_p<Cfg<128, 128, 2, 2, 2>>(la, lb, out_f32)
                 : pick_layout_p<Cfg<128, 128, 2, 2, 3>>(la, lb, out_f32);
  else if (bm == 128 && bn == 64)
    fn = ns == 2 ? pick_layout_p<Cfg<128, 64, 2, 2, 2>>(la, lb, out_f32)
                 : pick_layout_p<Cfg<128, 64, 2, 2, 3>>(la, lb, out_f32);
  else if (bm == 64 && bn == 128)
    fn = ns == 2 ? pick_layout_p<Cfg<64, 128, 2, 2, 2>>(la, lb, out_f32)
                 : pick_layout_p<Cfg<64, 128, 2, 2, 3>>(la, lb, out_f32);
  else if (bm == 64 && bn == 64)
    fn = ns == 2 ? pick_layout_p<Cfg<64, 64, 2, 2, 2>>(la, lb, out_f32)
                 : pick_layout_p<Cfg<64, 64, 2, 2, 3>>(la, lb, out_f32);
  else if (bm == 256 && bn == 256)
    fn = pick_layout_p<Cfg<256, 256, 4, 2, 2>>(la, lb, out_f32);
  else if (bm == 256 && bn == 128)
    fn = pick_layout_p<Cfg<256, 128, 4, 2, 2>>(la, lb, out_f32);
  else if (bm == 256 && bn == 64)
    fn = pick_layout_p<Cfg<256, 64, 4, 2, 2>>(la, lb, out_f32);
  else
    fn = pick_layout_p<Cfg<128, 256, 2, 4, 2>>(la, lb, out_f32);
  const int nt = gemm_tile_threads(bm, bn);
  const int tiles_n = (q.N + bn - 1) / bn, tiles_m = (q.M + bm - 1) / bm;
  const long total = (long)tiles_n * tiles_m * splits;
  long nwg = persist > 0 ? persist : (long)num_cus() * resident_per_cu(fn, nt);
  if (nwg > total) nwg = total;
  hipLaunchKernelGGL(fn, dim3((unsigned)nwg), dim3(nt), 0, stream, q, tiles_n, tiles_m, splits,
                     (int)nwg);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

}  // namespace dnn
