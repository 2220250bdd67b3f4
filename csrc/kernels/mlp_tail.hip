// Fused classifier tail: forward of the last two layers, softmax cross-entropy, and the
// dgrads of both layers in ONE launch (interface and math: mlp_tail.hpp).
//
// Why: on the headline 784-512-256-128-10 model the four kernels this replaces (fwd 256->128,
// fwd 128->10 + CE, dgrad 10->128, dgrad 128->256) are all latency-bound -- short contractions,
// one LDS stage in flight, an epilogue that re-reads the activation -- and cost ~63 us of a
// ~370 us step while their data is ~110 MB (23 us of HBM time). Their weights are 64 + 16 KiB,
// so they live in LDS for the whole launch and every intermediate stays on chip.
//
// Structure (one workgroup per CU; 16 waves for the ReLU form, 8 for other activations;
// 16-row blocks dealt round-robin over the workgroups, one per wave at 65536 rows):
//   * W3 [N3][K3] and W4 [64][N3] are staged once into LDS with LDS-DMA, in the MNMAJ image
//     layout of gemm_tile.hpp: the forward reads them row-wise (16-B chunks), the dgrads read
//     them transposed with ds_read_b64_tr_b16 (load_frag<MNMAJ>), so no transposed copy exists;
//   * every product is computed with SWAPPED operands, mfma(W-fragment, X-fragment): a lane
//     then holds 4 consecutive output features of ONE data row (row = lane & 15, features
//     16 j + 4 (lane >> 4) + r), which is the layout of the bias/activation epilogue, of the
//     ReLU derivative of the next dgrad, and of the softmax (a row's 16 class logits sit in 4
//     lanes); global stores pair two such blocks into 16-byte chunks (v_permlane16_swap);
//   * an output that feeds the next product becomes the next MFMA's B fragment in registers
//     (frag_from_out: two lane-group swaps), no LDS round trip;
//   * bias-gradient column sums: DPP row sums per block, accumulated across the wave's blocks
//     in the wave's own LDS row, reduced over the waves in fixed order at the end (one partial
//     per workgroup); softmax and loss follow xent_rows (gemm_tile.hpp) operation for operation.
// Every MFMA chain accumulates its contraction in the same ascending k order as the unfused
// GEMMs, so h3, dz4, dz3 and dz2 equal the unfused path's bit for bit (tests/test_mlp_tail_gpu.py).
//
// Reference parity: the forward is /root/reference/src/grpc_node.py:87 + :62-73 (z = x.W + b,
// activation, softmax); the backward replaces the centralised autograd of
// /root/reference/scripts/generate_mnist_pytorch.py:41-52.
//
// build-flags: -fno-slp-vectorize
// (SLP pairs independent DPP row sums into v_mov_b32_dpp + v_pk_add_f32; without it each step
// folds into one v_add_f32_dpp: -10 % instructions in the loop.)
#include "gemm_tile.hpp"
#include "mlp_tail.hpp"

// Probe builds only (bench/probes/tail_probe.py compiles this file into a separate library with
// -DDNN_TAIL_PROBE=bits to time the kernel with parts removed; results are then wrong): 1 = no
// bias-gradient column sums, 2 = no global stores of H3 / DZ4 / DZ3 / DZ2, 4 = no softmax.
#ifndef DNN_TAIL_PROBE
#define DNN_TAIL_PROBE 0
#endif

namespace dnn {
namespace tail {

// Waves per workgroup of the standalone launch: 16 (four per SIMD, <= 128 registers each) for
// the branch-free ReLU form, so one 16-row block per wave covers 65536 rows in one round and
// four independent block chains share each SIMD; the generic-activation form (runtime
// activation branches, <= 128 registers; not on the benchmarked models) runs 8. (A launch
// fusing the previous layer's forward in front of the tail lost in the step twice, rounds 2
// and 6: profiles/r6_prune/restore_fwd_tail.patch.)
template <bool RELU>
constexpr int waves() { return RELU ? 16 : 8; }
constexpr int MAX_CLS = 16;  // classes held by one 16-wide MFMA block
constexpr int W4_ROWS = 64;  // staged rows of W4 (the dgrad's contraction uses rows 0..31)

// LDS: the two weight images, b3, and one column-sum row per wave. No per-wave scratch: an
// output that feeds the next product is regrouped into that MFMA's B fragment in registers
// (frag_from_out), not written to LDS and read back.
template <int K3, int N3, int NW>
struct Geo {
  static constexpr int W3_BYTES = N3 * K3 * 2;
  static constexpr int W4_BYTES = W4_ROWS * N3 * 2;
  static constexpr int B3_BYTES = N3 * 4;
  static constexpr int RC = K3 + N3 + MAX_CLS + 4;  // per-wave reduction row (floats, 16-B rows)
  static constexpr int SMEM = W3_BYTES + W4_BYTES + B3_BYTES + NW * RC * 4;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(K3 / 16 <= 16 && N3 / 16 <= 16, "column-sum lanes");
};

__device__ __forceinline__ float lo_bf(unsigned x) { return __uint_as_float(x << 16); }
__device__ __forceinline__ float hi_bf(unsigned x) { return __uint_as_float(x & 0xffff0000u); }

// Global store of two 16-column blocks (j, j + 1) of one row as 16-byte chunks: the lanes of
// group q hold columns 4 q .. 4 q + 3 of each block; v_permlane16_swap regroups them so group
// 0 / 1 / 2 / 3 holds columns 0..7 of j / 0..7 of j+1 / 8..15 of j / 8..15 of j+1 (the
// register-direct epilogue of gemm_tile.hpp). `row` points at column 0 of the output row.
__device__ __forceinline__ void st16_pair(u16* row, int j, int q, uint2 a, uint2 b) {
  if constexpr (DNN_TAIL_PROBE & 2) return;
  const auto s0 = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  *(uint4*)(row + 16 * j + 16 * (q & 1) + 8 * (q >> 1)) =
      make_uint4(s0[0], s1[0], s0[1], s1[1]);
}

// Two output blocks of a 16-row block (a: columns 32 s .. 32 s + 15, b: 32 s + 16 .. 32 s + 31;
// lane (i, g) holds row i, 4 columns from 4 g) -> the MFMA B fragment of contraction step s
// (lane (i, g): row i, columns 32 s + 8 g .. 32 s + 8 g + 7). Writing a_g / b_g for the value
// lane group g holds, a 32-lane swap gives {a0 a1 b0 b1 | a2 a3 b2 b3} and a 16-lane swap of
// those {a0 a2 b0 b2 | a1 a3 b1 b3}: group g then holds the first and second 4 of its 8
// columns. Same bf16 values as the LDS write + transposing read it replaces.
__device__ __forceinline__ bf16x8_t frag_from_out(uint2 a, uint2 b) {
  const auto x = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
  const auto y = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
  const auto xs = __builtin_amdgcn_permlane16_swap(x[0], x[1], false, false);
  const auto ys = __builtin_amdgcn_permlane16_swap(y[0], y[1], false, false);
  return __builtin_bit_cast(bf16x8_t, make_uint4(xs[0], ys[0], xs[1], ys[1]));
}

// rw[0..3] += column sums over the 16 rows (lanes of a DPP row) of the 4 bf16 values in v
// (the four butterflies run step-major so consecutive DPP adds are independent: a DPP read of a
// VGPR written by the previous VALU instruction costs wait states)
__device__ __forceinline__ void acc4(float LDS_AS* rw, uint2 v) {
  if constexpr (DNN_TAIL_PROBE & 1) return;
  float x[4] = {lo_bf(v.x), hi_bf(v.x), lo_bf(v.y), hi_bf(v.y)};
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] += dpp_f<0xB1>(x[e]);
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] += dpp_f<0x4E>(x[e]);
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] += dpp_f<0x141>(x[e]);
#pragma unroll
  for (int e = 0; e < 4; ++e) x[e] += dpp_f<0x140>(x[e]);
  f32x4_t t = *(f32x4_t LDS_AS*)rw;
#pragma unroll
  for (int e = 0; e < 4; ++e) t[e] += x[e];
  *(f32x4_t LDS_AS*)rw = t;
}

// Activation / derivative: RELU = both activations are ReLU (the branch-free common case),
// otherwise the runtime Act code (a uniform branch per element).
template <bool RELU>
__device__ __forceinline__ float act(float v, int code) {
  if constexpr (RELU) return v > 0.f ? v : 0.f;
  return act_fwd(v, code);
}
template <bool RELU>
__device__ __forceinline__ float dact(float g, float y, int code) {
  if constexpr (RELU) return y > 0.f ? g : 0.f;
  return act_bwd(g, y, code);
}

// 16-B row chunk `c` of row `r` of an MNMAJ-swizzled [rows][T] image (the forward's A fragment:
// lane holds W[r = 16 blk + (lane & 15)][8 c .. 8 c + 7] with c = 4 s + (lane >> 4)).
template <int T>
__device__ __forceinline__ bf16x8_t row_frag(const char LDS_AS* img, int blk, int s, int lane) {
  const int r = blk * 16 + (lane & 15), c = 4 * s + (lane >> 4);
  return *(const bf16x8_t LDS_AS*)(img + r * (T * 2) + ((c ^ mn_swz<T>(r)) << 4));
}

// 64 rows [r0, r0 + 64) of a [rows][T] bf16 matrix -> the MNMAJ image layout of gemm_tile.hpp
// (stage_tile<MNMAJ>), by LDS-DMA in 1-KiB pieces dealt round-robin to the NW waves (any NW:
// T / 8 pieces need not divide evenly).
template <int T, int NW>
__device__ __forceinline__ void stage_rows64(const u16* __restrict__ g, long ld, int r0,
                                             char LDS_AS* dst, int wave, int lane) {
  constexpr int CPR = T / 8, PIECES = T / 8;  // 16-B chunks per row; 64 rows x 2T B / 1 KiB
  for (int piece = wave; piece < PIECES; piece += NW) {  // uniform per wave
    const int chunk = piece * 64 + lane;
    const int r = chunk / CPR, ph = chunk % CPR;
    const u16* src = g + (long)(r0 + r) * ld + (ph ^ mn_swz<T>(r)) * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, (void LDS_AS*)(dst + piece * 1024), 16, 0,
                                     0);
  }
}

}  // namespace tail

// The whole tail for the 16-row blocks rb = rb_first + wave * wave_stride, + rb_step, ... <
// rb_end of this workgroup (NW waves); its bias-gradient / loss partials go to row `wg` of the
// partial buffers.
template <int K3, int N3, int NW, bool RELU>
__device__ __forceinline__ void tail_body(const TailParams& p, char LDS_AS* lds, int rb_first,
                                          int wave_stride, int rb_step, int rb_end, long wg) {
  using tail::act;
  using tail::dact;
  using tail::frag_from_out;
  using G = tail::Geo<K3, N3, NW>;
  using tail::hi_bf;
  using tail::lo_bf;
  constexpr int NK = K3 / 32, NJ = N3 / 16, NS3 = N3 / 32, NKK = K3 / 16;
  char LDS_AS* w3 = lds;
  char LDS_AS* w4 = lds + G::W3_BYTES;
  float LDS_AS* b3s = (float LDS_AS*)(w4 + G::W4_BYTES);
  float LDS_AS* red = b3s + N3;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- weights -> LDS (64-row pieces of the MNMAJ image, LDS-DMA); b3 -> LDS ---------------
#pragma unroll
  for (int r0 = 0; r0 < N3; r0 += 64)
    tail::stage_rows64<K3, NW>(p.W3, p.ldw3, r0, w3 + r0 * K3 * 2, wave, lane);
  tail::stage_rows64<N3, NW>(p.W4, p.ldw4, 0, w4, wave, lane);
  for (int c = threadIdx.x; c < N3; c += NW * 64) b3s[c] = p.b3[c];

  const int i16 = lane & 15, q = lane >> 4;
  const int nrb = rb_end;
  const int nw = rb_step;
  int rb = rb_first + wave * wave_stride;

  float b4r[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) b4r[e] = p.b4[4 * q + e];

  // column sums accumulate in this wave's row of `red` (zeroed here; only this wave touches it
  // until the final barrier). A DPP row sum leaves the same bits in all 16 lanes of the row, so
  // all of them read-add-write the same 16-B slot: no lane masks, no registers per column.
  float LDS_AS* rw = red + wave * G::RC;
  for (int c = lane; c < G::RC; c += 64) rw[c] = 0.f;
  float loss_a = 0.f;
  int corr_a = 0;
  const int nc = p.n_cls;
  __syncthreads();  // weights and b3 landed (the fence waits for the LDS-DMA loads too)

  for (; rb < nrb; rb += nw) {
    // The lane index is laundered through an empty asm per block, so the dozens of fragment
    // and store addresses derived from it are recomputed in the body instead of hoisted out of
    // the block loop (live across it, they spill a 128-register wave; most waves run the body
    // once anyway).
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int i16 = ln & 15, q = ln >> 4;
    const long row = (long)rb * 16 + i16;
    const int label = p.labels[row];
    // this block's rows as the forward's B fragments (one block per wave at the headline size:
    // a prefetch of the next block would only hold 32 registers through the whole body)
    bf16x8_t xb[NK];
#pragma unroll
    for (int s = 0; s < NK; ++s) xb[s] = *(const bf16x8_t*)(p.X + row * p.ldx + 8 * q + 32 * s);

    // ---- h3 = act3(X . W3^T + b3) -------------------------------------------------------
    // (one output block at a time, fenced: with all 8 in flight the scheduler hoists their 64
    // weight-fragment reads and a 128-register wave spills)
    uint2 h3p[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      f32x4_t a3 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NK; ++s)
        a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tail::row_frag<K3>(w3, j, s, ln), xb[s], a3,
                                                     0, 0, 0);
      const f32x4_t b3 = *(const f32x4_t LDS_AS*)(b3s + 16 * j + 4 * q);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = act<RELU>(a3[e] + b3[e], p.act3);
      h3p[j] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      if (j & 1) tail::st16_pair(p.H3 + row * p.ldh3, j - 1, q, h3p[j - 1], h3p[j]);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- logits (classes 0..15) = h3 . W4^T + b4; softmax cross-entropy ------------------
    f32x4_t a4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS3; ++s)
      a4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tail::row_frag<N3>(w4, 0, s, ln),
                                                   frag_from_out(h3p[2 * s], h3p[2 * s + 1]), a4,
                                                   0, 0, 0);
    float lv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) lv[e] = a4[e] + b4r[e];
    float dz[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (DNN_TAIL_PROBE & 4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dz[e] = lv[e] * p.scale;
    } else {
      float vals[tail::MAX_CLS];
#pragma unroll
      for (int c = 0; c < tail::MAX_CLS; ++c) vals[c] = __shfl(lv[c & 3], i16 + 16 * (c >> 2), 64);
      float mx = -INFINITY;
      int amax = 0;
#pragma unroll
      for (int c = 0; c < tail::MAX_CLS; ++c)
        if (c < nc && vals[c] > mx) {
          mx = vals[c];
          amax = c;
        }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < tail::MAX_CLS; ++c)
        if (c < nc) se += __expf(vals[c] - mx);
      const float inv = 1.f / se;
      if (label >= 0) {
        float vl = 0.f;
#pragma unroll
        for (int c = 0; c < tail::MAX_CLS; ++c)
          if (c == label) vl = vals[c];
        if (q == 0) {
          loss_a += -(vl - mx - __logf(se));
          corr_a += amax == label;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * q + e;
          if (c < nc) dz[e] = (__expf(lv[e] - mx) * inv - (c == label ? 1.f : 0.f)) * p.scale;
        }
      }
    }
    const uint2 d4 = make_uint2(pack_bf16x2(dz[0], dz[1]), pack_bf16x2(dz[2], dz[3]));
    // the 16 class columns only (8 bytes per lane, 32 contiguous per row): the padding columns
    // are constant zero, left as the caller zeroed them (mlp_tail.hpp), 48 of 64 columns of
    // writes less per row
    if constexpr (!(DNN_TAIL_PROBE & 2)) *(uint2*)(p.DZ4 + row * p.lddz4 + 4 * q) = d4;
    tail::acc4(rw + K3 + N3 + 4 * q, d4);

    // ---- dz3 = (dz4 . W4) * act3'(h3): contraction over classes 0..31 -------------------
    const bf16x8_t df = frag_from_out(d4, make_uint2(0u, 0u));
    uint2 o3[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const f32x4_t a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
          load_frag<MNMAJ, N3>(w4, j, 0, ln), df, f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const float y[4] = {lo_bf(h3p[j].x), hi_bf(h3p[j].x), lo_bf(h3p[j].y), hi_bf(h3p[j].y)};
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = dact<RELU>(a[e], y[e], p.act3);
      o3[j] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      if (j & 1) tail::st16_pair(p.DZ3 + row * p.lddz3, j - 1, q, o3[j - 1], o3[j]);
      tail::acc4(rw + K3 + 16 * j + 4 * q, o3[j]);
      if (j & 1) __builtin_amdgcn_sched_barrier(0);
    }

    // ---- dz2 = (dz3 . W3) * act2'(X) ------------------------------------------------------
    bf16x8_t d3f[NS3];
#pragma unroll
    for (int s = 0; s < NS3; ++s) d3f[s] = frag_from_out(o3[2 * s], o3[2 * s + 1]);
    uint2 prev = make_uint2(0u, 0u);
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS3; ++s)
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(load_frag<MNMAJ, K3>(w3, kk, s, ln), d3f[s],
                                                    a, 0, 0, 0);
      // activation of layer L-3 at this lane's dz2 positions, read per output block (held
      // through the body, these 32 registers would spill a 128-register wave; the other waves
      // of the SIMD cover the load)
      const uint2 hv = *(const uint2*)(p.X + row * p.ldx + 16 * kk + 4 * q);
      const float y[4] = {lo_bf(hv.x), hi_bf(hv.x), lo_bf(hv.y), hi_bf(hv.y)};
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = dact<RELU>(a[e], y[e], p.act2);
      const uint2 o = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      if (kk & 1) tail::st16_pair(p.DZ2 + row * p.lddz2, kk - 1, q, prev, o);
      prev = o;
      tail::acc4(rw + 16 * kk + 4 * q, o);
      if (kk & 1) __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---- per-workgroup partials: the NW waves' column sums / loss / correct, fixed order ------
  loss_a = wave_sum(loss_a);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) corr_a += __shfl_xor(corr_a, o, 64);
  if (lane == 0) {
    rw[K3 + N3 + tail::MAX_CLS] = loss_a;
    rw[K3 + N3 + tail::MAX_CLS + 1] = (float)corr_a;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < K3 + N3 + tail::MAX_CLS + 2; c += NW * 64) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[w * G::RC + c];
    if (c < K3) p.cs2[wg * p.ld_cs2 + c] = t;
    else if (c < K3 + N3) p.cs3[wg * p.ld_cs3 + c - K3] = t;
    else if (c < K3 + N3 + tail::MAX_CLS) p.cs4[wg * p.ld_cs4 + c - K3 - N3] = t;
    else if (c == K3 + N3 + tail::MAX_CLS) {
      if (p.loss_part) p.loss_part[wg] = t;
    } else if (p.correct) {
      p.correct[wg] = (int)t;
    }
  }
  for (int c = tail::MAX_CLS + (int)threadIdx.x; c < p.N4; c += NW * 64)
    p.cs4[wg * p.ld_cs4 + c] = 0.f;
}

template <int K3, int N3, bool RELU>
__global__ __launch_bounds__(64 * tail::waves<RELU>()) void mlp_tail_kernel(TailParams p) {
  constexpr int NW = tail::waves<RELU>();
  __shared__ __attribute__((aligned(16))) char smem[tail::Geo<K3, N3, NW>::SMEM];
  // block rb -> workgroup rb % grid, wave (rb / grid) % NW: a launch of fewer blocks than
  // waves still spreads them over every workgroup (CU)
  tail_body<K3, N3, NW, RELU>(p, (char LDS_AS*)smem, blockIdx.x, gridDim.x, gridDim.x * NW,
                              p.M >> 4, blockIdx.x);
}

int mlp_tail_blocks(int M) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  // one workgroup per 16-row block up to one per CU (blocks are dealt round-robin)
  const int blocks = (M + 15) / 16;
  return blocks < cus ? (blocks > 0 ? blocks : 1) : cus;
}

const char* mlp_tail_error(int code) {
  switch (code) {
    case -1: return "mlp_tail: rows must be a positive multiple of 16";
    case -2: return "mlp_tail: unsupported widths (K3 in {64,128,256}, N3 in {64,128})";
    case -3: return "mlp_tail: classes must be 1..16 with 64 or 128 padded columns";
    case -4: return "mlp_tail: operand rows/columns must be 16-byte aligned";
    case -9: return "mlp_tail: kernel launch failed";
    default: return "mlp_tail: unknown error";
  }
}

int mlp_tail(const TailParams& p, hipStream_t stream) {
  if (p.M <= 0 || p.M % 16) return -1;
  if (p.n_cls < 1 || p.n_cls > tail::MAX_CLS || (p.N4 != 64 && p.N4 != 128)) return -3;
  const long lds[] = {p.ldx, p.ldw3, p.ldw4, p.ldh3, p.lddz4, p.lddz3, p.lddz2};
  for (long l : lds)
    if (l % 8) return -4;
  typedef void (*fn_t)(TailParams);
  fn_t fn = nullptr;
  const bool relu = p.act3 == ACT_RELU && p.act2 == ACT_RELU;
#define DNN_TAIL(K, N) \
  if (p.K3 == K && p.N3 == N) fn = relu ? mlp_tail_kernel<K, N, true> : mlp_tail_kernel<K, N, false>;
  DNN_TAIL(64, 64)
  DNN_TAIL(128, 64)
  DNN_TAIL(256, 64)
  DNN_TAIL(64, 128)
  DNN_TAIL(128, 128)
  DNN_TAIL(256, 128)
#undef DNN_TAIL
  if (!fn) return -2;
  hipLaunchKernelGGL(fn, dim3(mlp_tail_blocks(p.M)), dim3(64 * (relu ? tail::waves<true>()
                                                                 : tail::waves<false>())),
                     0, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

}  // namespace dnn
