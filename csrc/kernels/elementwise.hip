// Memory-bound kernels of the training/inference step (gfx950). All vectorised to 16-byte
// accesses (guide Guideline 13); each one replaces a piece of reference behaviour:
//   softmax_xent   : fused softmax + cross-entropy forward/backward + argmax accuracy
//                    (training replacement of the row softmax in
//                    /root/reference/src/grpc_node.py:68-71 and the CE loss of
//                    /root/reference/scripts/generate_mnist_pytorch.py:37,48)
//   softmax_rows   : inference softmax (grpc_node.py:68-71) + argmax/label compare
//                    (/root/reference/src/run_grpc_inference.py:192-193, 208-209)
//   colsum_partial : bias gradient partial column sums of dZ
//   reduce_slabs   : split-K slab / partial reduction into the flat gradient buffer
//   reduce_multi   : all of a stage's slab / partial reductions in one launch
//   sgd / adam     : fused multi-tensor optimizer over the flat fp32 master buffer, refreshing
//                    the bf16 shadow weights in the same pass
//   pack_bf16      : fp32 host data -> padded bf16 device layout (and back)
#include <algorithm>
#include "common.hpp"
#include "elementwise.hpp"

namespace dnn {

// ------------------------------------------------------------------------------------------
// softmax + cross-entropy. One wave per row, each wave walks XENT_ROWS_PER_WAVE rows, so a
// block covers 4 * XENT_ROWS_PER_WAVE rows (padded width <= 64*NCH columns).
// dz = (softmax(logits) - onehot(label)) * scale in the first n_cls columns, 0 elsewhere.
// Rows whose label is < 0 are padding: dz = 0 and no loss. The block's loss sum goes to
// loss_part[blockIdx.x] (summed later in a fixed order: bitwise reproducible, no float
// atomics); the correct-prediction count likewise goes to correct[blockIdx.x] (written, not
// accumulated, so nothing has to be zeroed per step).
// ------------------------------------------------------------------------------------------
constexpr int XENT_ROWS_PER_WAVE = 16;
constexpr int XENT_ROWS_PER_BLOCK = 4 * XENT_ROWS_PER_WAVE;

template <int NCH>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ logits,
                                                           long ld_logits,
                                                           const int* __restrict__ labels,
                                                           u16* __restrict__ dz, long ld_dz,
                                                           int rows, int n_cls, int width,
                                                           float scale, float* loss_part,
                                                           int* correct, float* colsum,
                                                           long ld_colsum) {
  __shared__ float s_loss[4];
  __shared__ int s_corr[4];
  __shared__ float s_col[4][64 * NCH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = blockIdx.x * XENT_ROWS_PER_BLOCK + wave * XENT_ROWS_PER_WAVE;
  // prefetch every row of this wave first: 16 independent loads in flight instead of 16
  // dependent round trips
  float xs[XENT_ROWS_PER_WAVE][NCH];
  int labs[XENT_ROWS_PER_WAVE];
#pragma unroll
  for (int k = 0; k < XENT_ROWS_PER_WAVE; ++k) {
    const int row = row0 + k;
    const bool ok = row < rows;
    labs[k] = ok ? labels[row] : -1;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 64 + lane;
      xs[k][c] = (ok && col < n_cls) ? logits[(long)row * ld_logits + col] : -INFINITY;
    }
  }
  float loss = 0.f;
  int corr = 0;
  float cs[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) cs[c] = 0.f;
#pragma unroll
  for (int k = 0; k < XENT_ROWS_PER_WAVE; ++k) {
    const int row = row0 + k;
    if (row >= rows) break;
    const int label = labs[k];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < NCH; ++c) mx = fmaxf(mx, xs[k][c]);
    mx = wave_max(mx);
    // argmax: lowest column index holding the max (np.argmax tie rule)
    int amax = 1 << 30;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 64 + lane;
      if (col < n_cls && xs[k][c] == mx) amax = min(amax, col);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = min(amax, __shfl_xor(amax, o, 64));
    float e[NCH], se = 0.f, xl = -INFINITY;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      e[c] = __expf(xs[k][c] - mx);  // exp(-inf) = 0 for padding
      se += e[c];
      if (c * 64 + lane == label) xl = xs[k][c];
    }
    se = wave_sum(se);
    xl = wave_max(xl);
    const float inv = 1.f / se;
    u16* dr = dz + (long)row * ld_dz;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 64 + lane;
      if (col < width) {
        float g = 0.f;
        if (label >= 0 && col < n_cls) g = (e[c] * inv - (col == label ? 1.f : 0.f)) * scale;
        const u16 h = f2bf(g);
        dr[col] = h;
        cs[c] += bf2f(h);
      }
    }
    if (label >= 0 && lane == 0) {
      loss += -(xl - mx - __logf(se));
      corr += amax == label;
    }
  }
  if (lane == 0) {
    s_loss[wave] = loss;
    s_corr[wave] = corr;
  }
  if (colsum) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) s_col[wave][c * 64 + lane] = cs[c];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float l = (s_loss[0] + s_loss[1]) + (s_loss[2] + s_loss[3]);
    const int cc = s_corr[0] + s_corr[1] + s_corr[2] + s_corr[3];
    if (loss_part) loss_part[blockIdx.x] = l;
    if (correct) correct[blockIdx.x] = cc;
  }
  if (colsum) {
    for (int col = threadIdx.x; col < width; col += 256)
      colsum[(long)blockIdx.x * ld_colsum + col] =
          (s_col[0][col] + s_col[1][col]) + (s_col[2][col] + s_col[3][col]);
  }
}

int softmax_xent_blocks(int rows) { return (rows + XENT_ROWS_PER_BLOCK - 1) / XENT_ROWS_PER_BLOCK; }

int softmax_xent(const float* logits, long ld_logits, const int* labels, uint16_t* dz, long ld_dz,
                 int rows, int n_cls, int width, float scale, float* loss_part, int* correct,
                 float* colsum, long ld_colsum, hipStream_t stream) {
  if (rows <= 0 || n_cls <= 0 || n_cls > width || width > 256 || ld_logits < n_cls ||
      ld_dz < width || (colsum && ld_colsum < width))
    return -1;
  const dim3 grid(softmax_xent_blocks(rows)), block(256);
  if (width <= 64)
    hipLaunchKernelGGL(softmax_xent_kernel<1>, grid, block, 0, stream, logits, ld_logits, labels,
                       dz, ld_dz, rows, n_cls, width, scale, loss_part, correct, colsum,
                       ld_colsum);
  else
    hipLaunchKernelGGL(softmax_xent_kernel<4>, grid, block, 0, stream, logits, ld_logits, labels,
                       dz, ld_dz, rows, n_cls, width, scale, loss_part, correct, colsum,
                       ld_colsum);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// Inference softmax over the first n_cls columns (rest zero) + optional argmax correctness.
// ------------------------------------------------------------------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ logits,
                                                           long ld_in, float* __restrict__ out,
                                                           long ld_out, int rows, int n_cls,
                                                           const int* __restrict__ labels,
                                                           int* __restrict__ pred, int* correct) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const float* lr = logits + (long)row * ld_in;
  float x[NCH];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 64 + lane;
    x[c] = col < n_cls ? lr[col] : -INFINITY;
    mx = fmaxf(mx, x[c]);
  }
  mx = wave_max(mx);
  int amax = 1 << 30;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 64 + lane;
    if (col < n_cls && x[c] == mx) amax = min(amax, col);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = min(amax, __shfl_xor(amax, o, 64));
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    x[c] = __expf(x[c] - mx);
    se += x[c];
  }
  se = wave_sum(se);
  const float inv = 1.f / se;
  if (out) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 64 + lane;
      if (col < n_cls) out[(long)row * ld_out + col] = x[c] * inv;
    }
  }
  if (lane == 0) {
    if (pred) pred[row] = amax;
    if (correct && labels && labels[row] == amax) atomicAdd(correct, 1);
  }
}

int softmax_rows(const float* logits, long ld_in, float* out, long ld_out, int rows, int n_cls,
                 const int* labels, int* pred, int* correct, hipStream_t stream) {
  if (rows <= 0 || n_cls <= 0 || n_cls > 256 || ld_in < n_cls || (out && ld_out < n_cls))
    return -1;
  const dim3 grid((rows + 3) / 4), block(256);
  if (n_cls <= 64)
    hipLaunchKernelGGL(softmax_rows_kernel<1>, grid, block, 0, stream, logits, ld_in, out, ld_out,
                       rows, n_cls, labels, pred, correct);
  else
    hipLaunchKernelGGL(softmax_rows_kernel<4>, grid, block, 0, stream, logits, ld_in, out, ld_out,
                       rows, n_cls, labels, pred, correct);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// Column partial sums of a bf16 [rows][ld] matrix (first `cols` columns, cols % 64 == 0).
// Block = 64 columns x (32 row lanes); grid.y = number of partial row blocks. Writes
// part[blockIdx.y][cols]; the optimizer-side reduce_slabs finishes the sum deterministically.
// ------------------------------------------------------------------------------------------
// With `aux` (dact_colsum): x = act'(aux) * x is applied in place first (the library-GEMM
// dgrad's epilogue, csrc/runtime/blaslt.hpp) and the sums are of the stored bf16 values.
template <bool DACT>
__global__ __launch_bounds__(256) void colsum_partial_kernel(u16* __restrict__ x, long ld,
                                                             int rows, int cols, int rows_per,
                                                             float* __restrict__ part,
                                                             const u16* __restrict__ aux,
                                                             long ld_aux, int act) {
  __shared__ float red[32][65];
  const int cc = threadIdx.x & 7;   // 8-column chunk within the 64-column strip
  const int rl = threadIdx.x >> 3;  // row lane 0..31
  const int col0 = blockIdx.x * 64 + cc * 8;
  const int r_begin = blockIdx.y * rows_per;
  const int r_end = min(rows, r_begin + rows_per);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = r_begin + rl; r < r_end; r += 32) {
    bf16x8_t v = *(const bf16x8_t*)(x + (long)r * ld + col0);
    if constexpr (DACT) {
      const bf16x8_t y = *(const bf16x8_t*)(aux + (long)r * ld_aux + col0);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (short)f2bf(act_bwd(bf2f((u16)v[e]), bf2f((u16)y[e]), act));
      *(bf16x8_t*)(x + (long)r * ld + col0) = v;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += bf2f((u16)v[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][cc * 8 + e] = s[e];
  __syncthreads();
  if (threadIdx.x < 64 && part) {
    float t = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) t += red[i][threadIdx.x];
    part[(long)blockIdx.y * cols + blockIdx.x * 64 + threadIdx.x] = t;
  }
}

int colsum_partial(const uint16_t* x, long ld, int rows, int cols, int n_part, float* part,
                   hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || cols % 64 || ld % 8 || ld < cols || n_part <= 0) return -1;
  if (((uintptr_t)x) & 15) return -5;
  const int rows_per = (rows + n_part - 1) / n_part;
  hipLaunchKernelGGL(colsum_partial_kernel<false>, dim3(cols / 64, n_part), dim3(256), 0, stream,
                     const_cast<u16*>(x), ld, rows, cols, rows_per, part, nullptr, 0L, 0);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int dact_colsum(uint16_t* x, long ld, const uint16_t* aux, long ld_aux, int act, int rows,
                int cols, int n_part, float* part, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || cols % 64 || ld % 8 || ld < cols || ld_aux % 8 || n_part <= 0 ||
      !aux)
    return -1;
  if ((((uintptr_t)x) | ((uintptr_t)aux)) & 15) return -5;
  const int rows_per = (rows + n_part - 1) / n_part;
  hipLaunchKernelGGL(colsum_partial_kernel<true>, dim3(cols / 64, n_part), dim3(256), 0, stream,
                     x, ld, rows, cols, rows_per, part, aux, ld_aux, act);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// out[i] (+)= scale * sum_{s < n_src} src[s * stride + i], i < n  (n % 4 == 0)
// Split-K wgrad reductions have few outputs and many sources (up to 128 slabs), so a block is
// TX float4-columns x TY source groups: each thread sums every TY-th slab with 4 independent
// loads in flight, then the TY partials are combined through LDS in a fixed order
// (bitwise reproducible).
// ------------------------------------------------------------------------------------------
template <int TY>
__global__ __launch_bounds__(256) void reduce_slabs_kernel(const float* __restrict__ src,
                                                           long stride, int n_src, long n4,
                                                           float scale, float* __restrict__ out,
                                                           int accumulate) {
  constexpr int TX = 256 / TY;
  __shared__ f32x4_t red[TY][TX];
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  for (long base = (long)blockIdx.x * TX; base < n4; base += (long)gridDim.x * TX) {
    const long i = base + tx;
    f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    if (i < n4) {
      const float* p = src + i * 4;
      int s = ty;
      for (; s + 3 * TY < n_src; s += 4 * TY) {
        a0 += *(const f32x4_t*)(p + (long)s * stride);
        a1 += *(const f32x4_t*)(p + (long)(s + TY) * stride);
        a2 += *(const f32x4_t*)(p + (long)(s + 2 * TY) * stride);
        a3 += *(const f32x4_t*)(p + (long)(s + 3 * TY) * stride);
      }
      for (; s < n_src; s += TY) a0 += *(const f32x4_t*)(p + (long)s * stride);
    }
    red[ty][tx] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (ty == 0 && i < n4) {
      f32x4_t t = red[0][tx];
#pragma unroll
      for (int k = 1; k < TY; ++k) t += red[k][tx];
      t *= scale;
      if (accumulate) t += *(const f32x4_t*)(out + i * 4);
      *(f32x4_t*)(out + i * 4) = t;
    }
    __syncthreads();
  }
}

static int grid_for(long n4) {
  long g = (n4 + 255) / 256;
  return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

// Source groups per block: about DNN_REDUCE_LOADS (16) loads per thread, then the LDS
// combine (headline reduction 24.0 us at 4 loads, 21.7 at 8, 20.3 at 16; step 0.3735 ->
// 0.3661 ms for 4 -> 8 in 4 alternating rounds: profiles/r2_sched/reduce_loads*_ab.jsonl). Few sources -> wide blocks over many columns; many sources
// over few columns (bias partials: 256 x 512) -> up to 64 groups, so no thread walks a long
// dependent chain of load rounds (16 groups left 16 loads per thread on those jobs and 1-2 on
// the 18-slab weight jobs, i.e. 4x the blocks with one load each).
#ifndef DNN_REDUCE_LOADS  // target loads per thread (A/B builds: DNN_HIP_DEFINES)
#define DNN_REDUCE_LOADS 16
#endif
static __host__ __device__ int reduce_ty(int n_src) {
  int ty = 1;
  while (ty < 64 && ty * 2 * DNN_REDUCE_LOADS <= n_src) ty *= 2;
  return ty;
}

int reduce_slabs(const float* src, long stride, int n_src, long n, float scale, float* out,
                 int accumulate, hipStream_t stream) {
  if (n <= 0 || n % 4 || n_src <= 0 || (n_src > 1 && stride % 4)) return -1;
  if ((((uintptr_t)src) | ((uintptr_t)out)) & 15) return -5;
  const long n4 = n / 4;
  const int ty = reduce_ty(n_src);
  long g = (n4 + 256 / ty - 1) / (256 / ty);
  const dim3 grid((unsigned)(g < 8192 ? g : 8192));
#define DNN_SLABS(TY)                                                                          \
  case TY:                                                                                     \
    hipLaunchKernelGGL(reduce_slabs_kernel<TY>, grid, dim3(256), 0, stream, src, stride, n_src, \
                       n4, scale, out, accumulate);                                            \
    break;
  switch (ty) {
    DNN_SLABS(64) DNN_SLABS(32) DNN_SLABS(16) DNN_SLABS(8) DNN_SLABS(4) DNN_SLABS(2)
    default: DNN_SLABS(1)
  }
#undef DNN_SLABS
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// Multi-job reduce: every split-K weight slab set and bias-partial set of a stage in ONE
// launch (they are small and latency-bound: one launch each cost ~5 us). The job table travels
// by value in the kernel arguments; blocks are assigned to jobs by a prefix table, and each
// job runs the TX x TY scheme of reduce_slabs_kernel with its own TY (same fixed summation
// order, so results are bitwise identical to reduce_slabs).
// ------------------------------------------------------------------------------------------
// sgd4 (one SGD step on 4 parameters) lives in common.hpp: shared with the GEMM epilogue.

// One Adam / AdamW step on 4 elements (torch.optim semantics): shared by adam_kernel and the
// fused reduction, so both paths produce the same bits.
__device__ __forceinline__ void adam4(float* __restrict__ p, f32x4_t gv, float* __restrict__ m,
                                      float* __restrict__ v, u16* __restrict__ shadow, float lr,
                                      float b1, float b2, float eps, float wd, int decoupled,
                                      float bc1, float bc2) {
  f32x4_t pv = *(const f32x4_t*)p;
  if (decoupled) pv *= (1.f - lr * wd);
  else gv += wd * pv;
  f32x4_t mv = *(const f32x4_t*)m;
  f32x4_t vv = *(const f32x4_t*)v;
  mv = b1 * mv + (1.f - b1) * gv;
  vv = b2 * vv + (1.f - b2) * gv * gv;
  *(f32x4_t*)m = mv;
  *(f32x4_t*)v = vv;
#pragma unroll
  for (int e = 0; e < 4; ++e) pv[e] -= lr * (mv[e] * bc1) / (sqrtf(vv[e] * bc2) + eps);
  *(f32x4_t*)p = pv;
  if (shadow) {
    bf16x4_t o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(pv[e]);
    *(bf16x4_t*)shadow = o;
  }
}

template <int TY>
__device__ __forceinline__ void reduce_block(const ReduceJob& jb, long blk, f32x4_t LDS_AS* red,
                                             const FusedSgd& sg) {
  constexpr int TX = 256 / TY;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const long i = blk * TX + tx;
  const long n4 = jb.n / 4;
  f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
  if (i < n4) {
    const float* p = jb.src + i * 4;
    const long stride = jb.stride;
    const int n_src = jb.n_src;
    int s = ty;
    for (; s + 3 * TY < n_src; s += 4 * TY) {
      a0 += *(const f32x4_t*)(p + (long)s * stride);
      a1 += *(const f32x4_t*)(p + (long)(s + TY) * stride);
      a2 += *(const f32x4_t*)(p + (long)(s + 2 * TY) * stride);
      a3 += *(const f32x4_t*)(p + (long)(s + 3 * TY) * stride);
    }
    for (; s < n_src; s += TY) a0 += *(const f32x4_t*)(p + (long)s * stride);
  }
  red[ty * TX + tx] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (ty == 0 && i < n4) {
    f32x4_t t = red[tx];
#pragma unroll
    for (int k = 1; k < TY; ++k) t += red[k * TX + tx];
    t *= jb.scale;
    if (jb.accumulate) t += *(const f32x4_t*)(jb.out + i * 4);
    *(f32x4_t*)(jb.out + i * 4) = t;
    if (sg.master) {
      const long off = (jb.out + i * 4) - sg.grad_base;
      const float lr = sg.lr_dev ? *sg.lr_dev : sg.lr;
      if (sg.adam) {
        float bc1 = sg.bc1, bc2 = sg.bc2;
        if (sg.step_dev) {  // the double arithmetic of adam_kernel
          const double tt = (double)(*sg.step_dev + 1);
          bc1 = (float)(1.0 / (1.0 - pow(sg.db1, tt)));
          bc2 = (float)(1.0 / (1.0 - pow(sg.db2, tt)));
        }
        adam4(sg.master + off, t, sg.mom + off, sg.v + off,
              sg.shadow ? sg.shadow + off : nullptr, lr, sg.b1, sg.b2, sg.eps, sg.wd,
              sg.decoupled, bc1, bc2);
      } else {
        sgd4(sg.master + off, t, sg.mom ? sg.mom + off : nullptr,
             sg.shadow ? sg.shadow + off : nullptr, lr, sg.mu, sg.wd);
      }
      if (jb.wt) {  // W^T refresh: this thread's 4 updated weights, read back in bf16
        const bf16x4_t w = *(const bf16x4_t*)(sg.shadow + off);
        const long k = i * 4, rows = jb.n / jb.wt_cols;
        const long r = k / jb.wt_cols, c = k % jb.wt_cols;
#pragma unroll
        for (int e = 0; e < 4; ++e) jb.wt[(c + e) * rows + r] = (u16)w[e];
      }
    }
  }
}

__global__ __launch_bounds__(256) void reduce_multi_kernel(ReduceJobs jobs, FusedSgd sg) {
  __shared__ f32x4_t red_s[256];
  f32x4_t LDS_AS* red = (f32x4_t LDS_AS*)red_s;
  // a workgroup per block, or -- a capped grid (max_blocks) -- every gridDim.x-th block
  const int total = jobs.block_start[jobs.n_jobs];
  for (int vb = blockIdx.x; vb < total; vb += gridDim.x) {  // (uniform per workgroup)
    int j = 0;
    while (j + 1 < jobs.n_jobs && vb >= jobs.block_start[j + 1]) ++j;
    const ReduceJob& jb = jobs.job[j];
    const long blk = (long)vb - jobs.block_start[j];
    switch (reduce_ty(jb.n_src)) {
      case 64: reduce_block<64>(jb, blk, red, sg); break;
      case 32: reduce_block<32>(jb, blk, red, sg); break;
      case 16: reduce_block<16>(jb, blk, red, sg); break;
      case 8: reduce_block<8>(jb, blk, red, sg); break;
      case 4: reduce_block<4>(jb, blk, red, sg); break;
      case 2: reduce_block<2>(jb, blk, red, sg); break;
      default: reduce_block<1>(jb, blk, red, sg); break;
    }
    __syncthreads();  // `red` is rewritten by the next block
  }
}

int reduce_multi(const ReduceJob* job, int n_jobs, hipStream_t stream, const FusedSgd* sgd,
                 int max_blocks) {
  if (n_jobs <= 0 || n_jobs > REDUCE_MAX_JOBS) return -1;
  ReduceJobs J{};
  J.n_jobs = n_jobs;
  int blocks = 0;
  for (int k = 0; k < n_jobs; ++k) {
    const ReduceJob& jb = job[k];
    if (jb.n <= 0 || jb.n % 4 || jb.n_src <= 0 || (jb.n_src > 1 && jb.stride % 4)) return -1;
    if ((((uintptr_t)jb.src) | ((uintptr_t)jb.out)) & 15) return -5;
    J.job[k] = jb;
    J.block_start[k] = blocks;
    const int tx = 256 / reduce_ty(jb.n_src);
    const long b = (jb.n / 4 + tx - 1) / tx;
    if (b > (1L << 30) - blocks) return -1;
    blocks += (int)b;
  }
  J.block_start[n_jobs] = blocks;
  FusedSgd sg{};
  if (sgd) {
    sg = *sgd;
    for (int k = 0; k < n_jobs; ++k)  // every output must lie in the flat gradient, 16-B aligned
      if (job[k].out < sg.grad_base || ((job[k].out - sg.grad_base) & 3)) return -1;
  }
  for (int k = 0; k < n_jobs; ++k)  // W^T needs the fused update (its shadow) and whole rows
    if (job[k].wt && (!sgd || !sg.shadow || job[k].wt_cols <= 0 || job[k].wt_cols % 4 ||
                      job[k].n % job[k].wt_cols))
      return -1;
  const int grid = max_blocks > 0 ? std::min(blocks, max_blocks) : blocks;
  hipLaunchKernelGGL(reduce_multi_kernel, dim3(grid), dim3(256), 0, stream, J, sg);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// Fused SGD (+momentum, +decoupled-from-nothing L2 weight decay like torch.optim.SGD):
//   g' = g + wd * p ; v = mu * v + g' (if mu != 0) ; p -= lr * (v or g') ; shadow = bf16(p)
// ------------------------------------------------------------------------------------------
// lr_dev (optional): learning rate read from device memory, so a recorded/replayed update
// follows an LR schedule without re-recording.
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ mom, u16* __restrict__ shadow,
                                                  long n4, float lr, float mu, float wd,
                                                  const float* __restrict__ lr_dev) {
  if (lr_dev) lr = *lr_dev;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    sgd4(p + i * 4, *(const f32x4_t*)(g + i * 4), mom ? mom + i * 4 : nullptr,
         shadow ? shadow + i * 4 : nullptr, lr, mu, wd);
}

int sgd_update(float* p, const float* g, float* mom, uint16_t* shadow, long n, float lr, float mu,
               float wd, hipStream_t stream, const float* lr_dev) {
  if (n <= 0 || n % 4) return -1;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n / 4)), dim3(256), 0, stream, p, g, mom, shadow,
                     n / 4, lr, mu, wd, lr_dev);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// Adam / AdamW (torch.optim semantics; bc1 = 1/(1-b1^t), bc2 = 1/(1-b2^t)). The corrections
// come from the host, or -- with step_dev -- are computed here in double from the device step
// counter (t = *step_dev + 1; the same double arithmetic as the host path, so both paths
// agree bit for bit) and lr from lr_dev: a recorded update then needs no per-step host values.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   u16* __restrict__ shadow, long n4, float lr,
                                                   float b1, float b2, float eps, float wd,
                                                   int decoupled, float bc1, float bc2,
                                                   const float* __restrict__ lr_dev,
                                                   const int* __restrict__ step_dev, double db1,
                                                   double db2) {
  if (lr_dev) lr = *lr_dev;
  if (step_dev) {
    const double t = (double)(*step_dev + 1);
    bc1 = (float)(1.0 / (1.0 - pow(db1, t)));
    bc2 = (float)(1.0 / (1.0 - pow(db2, t)));
  }
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    adam4(p + i * 4, *(const f32x4_t*)(g + i * 4), m + i * 4, v + i * 4,
          shadow ? shadow + i * 4 : nullptr, lr, b1, b2, eps, wd, decoupled, bc1, bc2);
}

int adam_update(float* p, const float* g, float* m, float* v, uint16_t* shadow, long n, float lr,
                float b1, float b2, float eps, float wd, int decoupled, float bc1, float bc2,
                hipStream_t stream, const float* lr_dev, const int* step_dev, double db1,
                double db2) {
  if (n <= 0 || n % 4) return -1;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4)), dim3(256), 0, stream, p, g, m, v, shadow,
                     n / 4, lr, b1, b2, eps, wd, decoupled, bc1, bc2, lr_dev, step_dev, db1, db2);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

__global__ void step_advance_kernel(int* step) { *step += 1; }

int step_advance(int* step, hipStream_t stream) {
  if (!step) return -1;
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, stream, step);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// fp32 [rows][cols] (ld_in) -> bf16 [rows_p][cols_p] (ld_out) with zero padding, and back.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_bf16_kernel(const float* __restrict__ in, long ld_in,
                                                        int rows, int cols, u16* __restrict__ out,
                                                        long ld_out, int rows_p, int cols_p) {
  const long total = (long)rows_p * cols_p;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int r = (int)(i / cols_p), c = (int)(i % cols_p);
    const float v = (r < rows && c < cols) ? in[(long)r * ld_in + c] : 0.f;
    out[(long)r * ld_out + c] = f2bf(v);
  }
}

int pack_bf16(const float* in, long ld_in, int rows, int cols, uint16_t* out, long ld_out,
              int rows_p, int cols_p, hipStream_t stream) {
  if (rows_p < rows || cols_p < cols || ld_out < cols_p || ld_in < cols) return -1;
  const long total = (long)rows_p * cols_p;
  hipLaunchKernelGGL(pack_bf16_kernel, dim3(grid_for((total + 3) / 4)), dim3(256), 0, stream, in,
                     ld_in, rows, cols, out, ld_out, rows_p, cols_p);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

__global__ __launch_bounds__(256) void unpack_bf16_kernel(const u16* __restrict__ in, long ld_in,
                                                          int rows, int cols,
                                                          float* __restrict__ out, long ld_out) {
  const long total = (long)rows * cols;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    out[(long)r * ld_out + c] = bf2f(in[(long)r * ld_in + c]);
  }
}

int unpack_bf16(const uint16_t* in, long ld_in, int rows, int cols, float* out, long ld_out,
                hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || ld_in < cols || ld_out < cols) return -1;
  hipLaunchKernelGGL(unpack_bf16_kernel, dim3(grid_for(((long)rows * cols + 3) / 4)), dim3(256), 0,
                     stream, in, ld_in, rows, cols, out, ld_out);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// out[r][c] = act(in[r][c] + bias[c]) as bf16: the epilogue of a row-parallel (tensor-parallel)
// layer, applied after the all-reduce of its fp32 partial sums (parallel/tensor.py).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bias_act_cast_kernel(const float* __restrict__ in,
                                                            long ld_in,
                                                            const float* __restrict__ bias,
                                                            int act, u16* __restrict__ out,
                                                            long ld_out, int rows, int cols4) {
  const long total = (long)rows * cols4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int r = (int)(i / cols4), c = (int)(i % cols4) * 4;
    f32x4_t v = *(const f32x4_t*)(in + (long)r * ld_in + c);
    if (bias) v += *(const f32x4_t*)(bias + c);
    bf16x4_t o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(act_fwd(v[e], act));
    *(bf16x4_t*)(out + (long)r * ld_out + c) = o;
  }
}

int bias_act_cast(const float* in, long ld_in, const float* bias, int act, uint16_t* out,
                  long ld_out, int rows, int cols, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || cols % 4 || ld_in % 4 || ld_out % 4) return -1;
  const long total = (long)rows * (cols / 4);
  hipLaunchKernelGGL(bias_act_cast_kernel, dim3(grid_for(total)), dim3(256), 0, stream, in,
                     ld_in, bias, act, out, ld_out, rows, cols / 4);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// bf16 transpose: dst[c][r] = src[r][c], 64x64 tiles through LDS (16-byte loads and stores).
// Refreshes the transposed weight shadow W^T[Kp][Np] after an optimizer update, so the dgrad
// GEMM reads both operands contraction-contiguous (ds_read_b128 fragments, the forward's main
// loop) instead of transposing W with ds_read_b64_tr_b16 in every tile.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void transpose_tile(const u16* __restrict__ src, long ld_src,
                                               u16* __restrict__ dst, long ld_dst, int tiles_c,
                                               int tile) {
  __shared__ u16 t[64][64 + 8];  // +16 B per row: the column reads below hit distinct banks
  const int r0 = (tile / tiles_c) * 64, c0 = (tile % tiles_c) * 64;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int chunk = threadIdx.x + 256 * i, r = chunk >> 3, c = (chunk & 7) * 8;
    const uint4 v = *(const uint4*)(src + (long)(r0 + r) * ld_src + c0 + c);
    const u16* e = (const u16*)&v;
#pragma unroll
    for (int k = 0; k < 8; ++k) t[r][c + k] = e[k];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int chunk = threadIdx.x + 256 * i, c = chunk >> 3, r = (chunk & 7) * 8;
    uint4 v;
    u16* e = (u16*)&v;
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = t[r + k][c];
    *(uint4*)(dst + (long)(c0 + c) * ld_dst + r0 + r) = v;
  }
}

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const u16* __restrict__ src,
                                                             long ld_src, u16* __restrict__ dst,
                                                             long ld_dst, int tiles_c) {
  transpose_tile(src, ld_src, dst, ld_dst, tiles_c, blockIdx.x);
}

// Several transposes in ONE launch (every W^T refresh of a stage after its update: small
// weights are launch-latency bound one by one).
__global__ __launch_bounds__(256) void transpose_multi_kernel(TransposeJobs J) {
  int j = 0;
  while (j + 1 < J.n && (int)blockIdx.x >= J.start[j + 1]) ++j;
  transpose_tile(J.src[j], J.ld_src[j], J.dst[j], J.ld_dst[j], J.tiles_c[j],
                 blockIdx.x - J.start[j]);
}

int transpose_multi(const TransposeJobs& jobs, hipStream_t stream) {
  if (jobs.n <= 0 || jobs.n > TRANSPOSE_MAX_JOBS) return -1;
  hipLaunchKernelGGL(transpose_multi_kernel, dim3(jobs.start[jobs.n]), dim3(256), 0, stream,
                     jobs);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int transpose_bf16(const uint16_t* src, long ld_src, int rows, int cols, uint16_t* dst,
                   long ld_dst, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || rows % 64 || cols % 64) return -1;
  if (ld_src < cols || ld_dst < rows || ld_src % 8 || ld_dst % 8) return -2;
  if ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) return -3;
  const int tiles_c = cols / 64;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((rows / 64) * tiles_c), dim3(256), 0, stream,
                     src, ld_src, dst, ld_dst, tiles_c);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// fp8 pipeline boundary (opt-in): a row of a bf16 activation / gradient is sent as OCP e4m3
// bytes plus one fp32 scale (row amax / 448), halving the bytes on the xGMI hop. One wave per
// row; 8 elements (one 16-byte bf16 load, one 8-byte fp8 store) per lane per iteration.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_amax(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(const u16* __restrict__ x, long ldx,
                                                             int rows, int cols,
                                                             unsigned char* __restrict__ q,
                                                             long ldq, float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // wave-uniform
  const u16* xr = x + (long)row * ldx;
  float amax = 0.f;
  for (int c = lane * 8; c < cols; c += 512) {
    const uint4 v = *(const uint4*)(xr + c);
    const u16* e = (const u16*)&v;
#pragma unroll
    for (int k = 0; k < 8; ++k) amax = fmaxf(amax, fabsf(bf2f(e[k])));
  }
  amax = wave_amax(amax);
  const float s = amax / 448.f, inv = amax > 0.f ? 448.f / amax : 0.f;
  if (lane == 0) scale[row] = s;
  unsigned char* qr = q + (long)row * ldq;
  for (int c = lane * 8; c < cols; c += 512) {
    const uint4 v = *(const uint4*)(xr + c);
    const u16* e = (const u16*)&v;
    unsigned lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(e[0]) * inv, bf2f(e[1]) * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(e[2]) * inv, bf2f(e[3]) * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(e[4]) * inv, bf2f(e[5]) * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(e[6]) * inv, bf2f(e[7]) * inv, hi, true);
    *(uint2*)(qr + c) = make_uint2(lo, hi);
  }
}

__global__ __launch_bounds__(256) void dequant_rows_fp8_kernel(const unsigned char* __restrict__ q,
                                                               long ldq,
                                                               const float* __restrict__ scale,
                                                               int rows, int cols,
                                                               u16* __restrict__ x, long ldx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float s = scale[row];
  const unsigned char* qr = q + (long)row * ldq;
  u16* xr = x + (long)row * ldx;
  for (int c = lane * 8; c < cols; c += 512) {
    const uint2 b = *(const uint2*)(qr + c);
    uint4 out;
    u16* o = (u16*)&out;
    o[0] = f2bf(__builtin_amdgcn_cvt_f32_fp8(b.x, 0) * s);
    o[1] = f2bf(__builtin_amdgcn_cvt_f32_fp8(b.x, 1) * s);
    o[2] = f2bf(__builtin_amdgcn_cvt_f32_fp8(b.x, 2) * s);
    o[3] = f2bf(__builtin_amdgcn_cvt_f32_fp8(b.x, 3) * s);
    o[4] = f2bf(__builtin_amdgcn_cvt_f32_fp8(b.y, 0) * s);
    o[5] = f2bf(__builtin_amdgcn_cvt_f32_fp8(b.y, 1) * s);
    o[6] = f2bf(__builtin_amdgcn_cvt_f32_fp8(b.y, 2) * s);
    o[7] = f2bf(__builtin_amdgcn_cvt_f32_fp8(b.y, 3) * s);
    *(uint4*)(xr + c) = out;
  }
}

int quant_rows_fp8(const uint16_t* x, long ldx, int rows, int cols, unsigned char* q, long ldq,
                   float* scale, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || cols % 8 || ldx < cols || ldq < cols || ldx % 8 || ldq % 8)
    return -1;
  if (((uintptr_t)x & 15) || ((uintptr_t)q & 7)) return -2;
  hipLaunchKernelGGL(quant_rows_fp8_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, x, ldx,
                     rows, cols, q, ldq, scale);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int dequant_rows_fp8(const unsigned char* q, long ldq, const float* scale, int rows, int cols,
                     uint16_t* x, long ldx, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || cols % 8 || ldx < cols || ldq < cols || ldx % 8 || ldq % 8)
    return -1;
  if (((uintptr_t)x & 15) || ((uintptr_t)q & 7)) return -2;
  hipLaunchKernelGGL(dequant_rows_fp8_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, q, ldq,
                     scale, rows, cols, x, ldx);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

// ------------------------------------------------------------------------------------------
// Stream-ordered peer copy and flag write as KERNELS. hipMemcpyAsync / hipStreamWriteValue32
// into IPC-imported memory were measured to block the issuing host thread until the stream's
// earlier work completed (bench/relay_diag.py, DNN_PLAN_TRACE): a rank then cannot enqueue the
// rest of its step (e.g. the relay copies another rank is waiting for) -- a cross-rank
// deadlock, and a host-serialised step even without one. A kernel launch never blocks.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void p2p_copy_kernel(const uint4* __restrict__ src,
                                                       uint4* __restrict__ dst, long n16,
                                                       const unsigned char* __restrict__ src_t,
                                                       unsigned char* __restrict__ dst_t,
                                                       int tail) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256)
    dst[i] = src[i];
  if (blockIdx.x == 0 && (int)threadIdx.x < tail) dst_t[threadIdx.x] = src_t[threadIdx.x];
}

// One lane stores the flag word with system-scope release semantics (a vector store; the
// kernel boundary before it has made the preceding copy's writes visible).
__global__ void p2p_signal_kernel(unsigned* flag, unsigned value) {
  const unsigned l = threadIdx.x;
  if (l == 0) __hip_atomic_store(flag + l, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Device-sequence forms (graph-capturable step plans): the step number lives in device memory
// and is advanced by a kernel at the start of every step, so a captured plan replays with the
// right flag values. The wait spins ONE lane on the flag (system-scope acquire loads, s_sleep
// between polls) and gives up after `timeout_ns`, recording the failure in *err instead of
// hanging the queue: every wave of the kernel always finishes.
__global__ void p2p_seq_advance_kernel(unsigned* seq) {
  const unsigned l = threadIdx.x;
  if (l == 0) seq[l] = seq[l] + 1u;
}

__global__ void p2p_signal_seq_kernel(unsigned* flag, const unsigned* seq, int delta) {
  const unsigned l = threadIdx.x;
  if (l == 0)
    __hip_atomic_store(flag + l, seq[l] + (unsigned)delta, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void p2p_wait_seq_kernel(const unsigned* flag, const unsigned* seq, int delta,
                                    unsigned* err, unsigned long long timeout_ticks) {
  const unsigned l = threadIdx.x;
  if (l != 0) return;
  const unsigned target = seq[l] + (unsigned)delta;
  const unsigned long long t0 = wall_clock64();
  // wrapping step counters: "reached" = (int)(flag - target) >= 0
  while ((int)(__hip_atomic_load(flag + l, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) -
               target) < 0) {
    __builtin_amdgcn_s_sleep(4);
    if (wall_clock64() - t0 > timeout_ticks) {
      __hip_atomic_store(err + l, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
}

int p2p_seq_advance(uint32_t* seq, hipStream_t stream) {
  hipLaunchKernelGGL(p2p_seq_advance_kernel, dim3(1), dim3(64), 0, stream, seq);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int p2p_signal_seq(uint32_t* flag, const uint32_t* seq, int delta, hipStream_t stream) {
  if (reinterpret_cast<uintptr_t>(flag) & 3) return -1;
  hipLaunchKernelGGL(p2p_signal_seq_kernel, dim3(1), dim3(64), 0, stream, flag, seq, delta);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int p2p_wait_seq(const uint32_t* flag, const uint32_t* seq, int delta, uint32_t* err,
                 double timeout_s, hipStream_t stream) {
  if (reinterpret_cast<uintptr_t>(flag) & 3) return -1;
  static int rate_khz = [] {  // wall_clock64 ticks per ms (100 MHz on gfx9)
    int r = 0, dev = 0;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&r, hipDeviceAttributeWallClockRate, dev);
    return r > 0 ? r : 100000;
  }();
  const unsigned long long ticks =
      (unsigned long long)(timeout_s * 1e3 * (double)rate_khz);
  hipLaunchKernelGGL(p2p_wait_seq_kernel, dim3(1), dim3(64), 0, stream, flag, seq, delta, err,
                     ticks);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int p2p_copy(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return 0;
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) return -1;
  const long n16 = (long)(bytes / 16);
  const int tail = (int)(bytes % 16);
  const int grid = (int)std::min<long>(std::max<long>(1, (n16 + 255) / 256), 2048);
  hipLaunchKernelGGL(p2p_copy_kernel, dim3(grid), dim3(256), 0, stream,
                     reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), n16,
                     reinterpret_cast<const unsigned char*>(src) + n16 * 16,
                     reinterpret_cast<unsigned char*>(dst) + n16 * 16, tail);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

int p2p_signal(uint32_t* flag, uint32_t value, hipStream_t stream) {
  if (reinterpret_cast<uintptr_t>(flag) & 3) return -1;
  hipLaunchKernelGGL(p2p_signal_kernel, dim3(1), dim3(64), 0, stream, flag, value);
  return hipGetLastError() == hipSuccess ? 0 : -9;
}

}  // namespace dnn
