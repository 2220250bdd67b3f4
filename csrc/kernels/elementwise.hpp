// Host-visible launchers of csrc/kernels/elementwise.hip. All return 0 on success and a
// negative code (nothing launched) when a host-side precondition fails.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dnn {

// loss_part: one fp32 partial per block (softmax_xent_blocks(rows) entries); colsum (optional):
// per-block column sums of dz ([blocks][ld_colsum]) = bias-gradient partials of the last layer
int softmax_xent(const float* logits, long ld_logits, const int* labels, uint16_t* dz, long ld_dz,
                 int rows, int n_cls, int width, float scale, float* loss_part, int* correct,
                 float* colsum, long ld_colsum, hipStream_t stream);
int softmax_xent_blocks(int rows);
int softmax_rows(const float* logits, long ld_in, float* out, long ld_out, int rows, int n_cls,
                 const int* labels, int* pred, int* correct, hipStream_t stream);
// x = act'(aux) * x in place, then colsum_partial of the result (library-GEMM dgrad epilogue).
int dact_colsum(uint16_t* x, long ld, const uint16_t* aux, long ld_aux, int act, int rows,
                int cols, int n_part, float* part, hipStream_t stream);
int colsum_partial(const uint16_t* x, long ld, int rows, int cols, int n_part, float* part,
                   hipStream_t stream);
int reduce_slabs(const float* src, long stride, int n_src, long n, float scale, float* out,
                 int accumulate, hipStream_t stream);
// One reduction of reduce_multi: out[i] (+)= scale * sum_{s < n_src} src[s * stride + i].
struct ReduceJob {
  const float* src;
  long stride;
  long n;  // multiple of 4
  float* out;
  int n_src;
  float scale;
  int accumulate;
  // Optional (fused-SGD launches only): the job's output is a [n / wt_cols][wt_cols] weight
  // gradient whose layer keeps a transposed bf16 shadow W^T[wt_cols][n / wt_cols]; the update
  // writes it too (bitwise the transpose of the refreshed shadow), so no transpose launch
  // follows the step's update.
  uint16_t* wt;
  int wt_cols;
};
constexpr int REDUCE_MAX_JOBS = 16;
struct ReduceJobs {  // passed by value as the kernel argument
  ReduceJob job[REDUCE_MAX_JOBS];
  int block_start[REDUCE_MAX_JOBS + 1];
  int n_jobs;
};
// Optional SGD fused into reduce_multi: every reduced gradient element out[k] (an element of
// the flat gradient starting at grad_base) also updates master / momentum / bf16 shadow at the
// same flat offset -- bitwise identical to reduce_multi followed by sgd_update over the
// covered elements (one launch and one gradient round trip fewer per step).
struct FusedSgd {
  const float* grad_base;
  float* master;
  float* mom;        // nullptr: no momentum (Adam: the first moment)
  uint16_t* shadow;  // nullptr: no bf16 refresh
  float lr, mu, wd;
  const float* lr_dev;  // optional device-resident learning rate
  // Adam / AdamW instead of SGD (adam != 0), the math of adam_update: v = second moment,
  // bias corrections from step_dev (t = *step_dev + 1, double pow) or bc1 / bc2.
  int adam;
  float* v;
  float b1, b2, eps;
  int decoupled;
  const int* step_dev;
  double db1, db2;
  float bc1, bc2;
};
// All jobs in one launch, each bitwise identical to reduce_slabs on the same inputs.
// max_blocks > 0: at most that many workgroups, each looping over the launch's blocks (the
// same per-output arithmetic; a reduction running beside other kernels then occupies fewer
// CUs).
int reduce_multi(const ReduceJob* job, int n_jobs, hipStream_t stream,
                 const FusedSgd* sgd = nullptr, int max_blocks = 0);
// lr_dev / step_dev (optional, device memory): see the kernels in elementwise.hip.
int sgd_update(float* p, const float* g, float* mom, uint16_t* shadow, long n, float lr, float mu,
               float wd, hipStream_t stream, const float* lr_dev = nullptr);
int adam_update(float* p, const float* g, float* m, float* v, uint16_t* shadow, long n, float lr,
                float b1, float b2, float eps, float wd, int decoupled, float bc1, float bc2,
                hipStream_t stream, const float* lr_dev = nullptr, const int* step_dev = nullptr,
                double db1 = 0.9, double db2 = 0.999);
// *step += 1 (one thread): advances a device-side optimizer step counter.
int step_advance(int* step, hipStream_t stream);
int pack_bf16(const float* in, long ld_in, int rows, int cols, uint16_t* out, long ld_out,
              int rows_p, int cols_p, hipStream_t stream);
int unpack_bf16(const uint16_t* in, long ld_in, int rows, int cols, float* out, long ld_out,
                hipStream_t stream);

constexpr int TRANSPOSE_MAX_JOBS = 16;
struct TransposeJobs {
  const uint16_t* src[TRANSPOSE_MAX_JOBS];
  uint16_t* dst[TRANSPOSE_MAX_JOBS];
  long ld_src[TRANSPOSE_MAX_JOBS], ld_dst[TRANSPOSE_MAX_JOBS];
  int tiles_c[TRANSPOSE_MAX_JOBS];
  int start[TRANSPOSE_MAX_JOBS + 1];  // first 64x64 tile (= workgroup) of each job
  int n;
};
// Every job of transpose_bf16 in one launch (jobs validated by the caller: see bindings).
int transpose_multi(const TransposeJobs& jobs, hipStream_t stream);
// dst[c][r] = src[r][c] for a bf16 [rows][cols] matrix (rows, cols multiples of 64).
int transpose_bf16(const uint16_t* src, long ld_src, int rows, int cols, uint16_t* dst,
                   long ld_dst, hipStream_t stream);

// fp8 (OCP e4m3) pipeline boundary: row-wise amax scaling; q [rows][ldq] bytes, scale [rows].
int quant_rows_fp8(const uint16_t* x, long ldx, int rows, int cols, unsigned char* q, long ldq,
                   float* scale, hipStream_t stream);
int dequant_rows_fp8(const unsigned char* q, long ldq, const float* scale, int rows, int cols,
                     uint16_t* x, long ldx, hipStream_t stream);

// out = act(in + bias) as bf16 (row-parallel layer epilogue after the all-reduce).
int bias_act_cast(const float* in, long ld_in, const float* bias, int act, uint16_t* out,
                  long ld_out, int rows, int cols, hipStream_t stream);
// Peer copy (16-byte aligned) and flag write as kernels: never block the issuing host thread.
int p2p_copy(void* dst, const void* src, size_t bytes, hipStream_t stream);
int p2p_signal(uint32_t* flag, uint32_t value, hipStream_t stream);
// Device-sequence flag protocol (graph-capturable): seq advanced in-stream, signal writes
// *seq + delta, wait spins until flag >= *seq + delta or times out (sets *err).
int p2p_seq_advance(uint32_t* seq, hipStream_t stream);
int p2p_signal_seq(uint32_t* flag, const uint32_t* seq, int delta, hipStream_t stream);
int p2p_wait_seq(const uint32_t* flag, const uint32_t* seq, int delta, uint32_t* err,
                 double timeout_s, hipStream_t stream);

}  // namespace dnn
