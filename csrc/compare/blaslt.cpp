// hipBLASLt library GEMMs (interface: blaslt.hpp).
#include "runtime/blaslt.hpp"

#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

namespace dnn {
namespace {

constexpr int MAX_ALGOS = 8;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
  bool ok = false;
  hipblasLtMatmulHeuristicResult_t cand[MAX_ALGOS];  // the heuristic's candidates
  int n_cand = 0;
};

using Key = std::tuple<int, int, int, int, int, long, long, long, int, int, int, int>;

std::mutex mu;
hipblasLtHandle_t handle = nullptr;
std::map<Key, Plan> plans;
std::map<hipStream_t, std::pair<void*, size_t>> workspaces;
constexpr size_t MAX_WS = 64ull << 20;

bool init() {
  if (handle) return true;
  return hipblasLtCreate(&handle) == HIPBLAS_STATUS_SUCCESS;
}

// Column-major view of the row-major problem: D^T[N][M] = op(B)^T . op(A)^T, so the library's
// "A" is our B and its "B" is our A.
Plan* plan_for(const BlasGemm& g) {
  const bool has_bias = g.bias != nullptr;
  Key k{g.trans_a, g.trans_b, g.M, g.N, g.K, g.lda, g.ldb, g.ldd, g.d_f32, has_bias, g.relu,
        g.accumulate};
  auto it = plans.find(k);
  if (it != plans.end()) return &it->second;
  Plan& p = plans[k];
  const hipDataType dt = g.d_f32 ? HIP_R_32F : HIP_R_16BF;
  // library A = our B: row-major [K][N] (trans_b 0) is column-major [N][K] -> op N;
  // row-major [N][K] (trans_b 1) is column-major [K][N] -> op T.
  hipblasOperation_t opa = g.trans_b ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  // library B = our A: row-major [M][K] (trans_a 0) is column-major [K][M] -> op N;
  // row-major [K][M] (trans_a 1) is column-major [M][K] -> op T.
  hipblasOperation_t opb = g.trans_a ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
    return &p;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb));
  if (has_bias) {
    hipblasLtEpilogue_t epi = g.relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
    hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    const void* bp = g.bias;  // patched per call
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp));
  } else if (g.relu) {
    hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_RELU;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  }
  // stored (column-major) shapes
  const uint64_t a_rows = g.trans_b ? g.K : g.N, a_cols = g.trans_b ? g.N : g.K;
  const uint64_t b_rows = g.trans_a ? g.M : g.K, b_cols = g.trans_a ? g.K : g.M;
  if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, a_rows, a_cols, g.ldb) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, b_rows, b_cols, g.lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.ld, dt, g.N, g.M, g.ldd) != HIPBLAS_STATUS_SUCCESS)
    return &p;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return &p;
  uint64_t ws = MAX_WS;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws,
                                        sizeof(ws));
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(handle, p.desc, p.la, p.lb, p.ld,
                                                             p.ld, pref, MAX_ALGOS, p.cand, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n < 1) return &p;
  p.n_cand = n;
  p.ok = true;
  return &p;
}

void* workspace(hipStream_t s, size_t bytes) {
  auto& w = workspaces[s];
  if (w.second < bytes) {
    if (w.first && hipFree(w.first) != hipSuccess) return nullptr;
    w = {nullptr, 0};
    if (hipMalloc(&w.first, bytes) != hipSuccess) return nullptr;
    w.second = bytes;
  }
  return w.first;
}

}  // namespace

int blas_gemm(const BlasGemm& g, hipStream_t stream) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0 || !g.A || !g.B || !g.D) return -1;
  if (g.accumulate && !g.d_f32) return -1;
  std::lock_guard<std::mutex> lock(mu);
  if (!init()) return -2;
  Plan* p = plan_for(g);
  if (!p->ok) return -3;
  if (g.bias) {
    const void* bp = g.bias;
    if (hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp,
                                        sizeof(bp)) != HIPBLAS_STATUS_SUCCESS)
      return -2;
  }
  // candidate g.algo when the heuristic offers it (a table from another library version may
  // name one it no longer lists: then its first choice)
  const int k = g.algo > 0 && g.algo < p->n_cand ? g.algo : 0;
  const size_t wsz = p->cand[k].workspaceSize;
  void* ws = wsz ? workspace(stream, wsz) : nullptr;
  if (wsz && !ws) return -2;
  const float alpha = 1.f, beta = g.accumulate ? 1.f : 0.f;
  const hipblasStatus_t st =
      hipblasLtMatmul(handle, p->desc, &alpha, g.B, p->la, g.A, p->lb, &beta, g.D, p->ld, g.D,
                      p->ld, &p->cand[k].algo, ws, wsz, stream);
  return st == HIPBLAS_STATUS_SUCCESS ? 0 : -2;
}

const char* blas_error(int code) {
  switch (code) {
    case -1: return "blas_gemm: bad arguments (accumulate needs an fp32 output)";
    case -2: return "blas_gemm: hipBLASLt call failed";
    case -3: return "blas_gemm: hipBLASLt has no algorithm for this problem";
    default: return "blas_gemm: unknown error";
  }
}

int blas_supported(const BlasGemm& g) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0 || (g.accumulate && !g.d_f32)) return 0;
  std::lock_guard<std::mutex> lock(mu);
  if (!init()) return 0;
  return plan_for(g)->ok ? 1 : 0;
}

int blas_available() {
  std::lock_guard<std::mutex> lock(mu);
  return init() ? 1 : 0;
}

}  // namespace dnn
