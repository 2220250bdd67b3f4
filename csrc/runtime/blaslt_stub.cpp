// Product build of the library-GEMM entry points: hipBLASLt is NOT linked. The engine runs its
// own gfx950 kernels only; the library path exists for A/B comparisons in a separate build
// (python -m docker_dist_nn_amd._build --blas compiles csrc/compare/blaslt.cpp instead of this
// file and links -lhipblaslt; bench/gemm_vs_blas.py).
#include "runtime/blaslt.hpp"

namespace dnn {

int blas_gemm(const BlasGemm&, hipStream_t) { return -4; }

const char* blas_error(int code) {
  return code == -4 ? "hipBLASLt is not in this build (comparison build: _build --blas)"
                    : "hipBLASLt error";
}

int blas_supported(const BlasGemm&) { return 0; }

int blas_available() { return 0; }

}  // namespace dnn
