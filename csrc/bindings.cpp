// pybind11 module `docker_dist_nn_amd._native`: the host entry points of the gfx950 kernels and
// the native runtime pieces (schedule generator/simulator, neuron-JSON weight IO, HIP graph
// executor). Device pointers and HIP streams cross the boundary as integers
// (torch.Tensor.data_ptr(), torch.cuda.Stream.cuda_stream); shapes are validated on the host
// before any launch and a failed check raises instead of launching.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "kernels/chain.hpp"
#include "kernels/elementwise.hpp"
#include "kernels/gemm.hpp"
#include "kernels/gemv.hpp"
#include "kernels/mlp_tail.hpp"
#include "runtime/blaslt.hpp"
#include "runtime/chain_host.hpp"
#include "runtime/graph.hpp"
#include "runtime/json_weights.hpp"
#include "runtime/matrix_codec.hpp"
#include "runtime/p2p.hpp"
#include "runtime/program.hpp"
#include "runtime/schedule.hpp"
#include "runtime/step_plan.hpp"

namespace py = pybind11;
using dnn::GemmParams;

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
template <class T>
static T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}

static void check(int rc, const char* what);

// Launch now, or append to the Program recording on this thread (see runtime/program.hpp).
template <class F>
static void launch(const char* what, F f, uintptr_t stream) {
  if (dnn::Program* pr = dnn::recording_program()) {
    pr->add(what, dnn::Program::Launch(std::move(f)));
    return;
  }
  static const dnn::Program identity;  // no regions: fix() is the identity
  check(f(S(stream), identity), what);
}

static void check(int rc, const char* what) {
  if (rc != 0) {
    std::string msg = std::string(what) + " failed: ";
    if (std::string(what).rfind("gemm_bf16", 0) == 0) msg += dnn::gemm_error_string(rc);
    else if (std::string(what) == "mlp_tail")
      msg += dnn::mlp_tail_error(rc);
    else if (std::string(what) == "blas_gemm") msg += dnn::blas_error(rc);
    else msg += "precondition/launch error code " + std::to_string(rc);
    if (rc == -9) msg += std::string(" (") + hipGetErrorString(hipGetLastError()) + ")";
    throw std::invalid_argument(msg);
  }
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "docker_dist_nn_amd native runtime + gfx950 HIP kernels";

  // Every kernel binding goes through launch(): it launches now, or -- while a Program is
  // recording on this thread -- appends the launch (pointers routed through Program::fix so
  // they can be relocated at replay; stream chosen at replay).
  m.def(
      "gemm_bf16",
      [](uintptr_t a, long lda, uintptr_t b, long ldb, uintptr_t c, long ldc, long c_split_stride,
         uintptr_t bias, uintptr_t aux, long ld_aux, int M, int N, int K, int act, int accumulate,
         int layout_a, int layout_b, int out_f32, int bm, int bn, int splits, uintptr_t stream,
         uintptr_t colsum, long ld_colsum, uintptr_t xent_labels, int n_cls, float xent_scale,
         uintptr_t loss_part, uintptr_t correct, int k_total, int stages, int group_m,
         int persist, uintptr_t mask_out, uintptr_t mask_in, long ld_mask, uintptr_t ct,
         long ld_ct, uintptr_t upd_master, uintptr_t upd_mom, uintptr_t upd_shadow,
         uintptr_t upd_lr, float upd_mu, float upd_wd, uintptr_t timeline, int epi_probe) {
        GemmParams p{};
        p.timeline = P<unsigned long long>(timeline);
        p.epi_probe = epi_probe;
        p.upd_master = P<float>(upd_master);
        p.upd_mom = P<float>(upd_mom);
        p.upd_shadow = P<uint16_t>(upd_shadow);
        p.upd_lr = P<const float>(upd_lr);
        p.upd_mu = upd_mu;
        p.upd_wd = upd_wd;
        p.ct = P<uint16_t>(ct);
        p.ld_ct = ld_ct;
        p.group_m = group_m;
        p.mask_out = P<unsigned char>(mask_out);
        p.mask_in = P<const unsigned char>(mask_in);
        p.ld_mask = ld_mask;
        p.k_total = k_total;
        p.colsum = P<float>(colsum);
        p.ld_colsum = ld_colsum;
        p.xent_labels = P<const int>(xent_labels);
        p.n_cls = n_cls;
        p.xent_scale = xent_scale;
        p.loss_part = P<float>(loss_part);
        p.correct = P<int>(correct);
        p.A = P<const uint16_t>(a);
        p.lda = lda;
        p.B = P<const uint16_t>(b);
        p.ldb = ldb;
        p.C = P<void>(c);
        p.ldc = ldc;
        p.c_split_stride = c_split_stride;
        p.bias = P<const float>(bias);
        p.aux = P<const uint16_t>(aux);
        p.ld_aux = ld_aux;
        p.M = M;
        p.N = N;
        p.K = K;
        p.act = act;
        p.accumulate = accumulate;
        launch(
            "gemm_bf16",
            [=](hipStream_t s, const dnn::Program& R) {
              GemmParams q = p;
              q.A = R.fix(q.A);
              q.B = R.fix(q.B);
              q.C = R.fix(q.C);
              q.bias = R.fix(q.bias);
              q.aux = R.fix(q.aux);
              q.colsum = R.fix(q.colsum);
              q.xent_labels = R.fix(q.xent_labels);
              q.loss_part = R.fix(q.loss_part);
              q.correct = R.fix(q.correct);
              q.mask_out = R.fix(q.mask_out);
              q.mask_in = R.fix(q.mask_in);
              q.ct = R.fix(q.ct);
              q.upd_master = R.fix(q.upd_master);
              q.upd_mom = R.fix(q.upd_mom);
              q.upd_shadow = R.fix(q.upd_shadow);
              q.upd_lr = R.fix(q.upd_lr);
              q.timeline = R.fix(q.timeline);
              return dnn::gemm_bf16(q, layout_a, layout_b, out_f32, bm, bn, splits, s, stages,
                                    persist);
            },
            stream);
      },
      py::arg("a"), py::arg("lda"), py::arg("b"), py::arg("ldb"), py::arg("c"), py::arg("ldc"),
      py::arg("c_split_stride"), py::arg("bias"), py::arg("aux"), py::arg("ld_aux"), py::arg("M"),
      py::arg("N"), py::arg("K"), py::arg("act"), py::arg("accumulate"), py::arg("layout_a"),
      py::arg("layout_b"), py::arg("out_f32"), py::arg("bm"), py::arg("bn"), py::arg("splits"),
      py::arg("stream"), py::arg("colsum") = 0, py::arg("ld_colsum") = 0,
      py::arg("xent_labels") = 0, py::arg("n_cls") = 0, py::arg("xent_scale") = 0.f,
      py::arg("loss_part") = 0, py::arg("correct") = 0, py::arg("k_total") = 0,
      py::arg("stages") = 0, py::arg("group_m") = 0, py::arg("persist") = 0,
      py::arg("mask_out") = 0, py::arg("mask_in") = 0, py::arg("ld_mask") = 0,
      py::arg("ct") = 0, py::arg("ld_ct") = 0, py::arg("upd_master") = 0,
      py::arg("upd_mom") = 0, py::arg("upd_shadow") = 0, py::arg("upd_lr") = 0,
      py::arg("upd_mu") = 0.f, py::arg("upd_wd") = 0.f, py::arg("timeline") = 0,
      py::arg("epi_probe") = 0);
  m.def("gemm_default_stages", &dnn::default_stages);

  m.def("gemv_max_rows", []() { return dnn::GEMV_MAX_ROWS; });
  m.def(
      "gemv_bf16",
      [](uintptr_t x, long ldx, uintptr_t w, long ldw, uintptr_t bias, uintptr_t y, long ldy,
         int M, int N, int K, int act, int out_f32, uintptr_t stream) {
        launch(
            "gemv_bf16",
            [=](hipStream_t s, const dnn::Program& R) {
              return dnn::gemv_bf16(R.fix(P<const uint16_t>(x)), ldx,
                                    R.fix(P<const uint16_t>(w)), ldw, R.fix(P<const float>(bias)),
                                    R.fix(P<void>(y)), ldy, M, N, K, act, out_f32, s);
            },
            stream);
      },
      py::arg("x"), py::arg("ldx"), py::arg("w"), py::arg("ldw"), py::arg("bias"), py::arg("y"),
      py::arg("ldy"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("act"),
      py::arg("out_f32"), py::arg("stream"));
  m.def(
      "gemm_bf16_streamk",
      [](uintptr_t a, long lda, uintptr_t b, long ldb, uintptr_t c, long ldc, int M, int N, int K,
         int accumulate, int layout_a, int layout_b, int bm, int bn, int nwg, uintptr_t part,
         uintptr_t stream) {
        GemmParams p{};
        p.A = P<const uint16_t>(a);
        p.lda = lda;
        p.B = P<const uint16_t>(b);
        p.ldb = ldb;
        p.C = P<void>(c);
        p.ldc = ldc;
        p.M = M;
        p.N = N;
        p.K = K;
        p.accumulate = accumulate;
        launch(
            "gemm_bf16_streamk",
            [=](hipStream_t s, const dnn::Program& R) {
              GemmParams q = p;
              q.A = R.fix(q.A);
              q.B = R.fix(q.B);
              q.C = R.fix(q.C);
              return dnn::gemm_bf16_streamk(q, layout_a, layout_b, bm, bn, nwg,
                                            R.fix(P<float>(part)), s);
            },
            stream);
      },
      py::arg("a"), py::arg("lda"), py::arg("b"), py::arg("ldb"), py::arg("c"), py::arg("ldc"),
      py::arg("M"), py::arg("N"), py::arg("K"), py::arg("accumulate"), py::arg("layout_a"),
      py::arg("layout_b"), py::arg("bm"), py::arg("bn"), py::arg("nwg"), py::arg("part"),
      py::arg("stream"));
  m.def("softmax_xent",
        [](uintptr_t logits, long ld_logits, uintptr_t labels, uintptr_t dz, long ld_dz, int rows,
           int n_cls, int width, float scale, uintptr_t loss_part, uintptr_t correct,
           uintptr_t stream, uintptr_t colsum, long ld_colsum) {
          launch(
              "softmax_xent",
              [=](hipStream_t s, const dnn::Program& R) {
                return dnn::softmax_xent(R.fix(P<const float>(logits)), ld_logits,
                                         R.fix(P<const int>(labels)), R.fix(P<uint16_t>(dz)),
                                         ld_dz, rows, n_cls, width, scale,
                                         R.fix(P<float>(loss_part)), R.fix(P<int>(correct)),
                                         R.fix(P<float>(colsum)), ld_colsum, s);
              },
              stream);
        },
        py::arg("logits"), py::arg("ld_logits"), py::arg("labels"), py::arg("dz"),
        py::arg("ld_dz"), py::arg("rows"), py::arg("n_cls"), py::arg("width"), py::arg("scale"),
        py::arg("loss_part"), py::arg("correct"), py::arg("stream"), py::arg("colsum") = 0,
        py::arg("ld_colsum") = 0);
  m.def("softmax_xent_blocks", &dnn::softmax_xent_blocks);
  m.def(
      "mlp_tail",
      [](uintptr_t x, long ldx, uintptr_t w3, long ldw3, uintptr_t b3, uintptr_t w4, long ldw4,
         uintptr_t b4, uintptr_t labels, uintptr_t h3, long ldh3, uintptr_t dz4, long lddz4,
         uintptr_t dz3, long lddz3, uintptr_t dz2, long lddz2, uintptr_t loss_part,
         uintptr_t correct, uintptr_t cs4, long ld_cs4, uintptr_t cs3, long ld_cs3, uintptr_t cs2,
         long ld_cs2, int M, int K3, int N3, int N4, int n_cls, float scale, int act3, int act2,
         uintptr_t stream) {
        launch(
            "mlp_tail",
            [=](hipStream_t s, const dnn::Program& R) {
              dnn::TailParams p{};
              p.X = R.fix(P<const uint16_t>(x));
              p.ldx = ldx;
              p.W3 = R.fix(P<const uint16_t>(w3));
              p.ldw3 = ldw3;
              p.b3 = R.fix(P<const float>(b3));
              p.W4 = R.fix(P<const uint16_t>(w4));
              p.ldw4 = ldw4;
              p.b4 = R.fix(P<const float>(b4));
              p.labels = R.fix(P<const int>(labels));
              p.H3 = R.fix(P<uint16_t>(h3));
              p.ldh3 = ldh3;
              p.DZ4 = R.fix(P<uint16_t>(dz4));
              p.lddz4 = lddz4;
              p.DZ3 = R.fix(P<uint16_t>(dz3));
              p.lddz3 = lddz3;
              p.DZ2 = R.fix(P<uint16_t>(dz2));
              p.lddz2 = lddz2;
              p.loss_part = R.fix(P<float>(loss_part));
              p.correct = R.fix(P<int>(correct));
              p.cs4 = R.fix(P<float>(cs4));
              p.ld_cs4 = ld_cs4;
              p.cs3 = R.fix(P<float>(cs3));
              p.ld_cs3 = ld_cs3;
              p.cs2 = R.fix(P<float>(cs2));
              p.ld_cs2 = ld_cs2;
              p.M = M;
              p.K3 = K3;
              p.N3 = N3;
              p.N4 = N4;
              p.n_cls = n_cls;
              p.scale = scale;
              p.act3 = act3;
              p.act2 = act2;
              return dnn::mlp_tail(p, s);
            },
            stream);
      },
      py::arg("x"), py::arg("ldx"), py::arg("w3"), py::arg("ldw3"), py::arg("b3"), py::arg("w4"),
      py::arg("ldw4"), py::arg("b4"), py::arg("labels"), py::arg("h3"), py::arg("ldh3"),
      py::arg("dz4"), py::arg("lddz4"), py::arg("dz3"), py::arg("lddz3"), py::arg("dz2"),
      py::arg("lddz2"), py::arg("loss_part"), py::arg("correct"), py::arg("cs4"),
      py::arg("ld_cs4"), py::arg("cs3"), py::arg("ld_cs3"), py::arg("cs2"), py::arg("ld_cs2"),
      py::arg("M"), py::arg("K3"), py::arg("N3"), py::arg("N4"), py::arg("n_cls"),
      py::arg("scale"), py::arg("act3"), py::arg("act2"), py::arg("stream"));
  m.def("mlp_tail_blocks", &dnn::mlp_tail_blocks);
  // Grouped GEMM launch (no epilogue extras: the split-K weight gradients of a step). problems:
  // (a, lda, b, ldb, c, ldc, c_split_stride, M, N, K, k_total, accumulate, splits)
  m.def(
      "gemm_bf16_group",
      [](const std::vector<std::tuple<uintptr_t, long, uintptr_t, long, uintptr_t, long, long,
                                      int, int, int, int, int, int>>& probs,
         int layout_a, int layout_b, int out_f32, int bm, int bn, int stages, uintptr_t stream) {
        if (probs.empty() || probs.size() > (size_t)dnn::GEMM_GROUP_MAX)
          throw std::invalid_argument("gemm_bf16_group: 1..8 problems");
        std::vector<GemmParams> ps;
        std::vector<int> splits;
        for (const auto& t : probs) {
          GemmParams p{};
          p.A = P<const uint16_t>(std::get<0>(t));
          p.lda = std::get<1>(t);
          p.B = P<const uint16_t>(std::get<2>(t));
          p.ldb = std::get<3>(t);
          p.C = P<void>(std::get<4>(t));
          p.ldc = std::get<5>(t);
          p.c_split_stride = std::get<6>(t);
          p.M = std::get<7>(t);
          p.N = std::get<8>(t);
          p.K = std::get<9>(t);
          p.k_total = std::get<10>(t);
          p.accumulate = std::get<11>(t);
          ps.push_back(p);
          splits.push_back(std::get<12>(t));
        }
        launch(
            "gemm_bf16_group",
            [=](hipStream_t s, const dnn::Program& R) {
              std::vector<GemmParams> q = ps;
              for (auto& p : q) {
                p.A = R.fix(p.A);
                p.B = R.fix(p.B);
                p.C = R.fix(p.C);
              }
              return dnn::gemm_bf16_group(q.data(), splits.data(), (int)q.size(), layout_a,
                                          layout_b, out_f32, bm, bn, stages, s);
            },
            stream);
      },
      py::arg("problems"), py::arg("layout_a"), py::arg("layout_b"), py::arg("out_f32"),
      py::arg("bm"), py::arg("bn"), py::arg("stages"), py::arg("stream"));
  m.def(
      "blas_gemm",
      [](int trans_a, int trans_b, int M, int N, int K, uintptr_t a, long lda, uintptr_t b,
         long ldb, uintptr_t d, long ldd, int d_f32, uintptr_t bias, int relu, int accumulate,
         uintptr_t stream, int algo) {
        launch(
            "blas_gemm",
            [=](hipStream_t s, const dnn::Program& R) {
              dnn::BlasGemm g{};
              g.trans_a = trans_a;
              g.trans_b = trans_b;
              g.M = M;
              g.N = N;
              g.K = K;
              g.A = R.fix(P<const uint16_t>(a));
              g.lda = lda;
              g.B = R.fix(P<const uint16_t>(b));
              g.ldb = ldb;
              g.D = R.fix(P<void>(d));
              g.ldd = ldd;
              g.d_f32 = d_f32;
              g.bias = R.fix(P<const float>(bias));
              g.relu = relu;
              g.accumulate = accumulate;
              g.algo = algo;
              return dnn::blas_gemm(g, s);
            },
            stream);
      },
      py::arg("trans_a"), py::arg("trans_b"), py::arg("M"), py::arg("N"), py::arg("K"),
      py::arg("a"), py::arg("lda"), py::arg("b"), py::arg("ldb"), py::arg("d"), py::arg("ldd"),
      py::arg("d_f32"), py::arg("bias"), py::arg("relu"), py::arg("accumulate"),
      py::arg("stream"), py::arg("algo") = 0);
  m.def("blas_available", &dnn::blas_available);
  m.def("blas_supported", [](int trans_a, int trans_b, int M, int N, int K, long lda, long ldb,
                             long ldd, int d_f32, int has_bias, int relu, int accumulate) {
    dnn::BlasGemm g{};
    g.trans_a = trans_a;
    g.trans_b = trans_b;
    g.M = M;
    g.N = N;
    g.K = K;
    g.lda = lda;
    g.ldb = ldb;
    g.ldd = ldd;
    g.d_f32 = d_f32;
    static const float one = 0.f;
    g.bias = has_bias ? &one : nullptr;  // only its presence selects the epilogue
    g.relu = relu;
    g.accumulate = accumulate;
    return dnn::blas_supported(g);
  });
  m.def("dact_colsum", [](uintptr_t x, long ld, uintptr_t aux, long ld_aux, int act, int rows,
                          int cols, int n_part, uintptr_t part, uintptr_t stream) {
    launch(
        "dact_colsum",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::dact_colsum(R.fix(P<uint16_t>(x)), ld, R.fix(P<const uint16_t>(aux)),
                                  ld_aux, act, rows, cols, n_part, R.fix(P<float>(part)), s);
        },
        stream);
  });
  m.def("softmax_rows", [](uintptr_t logits, long ld_in, uintptr_t out, long ld_out, int rows,
                           int n_cls, uintptr_t labels, uintptr_t pred, uintptr_t correct,
                           uintptr_t stream) {
    launch(
        "softmax_rows",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::softmax_rows(R.fix(P<const float>(logits)), ld_in, R.fix(P<float>(out)),
                                   ld_out, rows, n_cls, R.fix(P<const int>(labels)),
                                   R.fix(P<int>(pred)), R.fix(P<int>(correct)), s);
        },
        stream);
  });
  m.def("colsum_partial", [](uintptr_t x, long ld, int rows, int cols, int n_part, uintptr_t part,
                             uintptr_t stream) {
    launch(
        "colsum_partial",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::colsum_partial(R.fix(P<const uint16_t>(x)), ld, rows, cols, n_part,
                                     R.fix(P<float>(part)), s);
        },
        stream);
  });
  m.def("reduce_slabs", [](uintptr_t src, long stride, int n_src, long n, float scale,
                           uintptr_t out, int accumulate, uintptr_t stream) {
    launch(
        "reduce_slabs",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::reduce_slabs(R.fix(P<const float>(src)), stride, n_src, n, scale,
                                   R.fix(P<float>(out)), accumulate, s);
        },
        stream);
  });
  // jobs: sequence of (src, stride, n_src, n, out, scale, accumulate); > 16 jobs -> several
  // launches
  m.def("reduce_multi", [](const std::vector<std::tuple<uintptr_t, long, int, long, uintptr_t,
                                                        float, int, uintptr_t, int>>& jobs,
                           uintptr_t stream, uintptr_t grad_base, uintptr_t master,
                           uintptr_t mom, uintptr_t shadow, float lr, float mu, float wd,
                           uintptr_t lr_dev, int adam, uintptr_t v, float b1, float b2,
                           float eps, int decoupled, uintptr_t step_dev, double db1, double db2,
                           float bc1, float bc2, int max_blocks) {
    std::vector<dnn::ReduceJob> J;
    J.reserve(jobs.size());
    for (const auto& t : jobs)
      J.push_back({P<const float>(std::get<0>(t)), std::get<1>(t), std::get<3>(t),
                   P<float>(std::get<4>(t)), std::get<2>(t), std::get<5>(t), std::get<6>(t),
                   P<uint16_t>(std::get<7>(t)), std::get<8>(t)});
    const bool fused = master != 0;
    dnn::FusedSgd sg{P<const float>(grad_base), P<float>(master), P<float>(mom),
                     P<uint16_t>(shadow), lr, mu, wd, P<const float>(lr_dev)};
    sg.adam = adam;
    sg.v = P<float>(v);
    sg.b1 = b1;
    sg.b2 = b2;
    sg.eps = eps;
    sg.decoupled = decoupled;
    sg.step_dev = P<const int>(step_dev);
    sg.db1 = db1;
    sg.db2 = db2;
    sg.bc1 = bc1;
    sg.bc2 = bc2;
    if (adam && (!mom || !v)) throw std::invalid_argument("fused Adam needs both moments");
    for (size_t k = 0; k < J.size(); k += dnn::REDUCE_MAX_JOBS) {
      const int n = (int)std::min<size_t>(dnn::REDUCE_MAX_JOBS, J.size() - k);
      std::vector<dnn::ReduceJob> part(J.begin() + k, J.begin() + k + n);
      launch(
          "reduce_multi",
          [part, fused, sg, max_blocks](hipStream_t s, const dnn::Program& R) mutable {
            std::vector<dnn::ReduceJob> q = part;
            for (auto& j : q) {
              j.src = R.fix(j.src);
              j.out = R.fix(j.out);
              j.wt = R.fix(j.wt);
            }
            dnn::FusedSgd f = sg;
            f.grad_base = R.fix(f.grad_base);
            f.master = R.fix(f.master);
            f.mom = R.fix(f.mom);
            f.shadow = R.fix(f.shadow);
            f.v = R.fix(f.v);
            return dnn::reduce_multi(q.data(), (int)q.size(), s, fused ? &f : nullptr,
                                     max_blocks);
          },
          stream);
    }
  }, py::arg("jobs"), py::arg("stream"), py::arg("grad_base") = 0, py::arg("master") = 0,
     py::arg("mom") = 0, py::arg("shadow") = 0, py::arg("lr") = 0.f, py::arg("mu") = 0.f,
     py::arg("wd") = 0.f, py::arg("lr_dev") = 0, py::arg("adam") = 0, py::arg("v") = 0,
     py::arg("b1") = 0.f, py::arg("b2") = 0.f, py::arg("eps") = 0.f, py::arg("decoupled") = 0,
     py::arg("step_dev") = 0, py::arg("db1") = 0.0, py::arg("db2") = 0.0, py::arg("bc1") = 1.f,
     py::arg("bc2") = 1.f, py::arg("max_blocks") = 0);
  m.def(
      "sgd_update",
      [](uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t shadow, long n, float lr, float mu,
         float wd, uintptr_t stream, uintptr_t lr_dev) {
        launch(
            "sgd_update",
            [=](hipStream_t s, const dnn::Program& R) {
              return dnn::sgd_update(R.fix(P<float>(p)), R.fix(P<const float>(g)),
                                     R.fix(P<float>(mom)), R.fix(P<uint16_t>(shadow)), n, lr, mu,
                                     wd, s, P<const float>(lr_dev));
            },
            stream);
      },
      py::arg("p"), py::arg("g"), py::arg("mom"), py::arg("shadow"), py::arg("n"), py::arg("lr"),
      py::arg("mu"), py::arg("wd"), py::arg("stream"), py::arg("lr_dev") = 0);
  m.def(
      "adam_update",
      [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t vv, uintptr_t shadow, long n, float lr,
         float b1, float b2, float eps, float wd, int decoupled, float bc1, float bc2,
         uintptr_t stream, uintptr_t lr_dev, uintptr_t step_dev, double db1, double db2) {
        launch(
            "adam_update",
            [=](hipStream_t s, const dnn::Program& R) {
              return dnn::adam_update(R.fix(P<float>(p)), R.fix(P<const float>(g)),
                                      R.fix(P<float>(mm)), R.fix(P<float>(vv)),
                                      R.fix(P<uint16_t>(shadow)), n, lr, b1, b2, eps, wd,
                                      decoupled, bc1, bc2, s, P<const float>(lr_dev),
                                      P<const int>(step_dev), db1, db2);
            },
            stream);
      },
      py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("shadow"), py::arg("n"),
      py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"),
      py::arg("decoupled"), py::arg("bc1"), py::arg("bc2"), py::arg("stream"),
      py::arg("lr_dev") = 0, py::arg("step_dev") = 0, py::arg("db1") = 0.9,
      py::arg("db2") = 0.999);
  m.def("step_advance", [](uintptr_t step, uintptr_t stream) {
    launch(
        "step_advance",
        [=](hipStream_t s, const dnn::Program&) { return dnn::step_advance(P<int>(step), s); },
        stream);
  });
  m.def("pack_bf16", [](uintptr_t in, long ld_in, int rows, int cols, uintptr_t out, long ld_out,
                        int rows_p, int cols_p, uintptr_t stream) {
    launch(
        "pack_bf16",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::pack_bf16(R.fix(P<const float>(in)), ld_in, rows, cols,
                                R.fix(P<uint16_t>(out)), ld_out, rows_p, cols_p, s);
        },
        stream);
  });
  m.def("transpose_bf16", [](uintptr_t src, long ld_src, int rows, int cols, uintptr_t dst,
                             long ld_dst, uintptr_t stream) {
    launch(
        "transpose_bf16",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::transpose_bf16(R.fix(P<const uint16_t>(src)), ld_src, rows, cols,
                                     R.fix(P<uint16_t>(dst)), ld_dst, s);
        },
        stream);
  });
  m.def("transpose_multi",
        [](const std::vector<std::tuple<uintptr_t, long, int, int, uintptr_t, long>>& jobs,
           uintptr_t stream) {
          if (jobs.empty() || jobs.size() > (size_t)dnn::TRANSPOSE_MAX_JOBS)
            throw std::invalid_argument("transpose_multi: 1..16 jobs");
          for (const auto& [src, lds, rows, cols, dst, ldd] : jobs)
            if (rows <= 0 || cols <= 0 || rows % 64 || cols % 64 || lds < cols || ldd < rows ||
                lds % 8 || ldd % 8 || ((src | dst) & 15))
              throw std::invalid_argument("transpose_multi: bad job shape / alignment");
          launch(
              "transpose_multi",
              [=](hipStream_t s, const dnn::Program& R) {
                dnn::TransposeJobs J{};
                J.n = (int)jobs.size();
                int t = 0;
                for (int k = 0; k < J.n; ++k) {
                  const auto& [src, lds, rows, cols, dst, ldd] = jobs[k];
                  J.src[k] = R.fix(P<const uint16_t>(src));
                  J.dst[k] = R.fix(P<uint16_t>(dst));
                  J.ld_src[k] = lds;
                  J.ld_dst[k] = ldd;
                  J.tiles_c[k] = cols / 64;
                  J.start[k] = t;
                  t += (rows / 64) * (cols / 64);
                }
                J.start[J.n] = t;
                return dnn::transpose_multi(J, s);
              },
              stream);
        });
  m.def("quant_rows_fp8", [](uintptr_t x, long ldx, int rows, int cols, uintptr_t q, long ldq,
                             uintptr_t scale, uintptr_t stream) {
    launch(
        "quant_rows_fp8",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::quant_rows_fp8(R.fix(P<const uint16_t>(x)), ldx, rows, cols,
                                     R.fix(P<unsigned char>(q)), ldq, R.fix(P<float>(scale)), s);
        },
        stream);
  });
  m.def("dequant_rows_fp8", [](uintptr_t q, long ldq, uintptr_t scale, int rows, int cols,
                               uintptr_t x, long ldx, uintptr_t stream) {
    launch(
        "dequant_rows_fp8",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::dequant_rows_fp8(R.fix(P<const unsigned char>(q)), ldq,
                                       R.fix(P<const float>(scale)), rows, cols,
                                       R.fix(P<uint16_t>(x)), ldx, s);
        },
        stream);
  });
  m.def("unpack_bf16", [](uintptr_t in, long ld_in, int rows, int cols, uintptr_t out,
                          long ld_out, uintptr_t stream) {
    launch(
        "unpack_bf16",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::unpack_bf16(R.fix(P<const uint16_t>(in)), ld_in, rows, cols,
                                  R.fix(P<float>(out)), ld_out, s);
        },
        stream);
  });

  m.def("bias_act_cast", [](uintptr_t in, long ld_in, uintptr_t bias, int act, uintptr_t out,
                            long ld_out, int rows, int cols, uintptr_t stream) {
    launch(
        "bias_act_cast",
        [=](hipStream_t s, const dnn::Program& R) {
          return dnn::bias_act_cast(R.fix(P<const float>(in)), ld_in,
                                    R.fix(P<const float>(bias)), act, R.fix(P<uint16_t>(out)),
                                    ld_out, rows, cols, s);
        },
        stream);
  });

  // ---- runtime: native step executor (recorded launch programs) ---------------------------
  py::class_<dnn::Program>(m, "Program",
                           "Recorded kernel launches in named segments, replayed from C++.")
      .def(py::init<>())
      .def("mark", &dnn::Program::mark, py::arg("name"))
      .def("close", &dnn::Program::close)
      .def("region", &dnn::Program::region, py::arg("base"), py::arg("size"))
      .def("rebase", &dnn::Program::rebase, py::arg("id"), py::arg("new_base"))
      .def(
          "run",
          [](const dnn::Program& pr, const std::vector<std::string>& names, uintptr_t stream) {
            py::gil_scoped_release nogil;
            pr.run(names, S(stream));
          },
          py::arg("names"), py::arg("stream"))
      .def(
          "run_all",
          [](const dnn::Program& pr, uintptr_t stream) {
            py::gil_scoped_release nogil;
            pr.run_all(S(stream));
          },
          py::arg("stream"))
      .def_property_readonly("size", &dnn::Program::size)
      .def("segments", &dnn::Program::segments)
      .def("segment_size", &dnn::Program::segment_size)
      .def("clear", &dnn::Program::clear);
  // A whole step of a single-process (loopback) pipeline: (program, segment) pairs in
  // schedule order, one call, GIL released.
  // A whole step of a single-process (loopback) pipeline: (program, segment, stream) triples
  // in schedule order, one call, GIL released. stream 0 = `stream`, 1 = `side`; the pseudo
  // segments "@fork" (side waits for main) and "@join" (main waits for side) order the two.
  m.def(
      "run_plan",
      [](const std::vector<std::tuple<const dnn::Program*, std::string, int>>& plan,
         uintptr_t stream, uintptr_t side, bool device_fence, uint64_t xkey) {
        py::gil_scoped_release nogil;
        // fork / join events: both streams are on this device, so the ordering needs no
        // system-scope fence (cache write-back / invalidate at every record: the ~6 us
        // "event packets" of profiles/r2_sched). device_fence = hipEventDisableSystemFence.
        static thread_local hipEvent_t evs[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
        hipEvent_t& ev_fork = evs[device_fence][0];
        hipEvent_t& ev_join = evs[device_fence][1];
        if (!ev_fork) {
          const unsigned fl =
              hipEventDisableTiming | (device_fence ? hipEventDisableSystemFence : 0u);
          if (hipEventCreateWithFlags(&ev_fork, fl) != hipSuccess ||
              hipEventCreateWithFlags(&ev_join, fl) != hipSuccess)
            throw std::runtime_error("run_plan: hipEventCreate failed");
        }
        // cross-step events ("@xmark:<k>" records on the side stream, "@xwait:<k>" makes the
        // main stream wait on the LAST such record -- possibly made by the previous step's
        // call: a step's first kernels overlap the previous step's side-stream tail). They
        // belong to one executor (`xkey`, its id): two executors stepping in turn on one
        // thread must each wait on their OWN side stream's marks. Process-wide,
        // under a mutex, so a step issued from another thread finds the same events.
        static std::mutex xmu;
        static std::map<std::tuple<uint64_t, bool, std::string>, hipEvent_t> xev;
        auto xevent = [&](const std::string& k) {
          std::lock_guard<std::mutex> lk(xmu);
          hipEvent_t& e = xev[{xkey, device_fence, k}];
          if (!e) {
            const unsigned fl =
                hipEventDisableTiming | (device_fence ? hipEventDisableSystemFence : 0u);
            if (hipEventCreateWithFlags(&e, fl) != hipSuccess)
              throw std::runtime_error("run_plan: hipEventCreate failed");
          }
          return e;
        };
        std::vector<std::string> one(1);
        for (const auto& [pr, seg, si] : plan) {
          if (seg.rfind("@xmark:", 0) == 0 || seg.rfind("@xwait:", 0) == 0) {
            if (!side) throw std::invalid_argument("run_plan: cross-step event without a side");
            hipEvent_t e = xevent(seg.substr(7));
            const bool mark = seg[2] == 'm';
            if ((mark ? hipEventRecord(e, S(side)) : hipStreamWaitEvent(S(stream), e, 0)) !=
                hipSuccess)
              throw std::runtime_error("run_plan: cross-step event failed");
            continue;
          }
          if (seg == "@fork" || seg == "@join") {
            if (!side) throw std::invalid_argument("run_plan: fork/join without a side stream");
            hipEvent_t ev = seg == "@fork" ? ev_fork : ev_join;
            hipStream_t from = seg == "@fork" ? S(stream) : S(side);
            hipStream_t to = seg == "@fork" ? S(side) : S(stream);
            if (hipEventRecord(ev, from) != hipSuccess || hipStreamWaitEvent(to, ev, 0) != hipSuccess)
              throw std::runtime_error("run_plan: event fork/join failed");
            continue;
          }
          one[0] = seg;
          pr->run(one, si ? S(side) : S(stream));
        }
      },
      py::arg("plan"), py::arg("stream"), py::arg("side") = 0, py::arg("device_fence") = false,
      py::arg("xkey") = 0);
  m.def("record_begin", [](dnn::Program& pr) {
    if (dnn::recording_program()) throw std::runtime_error("already recording a Program");
    dnn::recording_program() = &pr;
  });
  m.def("record_end", []() {
    if (dnn::recording_program()) dnn::recording_program()->close();
    dnn::recording_program() = nullptr;
  });
  m.def("is_recording", []() { return dnn::recording_program() != nullptr; });
  m.def("roctx_push", [](const std::string& n) { dnn::roctx_push(n.c_str()); });
  m.def("roctx_pop", []() { dnn::roctx_pop(); });

  // ---- runtime: pipeline schedules -------------------------------------------------------
  py::enum_<dnn::OpKind>(m, "OpKind")
      .value("FWD", dnn::OpKind::FWD)
      .value("BWD", dnn::OpKind::BWD)
      .value("WGRAD", dnn::OpKind::WGRAD)
      .value("OPT", dnn::OpKind::OPT);
  py::class_<dnn::SchedOp>(m, "SchedOp")
      .def_readonly("kind", &dnn::SchedOp::kind)
      .def_readonly("micro", &dnn::SchedOp::micro)
      .def("__repr__", [](const dnn::SchedOp& o) {
        static const char* n[] = {"F", "B", "W", "O"};
        return std::string(n[(int)o.kind]) + std::to_string(o.micro);
      });
  m.def("make_schedule", &dnn::make_schedule, py::arg("kind"), py::arg("num_stages"),
        py::arg("num_micro"), py::arg("stage"),
        "Ordered compute ops of one pipeline stage for one training step.");
  m.def("simulate_schedule", &dnn::simulate_schedule, py::arg("kind"), py::arg("num_stages"),
        py::arg("num_micro"), py::arg("t_fwd"), py::arg("t_bwd"), py::arg("t_wgrad"),
        py::arg("t_comm"),
        "Event simulation of a step; returns (makespan, per-stage busy time, bubble fraction).");

  // ---- runtime: neuron-JSON weight IO -----------------------------------------------------
  m.def(
      "parse_neuron_json",
      [](const std::string& path) {
        dnn::ParsedModel pm = dnn::parse_neuron_json_file(path);
        py::list layers;
        for (auto& L : pm.layers) {
          py::dict d;
          d["key"] = L.key;
          d["type"] = L.type;
          d["nodes"] = L.nodes;
          d["activation"] = L.activation;
          d["mixed_activation"] = L.mixed_activation;
          d["in_dim"] = L.in_dim;
          const py::ssize_t n_out = (py::ssize_t)L.bias.size();  // neurons actually present
          py::array_t<float> w({n_out, (py::ssize_t)L.in_dim});
          if (!L.weights.empty())
            std::memcpy(w.mutable_data(), L.weights.data(), L.weights.size() * sizeof(float));
          py::array_t<float> b(n_out);
          if (n_out) std::memcpy(b.mutable_data(), L.bias.data(), L.bias.size() * sizeof(float));
          d["weights"] = w;
          d["bias"] = b;
          layers.append(d);
        }
        py::dict out;
        out["layers"] = layers;
        out["layer_distribution"] = pm.layer_distribution;
        out["has_distribution"] = pm.has_distribution;
        out["wrapped"] = pm.wrapped;
        out["stage_file"] = pm.stage_file;
        return out;
      },
      py::arg("path"),
      "Parse a reference model config / stage file into float32 weight matrices.");
  m.def(
      "write_neuron_json",
      [](const std::string& path, const std::vector<py::array_t<float, py::array::c_style>>& ws,
         const std::vector<py::array_t<float, py::array::c_style>>& bs,
         const std::vector<std::string>& acts, const std::vector<std::string>& types,
         const std::vector<int>& distribution, bool stage_file) {
        std::vector<dnn::LayerOut> L(ws.size());
        for (size_t i = 0; i < ws.size(); ++i) {
          if (ws[i].ndim() != 2 || bs[i].ndim() != 1 || bs[i].shape(0) != ws[i].shape(0))
            throw std::invalid_argument("weights must be [out,in] and bias [out]");
          L[i].out = (int)ws[i].shape(0);
          L[i].in = (int)ws[i].shape(1);
          L[i].w = ws[i].data();
          L[i].b = bs[i].data();
          L[i].activation = acts.at(i);
          L[i].type = types.at(i);
        }
        dnn::write_neuron_json_file(path, L, distribution, stage_file);
      },
      py::arg("path"), py::arg("weights"), py::arg("biases"), py::arg("activations"),
      py::arg("types"), py::arg("layer_distribution"), py::arg("stage_file"));

  m.def(
      "parse_examples_json",
      [](const std::string& path) {
        dnn::ParsedExamples E = dnn::parse_examples_json_file(path);
        py::array_t<float> x({(py::ssize_t)E.n, (py::ssize_t)E.dim});
        if (!E.x.empty()) std::memcpy(x.mutable_data(), E.x.data(), E.x.size() * sizeof(float));
        py::array_t<int> y((py::ssize_t)E.n);
        if (!E.labels.empty())
          std::memcpy(y.mutable_data(), E.labels.data(), E.labels.size() * sizeof(int));
        py::dict out;
        out["x"] = x;
        out["labels"] = y;
        out["outer_len"] = E.outer_len;
        out["raw_list"] = E.raw_list;
        return out;
      },
      py::arg("path"), "Parse an inputs JSON ({\"examples\": [...]}) into float32 + int32 arrays.");

  // ---- runtime: protobuf Matrix codec (gRPC compat ingress) -----------------------------
  m.def(
      "decode_matrix",
      [](py::bytes b) {
        char* buf;
        py::ssize_t n;
        PYBIND11_BYTES_AS_STRING_AND_SIZE(b.ptr(), &buf, &n);
        const uint8_t* u = reinterpret_cast<const uint8_t*>(buf);
        long rows = 0, cols = 0;
        {
          py::gil_scoped_release nogil;
          dnn::scan_matrix(u, (size_t)n, &rows, &cols);
        }
        // decode straight into the numpy array: no intermediate vector, one copy of the data
        py::array_t<double> a({(py::ssize_t)rows, (py::ssize_t)cols});
        double* out = a.mutable_data();
        if (rows && cols) {
          py::gil_scoped_release nogil;
          dnn::fill_matrix(u, (size_t)n, out, cols);
        }
        return a;
      },
      py::arg("data"), "Matrix wire bytes -> float64 [rows][cols]");
  m.def(
      "encode_matrix",
      [](py::array_t<double, py::array::c_style | py::array::forcecast> a) {
        if (a.ndim() != 2) throw std::invalid_argument("encode_matrix needs a 2-D array");
        const long rows = (long)a.shape(0), cols = (long)a.shape(1);
        const size_t sz = dnn::encoded_size(rows, cols);
        // the bytes object is the output buffer: the wire bytes are written once
        PyObject* o = PyBytes_FromStringAndSize(nullptr, (py::ssize_t)sz);
        if (!o) throw py::error_already_set();
        char* dst = PyBytes_AS_STRING(o);
        {
          py::gil_scoped_release nogil;
          dnn::encode_matrix_into(a.data(), rows, cols, dst);
        }
        return py::reinterpret_steal<py::bytes>(o);
      },
      py::arg("array"), "float64 [rows][cols] -> Matrix wire bytes");

  // ---- runtime: HIP graph executor ------------------------------------------------------
  // ---- runtime: native multi-rank step (runtime/step_plan.hpp) ----------------------------
  m.def("nccl_load", [](const std::string& path) { return dnn::nccl_load(path).path; },
        py::arg("path"));
  m.def("nccl_comm_info", [](uintptr_t comm) {
    const dnn::NcclApi* a = dnn::nccl_api();
    if (!a) throw std::runtime_error("nccl_load first");
    int n = 0, r = 0;
    if (a->comm_count(reinterpret_cast<void*>(comm), &n) != 0 ||
        a->comm_user_rank(reinterpret_cast<void*>(comm), &r) != 0)
      throw std::runtime_error("ncclCommCount / ncclCommUserRank failed");
    return std::make_pair(n, r);
  });
  py::class_<dnn::StepPlan>(m, "StepPlan")
      .def(py::init<int, int>(), py::arg("n_streams"), py::arg("n_events"))
      .def(
          "add",
          [](dnn::StepPlan& sp, int kind, int stream, const dnn::Program* prog,
             const std::string& seg, uintptr_t comm, uintptr_t a, uintptr_t b, uint64_t count,
             int dtype, int peer, int64_t delta, int event) {
            dnn::StepPlan::Op o;
            o.kind = static_cast<dnn::StepPlan::Kind>(kind);
            o.stream = stream;
            o.prog = prog;
            o.seg = seg;
            o.comm = reinterpret_cast<void*>(comm);
            o.a = a;
            o.b = b;
            o.count = count;
            o.dtype = dtype;
            o.peer = peer;
            o.delta = delta;
            o.event = event;
            sp.add(o);
          },
          py::arg("kind"), py::arg("stream") = 0, py::arg("prog") = nullptr,
          py::arg("seg") = std::string(), py::arg("comm") = 0, py::arg("a") = 0,
          py::arg("b") = 0, py::arg("count") = 0, py::arg("dtype") = 0, py::arg("peer") = 0,
          py::arg("delta") = 0, py::arg("event") = 0, py::keep_alive<1, 4>())
      .def(
          "run",
          [](dnn::StepPlan& sp, uintptr_t stream) {
            py::gil_scoped_release nogil;
            sp.run(S(stream));
          },
          py::arg("stream"))
      .def_property("seq", &dnn::StepPlan::seq, &dnn::StepPlan::set_seq)
      .def_property_readonly("size", &dnn::StepPlan::size)
      .def_property_readonly("n_streams", &dnn::StepPlan::n_streams)
      .def("comm_error", &dnn::StepPlan::comm_error)
      .def("flag_timeouts", &dnn::StepPlan::flag_timeouts)
      .def_property("wait_timeout", &dnn::StepPlan::wait_timeout,
                    &dnn::StepPlan::set_wait_timeout)
      .def("sync_seq", &dnn::StepPlan::sync_seq)
      .def("clear_ops", &dnn::StepPlan::clear_ops);
  py::class_<dnn::GraphExec>(m, "GraphExec")
      .def(py::init<>())
      .def("begin_capture", [](dnn::GraphExec& g, uintptr_t s) { g.begin_capture(S(s)); })
      .def("end_capture", &dnn::GraphExec::end_capture)
      .def("replay", [](dnn::GraphExec& g, uintptr_t s) { g.replay(S(s)); })
      .def_property_readonly("captured", &dnn::GraphExec::captured)
      .def_property_readonly("num_nodes", &dnn::GraphExec::num_nodes)
      .def("reset", &dnn::GraphExec::reset);
  // ---- runtime: xGMI peer-to-peer pipeline transport (csrc/runtime/p2p.hpp) ---------------
  m.def(
      "ipc_export",
      [](uintptr_t ptr) {
        auto r = dnn::ipc_export(reinterpret_cast<void*>(ptr));
        return py::make_tuple(py::bytes(r.first), r.second);
      },
      py::arg("ptr"), "device pointer -> (IPC handle bytes, offset in its allocation)");
  m.def(
      "ipc_import",
      [](py::bytes h, uint64_t off) {
        return reinterpret_cast<uintptr_t>(dnn::ipc_import(std::string(h), off));
      },
      py::arg("handle"), py::arg("offset"));
  m.def("ipc_close_all", &dnn::ipc_close_all);
  m.def(
      "alloc_uncached",
      [](size_t bytes) { return reinterpret_cast<uintptr_t>(dnn::alloc_uncached(bytes)); },
      py::arg("bytes"), "zeroed device memory the L2 does not cache (xGMI receive buffers)");
  m.def(
      "free_device", [](uintptr_t p) { dnn::free_device(reinterpret_cast<void*>(p)); },
      py::arg("ptr"));
  m.def(
      "host_alloc_mapped",
      [](size_t bytes) {
        // pinned, coherent host memory the GPU reads and writes directly (a persistent
        // kernel's stop word and progress counter: no stream operation needed while it runs)
        void* p = nullptr;
        if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
          throw std::runtime_error("hipHostMalloc failed");
        std::memset(p, 0, bytes);
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
          (void)hipHostFree(p);
          throw std::runtime_error("hipHostGetDevicePointer failed");
        }
        return py::make_tuple(reinterpret_cast<uintptr_t>(p), reinterpret_cast<uintptr_t>(d));
      },
      py::arg("bytes"), "(host pointer, device pointer) of zeroed coherent pinned memory");
  m.def(
      "host_free", [](uintptr_t p) { (void)hipHostFree(reinterpret_cast<void*>(p)); },
      py::arg("ptr"));
  m.def(
      "host_register",
      [](uintptr_t p, size_t bytes) {
        // page-locks and maps existing host memory (e.g. a /dev/shm mapping shared by two
        // processes) for the GPU; returns its device pointer
        if (hipHostRegister(reinterpret_cast<void*>(p), bytes, hipHostRegisterMapped) !=
            hipSuccess)
          throw std::runtime_error("hipHostRegister failed");
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(p), 0) != hipSuccess) {
          (void)hipHostUnregister(reinterpret_cast<void*>(p));
          throw std::runtime_error("hipHostGetDevicePointer failed");
        }
        return reinterpret_cast<uintptr_t>(d);
      },
      py::arg("ptr"), py::arg("bytes"));
  m.def(
      "host_unregister",
      [](uintptr_t p) { (void)hipHostUnregister(reinterpret_cast<void*>(p)); }, py::arg("ptr"));
  m.def(
      "stream_create_dedicated",
      []() {
        // a stream on a hardware queue of its own (the runtime gives a CU-masked stream a new
        // queue instead of a slot in the shared pool): a persistent kernel on it cannot stall
        // the work of other streams queued behind it on a shared queue
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
          throw std::runtime_error("stream_create_dedicated: no device");
        std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
        hipStream_t st = nullptr;
        if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess)
          throw std::runtime_error("hipExtStreamCreateWithCUMask failed");
        return reinterpret_cast<uintptr_t>(st);
      },
      "a stream with a hardware queue of its own (all CUs)");
  m.def(
      "stream_destroy",
      [](uintptr_t st) { (void)hipStreamDestroy(reinterpret_cast<hipStream_t>(st)); },
      py::arg("stream"));
  m.def("can_access_peer", &dnn::can_access_peer, py::arg("dev"), py::arg("peer"));
  m.def(
      "copy_async",
      [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t s) {
        dnn::copy_async(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n,
                        S(s));
      },
      py::arg("dst"), py::arg("src"), py::arg("nbytes"), py::arg("stream"));
  m.def(
      "signal_u32",
      [](uintptr_t s, uintptr_t flag, uint32_t v) {
        dnn::signal_u32(S(s), reinterpret_cast<void*>(flag), v);
      },
      py::arg("stream"), py::arg("flag"), py::arg("value"));
  m.def(
      "wait_geq_u32",
      [](uintptr_t s, uintptr_t flag, uint32_t v) {
        dnn::wait_geq_u32(S(s), reinterpret_cast<void*>(flag), v);
      },
      py::arg("stream"), py::arg("flag"), py::arg("value"));
  // ---- device-side serving chain (csrc/kernels/chain.hpp, serve/fastpath.py) ---------------
  auto ptr = [](uintptr_t p) { return reinterpret_cast<void*>(p); };
  auto chk = [](int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + ")");
  };
  m.def(
      "chain_wait",
      [=](uintptr_t s, uintptr_t flag, uint32_t target, uintptr_t err, double timeout_s) {
        chk(dnn::chain_wait(static_cast<const uint32_t*>(ptr(flag)), target,
                            static_cast<uint32_t*>(ptr(err)), timeout_s, S(s)),
            "chain_wait");
      },
      py::arg("stream"), py::arg("flag"), py::arg("target"), py::arg("err"),
      py::arg("timeout_s"));
  m.def(
      "chain_recv",
      [=](uintptr_t s, uintptr_t flag, uintptr_t slot, long slot_ld, uintptr_t slot_hdr,
          uintptr_t dst, long dst_ld, uintptr_t dst_hdr, int rows, int row_bytes, uintptr_t err,
          uint32_t seq, uintptr_t prev_ack, double timeout_s) {
        dnn::ChainRecv p{};
        p.flag = static_cast<const uint32_t*>(ptr(flag));
        p.slot = ptr(slot);
        p.slot_ld = slot_ld;
        p.slot_hdr = static_cast<const uint32_t*>(ptr(slot_hdr));
        p.dst = ptr(dst);
        p.dst_ld = dst_ld;
        p.dst_hdr = static_cast<uint32_t*>(ptr(dst_hdr));
        p.rows = rows;
        p.row_bytes = row_bytes;
        p.err = static_cast<uint32_t*>(ptr(err));
        p.seq = seq;
        p.prev_ack = static_cast<uint32_t*>(ptr(prev_ack));
        p.timeout_ticks = dnn::chain_ticks(timeout_s);
        chk(dnn::chain_recv(p, S(s)), "chain_recv");
      },
      py::arg("stream"), py::arg("flag"), py::arg("slot"), py::arg("slot_ld"),
      py::arg("slot_hdr"), py::arg("dst"), py::arg("dst_ld"), py::arg("dst_hdr"),
      py::arg("rows"), py::arg("row_bytes"), py::arg("err"), py::arg("seq"),
      py::arg("prev_ack"), py::arg("timeout_s"));
  m.def(
      "chain_send",
      [=](uintptr_t s, uintptr_t src, long src_ld, uintptr_t dst, long dst_ld, int rows,
          int row_bytes, uintptr_t dst_hdr, uintptr_t in_hdr, uintptr_t err, int stage,
          uint32_t status, uintptr_t ack, uint32_t ack_target, uintptr_t next_flag, uint32_t seq,
          uintptr_t prev_ack, double timeout_s) {
        dnn::ChainSend p{};
        p.src = ptr(src);
        p.src_ld = src_ld;
        p.dst = ptr(dst);
        p.dst_ld = dst_ld;
        p.rows = rows;
        p.row_bytes = row_bytes;
        p.dst_hdr = static_cast<uint32_t*>(ptr(dst_hdr));
        p.in_hdr = static_cast<const uint32_t*>(ptr(in_hdr));
        p.err = static_cast<uint32_t*>(ptr(err));
        p.stage = stage;
        p.status = status;
        p.ack = static_cast<const uint32_t*>(ptr(ack));
        p.ack_target = ack_target;
        p.next_flag = static_cast<uint32_t*>(ptr(next_flag));
        p.seq = seq;
        p.prev_ack = static_cast<uint32_t*>(ptr(prev_ack));
        p.timeout_ticks = dnn::chain_ticks(timeout_s);
        chk(dnn::chain_send(p, S(s)), "chain_send");
      },
      py::arg("stream"), py::arg("src"), py::arg("src_ld"), py::arg("dst"), py::arg("dst_ld"),
      py::arg("rows"), py::arg("row_bytes"), py::arg("dst_hdr"), py::arg("in_hdr"),
      py::arg("err"), py::arg("stage"), py::arg("status"), py::arg("ack"),
      py::arg("ack_target"), py::arg("next_flag"), py::arg("seq"), py::arg("prev_ack"),
      py::arg("timeout_s"));
  m.def(
      "chain_gemv_send",
      [=](uintptr_t s, uintptr_t x, long ldx, uintptr_t w, long ldw, uintptr_t bias, int act,
          int rows, int N, int K, int out_f32, uintptr_t dst, long dst_ld, uintptr_t dst_hdr,
          uintptr_t in_hdr, uintptr_t err, int stage, uint32_t status, uintptr_t ack,
          uint32_t ack_target, uintptr_t next_flag, uint32_t seq, uintptr_t prev_ack,
          uintptr_t counter, double timeout_s, uintptr_t in_flag) {
        dnn::ChainGemvSend p{};
        p.in_flag = static_cast<const uint32_t*>(ptr(in_flag));
        p.x = static_cast<const uint16_t*>(ptr(x));
        p.ldx = ldx;
        p.w = static_cast<const uint16_t*>(ptr(w));
        p.ldw = ldw;
        p.bias = static_cast<const float*>(ptr(bias));
        p.act = act;
        p.rows = rows;
        p.N = N;
        p.K = K;
        p.out_f32 = out_f32;
        p.dst = ptr(dst);
        p.dst_ld = dst_ld;
        p.dst_hdr = static_cast<uint32_t*>(ptr(dst_hdr));
        p.in_hdr = static_cast<const uint32_t*>(ptr(in_hdr));
        p.err = static_cast<uint32_t*>(ptr(err));
        p.stage = stage;
        p.status = status;
        p.ack = static_cast<const uint32_t*>(ptr(ack));
        p.ack_target = ack_target;
        p.next_flag = static_cast<uint32_t*>(ptr(next_flag));
        p.seq = seq;
        p.prev_ack = static_cast<uint32_t*>(ptr(prev_ack));
        p.counter = static_cast<uint32_t*>(ptr(counter));
        p.timeout_ticks = dnn::chain_ticks(timeout_s);
        chk(dnn::chain_gemv_send(p, S(s)), "chain_gemv_send");
      },
      py::arg("stream"), py::arg("x"), py::arg("ldx"), py::arg("w"), py::arg("ldw"),
      py::arg("bias"), py::arg("act"), py::arg("rows"), py::arg("N"), py::arg("K"),
      py::arg("out_f32"), py::arg("dst"), py::arg("dst_ld"), py::arg("dst_hdr"),
      py::arg("in_hdr"), py::arg("err"), py::arg("stage"), py::arg("status"), py::arg("ack"),
      py::arg("ack_target"), py::arg("next_flag"), py::arg("seq"), py::arg("prev_ack"),
      py::arg("counter"), py::arg("timeout_s"), py::arg("in_flag") = 0);
  py::class_<dnn::ChainHost>(m, "ChainHost",
                             "rank 0's native request path of the device-side chain "
                             "(runtime/chain_host.hpp)")
      .def(py::init<int>(), py::arg("slots"))
      .def(
          "request",
          [=](dnn::ChainHost& h, int slot, uintptr_t stream, uintptr_t res_stream,
              uintptr_t x_dev, uintptr_t x_host, size_t x_bytes, uintptr_t w, long ldw,
              uintptr_t bias, int act, int rows, int N, int K, uintptr_t dst, long dst_ld,
              uintptr_t dst_hdr, uintptr_t err, uintptr_t ack, uint32_t ack_target,
              uintptr_t next_flag, uint32_t seq, uintptr_t counter, double hop_timeout_s,
              uintptr_t res_flag, uintptr_t res_err, uintptr_t res_dev, uintptr_t res_host,
              size_t res_bytes, uintptr_t last_ack, double wait_timeout_s) {
            dnn::ChainRequest r{};
            r.stream = S(stream);
            r.res_stream = S(res_stream);
            r.x_dev = ptr(x_dev);
            r.x_host = ptr(x_host);
            r.x_bytes = x_bytes;
            dnn::ChainGemvSend& p = r.send;
            p.x = static_cast<const uint16_t*>(ptr(x_dev));
            p.ldx = K;
            p.w = static_cast<const uint16_t*>(ptr(w));
            p.ldw = ldw;
            p.bias = static_cast<const float*>(ptr(bias));
            p.act = act;
            p.rows = rows;
            p.N = N;
            p.K = K;
            p.dst = ptr(dst);
            p.dst_ld = dst_ld;
            p.dst_hdr = static_cast<uint32_t*>(ptr(dst_hdr));
            p.err = static_cast<uint32_t*>(ptr(err));
            p.ack = static_cast<const uint32_t*>(ptr(ack));
            p.ack_target = ack_target;
            p.next_flag = static_cast<uint32_t*>(ptr(next_flag));
            p.seq = seq;
            p.counter = static_cast<uint32_t*>(ptr(counter));
            p.timeout_ticks = dnn::chain_ticks(hop_timeout_s);
            r.res_flag = static_cast<const uint32_t*>(ptr(res_flag));
            r.res_err = static_cast<uint32_t*>(ptr(res_err));
            r.res_dev = ptr(res_dev);
            r.res_host = ptr(res_host);
            r.res_bytes = res_bytes;
            r.last_ack = static_cast<uint32_t*>(ptr(last_ack));
            r.wait_timeout_s = wait_timeout_s;
            chk(h.enqueue(r, slot), "ChainHost.request");
          },
          py::arg("slot"), py::arg("stream"), py::arg("res_stream"), py::arg("x_dev"),
          py::arg("x_host"), py::arg("x_bytes"), py::arg("w"), py::arg("ldw"), py::arg("bias"),
          py::arg("act"), py::arg("rows"), py::arg("N"), py::arg("K"), py::arg("dst"),
          py::arg("dst_ld"), py::arg("dst_hdr"), py::arg("err"), py::arg("ack"),
          py::arg("ack_target"), py::arg("next_flag"), py::arg("seq"), py::arg("counter"),
          py::arg("hop_timeout_s"), py::arg("res_flag"), py::arg("res_err"), py::arg("res_dev"),
          py::arg("res_host"), py::arg("res_bytes"), py::arg("last_ack"),
          py::arg("wait_timeout_s"))
      .def(
          "wait",
          [](dnn::ChainHost& h, int slot, double timeout_s) {
            py::gil_scoped_release nogil;
            const int rc = h.wait(slot, timeout_s);
            if (rc < 0) throw std::runtime_error("ChainHost.wait: hipEventQuery failed");
            return rc;
          },
          py::arg("slot"), py::arg("timeout_s"));
  m.def(
      "chain_stage_run",
      [=](uintptr_t s, uintptr_t in_flags, uintptr_t in_hdrs, uintptr_t in_slots, long ldx,
          uintptr_t prev_ack, uintptr_t w, long ldw, uintptr_t bias, int act, int N, int K,
          int out_f32, uintptr_t dst, long dst_slot_bytes, long dst_ld, uintptr_t dst_hdr,
          long hdr_stride, uintptr_t next_flags, uintptr_t ack, uintptr_t stop, uintptr_t done,
          uintptr_t sync, uint32_t start_seq, uint32_t epoch, int stage, int nslot,
          int max_rows, double idle_s, double timeout_s, int workgroups, int share) {
        dnn::ChainStage p{};
        p.in_flags = static_cast<const uint32_t*>(ptr(in_flags));
        p.in_hdrs = static_cast<const uint32_t*>(ptr(in_hdrs));
        p.in_slots = static_cast<const uint16_t*>(ptr(in_slots));
        p.ldx = ldx;
        p.prev_ack = static_cast<uint32_t*>(ptr(prev_ack));
        p.w = static_cast<const uint16_t*>(ptr(w));
        p.ldw = ldw;
        p.bias = static_cast<const float*>(ptr(bias));
        p.act = act;
        p.N = N;
        p.K = K;
        p.out_f32 = out_f32;
        p.dst = static_cast<char*>(ptr(dst));
        p.dst_slot_bytes = dst_slot_bytes;
        p.dst_ld = dst_ld;
        p.dst_hdr = static_cast<uint32_t*>(ptr(dst_hdr));
        p.hdr_stride = hdr_stride;
        p.next_flags = static_cast<uint32_t*>(ptr(next_flags));
        p.ack = static_cast<const uint32_t*>(ptr(ack));
        p.stop = static_cast<const uint32_t*>(ptr(stop));
        p.done = static_cast<uint32_t*>(ptr(done));
        p.sync = static_cast<uint32_t*>(ptr(sync));
        p.start_seq = start_seq;
        p.epoch = epoch;
        p.stage = stage;
        p.nslot = nslot;
        p.max_rows = max_rows;
        p.idle_ticks = dnn::chain_ticks(idle_s);
        p.timeout_ticks = dnn::chain_ticks(timeout_s);
        const int want = workgroups > 0 ? workgroups : dnn::chain_stage_workgroups(N, act);
        const int wg = dnn::chain_stage_run(p, want, share, S(s));
        if (wg < 1) chk(wg, "chain_stage_run");
        return wg;
      },
      py::arg("stream"), py::arg("in_flags"), py::arg("in_hdrs"), py::arg("in_slots"),
      py::arg("ldx"), py::arg("prev_ack"), py::arg("w"), py::arg("ldw"), py::arg("bias"),
      py::arg("act"), py::arg("N"), py::arg("K"), py::arg("out_f32"), py::arg("dst"),
      py::arg("dst_slot_bytes"), py::arg("dst_ld"), py::arg("dst_hdr"), py::arg("hdr_stride"),
      py::arg("next_flags"), py::arg("ack"), py::arg("stop"), py::arg("done"), py::arg("sync"),
      py::arg("start_seq"), py::arg("epoch"), py::arg("stage"), py::arg("nslot"),
      py::arg("max_rows"), py::arg("idle_s"), py::arg("timeout_s"), py::arg("workgroups") = 0,
      py::arg("share") = 1);
  m.def(
      "chain_signal",
      [=](uintptr_t s, uintptr_t flag, uint32_t value) {
        chk(dnn::chain_signal(static_cast<uint32_t*>(ptr(flag)), value, S(s)), "chain_signal");
      },
      py::arg("stream"), py::arg("flag"), py::arg("value"));
  m.def("device_sync", []() {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) throw std::runtime_error(hipGetErrorString(e));
  });
}
