// Host-only self-test of the native runtime, built with -fsanitize=address,undefined by
// tests/test_native_asan.py (GPU sanitizers are not available on the pool; the host runtime --
// JSON weight IO, protobuf codec, schedule generator/simulator -- is where memory bugs in our
// C++ would live). Exits non-zero on any failed check; ASan/UBSan abort on memory errors.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>

#include "runtime/json_weights.hpp"
#include "runtime/matrix_codec.hpp"
#include "runtime/schedule.hpp"

static int failures = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

template <class F>
static bool throws(F f) {
  try {
    f();
  } catch (const std::exception&) {
    return true;
  }
  return false;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(-1.f, 1.f);

  // ---- neuron JSON: write -> parse round trip (model + stage forms) ----
  std::vector<std::vector<float>> W = {std::vector<float>(16 * 7), std::vector<float>(3 * 16)};
  std::vector<std::vector<float>> B = {std::vector<float>(16), std::vector<float>(3)};
  for (auto& v : W)
    for (auto& x : v) x = U(rng);
  for (auto& v : B)
    for (auto& x : v) x = U(rng);
  std::vector<dnn::LayerOut> L(2);
  L[0] = {16, 7, W[0].data(), B[0].data(), "relu", "hidden"};
  L[1] = {3, 16, W[1].data(), B[1].data(), "softmax", "output"};
  for (int stage = 0; stage < 2; ++stage) {
    const std::string p = dir + (stage ? "/st.json" : "/m.json");
    dnn::write_neuron_json_file(p, L, stage ? std::vector<int>{} : std::vector<int>{1, 1}, stage);
    dnn::ParsedModel M = dnn::parse_neuron_json_file(p);
    CHECK(M.layers.size() == 2);
    CHECK(M.stage_file == (stage == 1));
    CHECK(M.layers[0].in_dim == 7 && M.layers[1].in_dim == 16);
    CHECK(M.layers[1].activation == "softmax");
    for (size_t i = 0; i < W[0].size(); ++i) CHECK(M.layers[0].weights[i] == W[0][i]);
    for (size_t i = 0; i < B[1].size(); ++i) CHECK(M.layers[1].bias[i] == B[1][i]);
    if (!stage) CHECK(M.has_distribution && M.layer_distribution.size() == 2);
  }
  // malformed / adversarial inputs must throw, never read out of bounds
  const char* bad[] = {"", "{", "{\"layers\":[", "{\"layers\":[{\"neurons\":[{\"weights\":[1,2",
                       "{\"layers\":[{\"neurons\":[{\"weights\":[1],\"bias\":1},{\"weights\":[1,2]}]}]}",
                       "{\"layer_x\":[{\"weights\":[1]}]}", "{\"layers\":[{\"neurons\":[{\"bias\":1}]}]}",
                       "{\"a\":\"unterminated"};
  for (const char* s : bad) {
    std::string buf(s);  // exact-size heap buffer: ASan catches any over-read
    char* heap = (char*)std::malloc(buf.size() ? buf.size() : 1);
    std::memcpy(heap, buf.data(), buf.size());
    CHECK(throws([&] { dnn::parse_neuron_json(heap, buf.size()); }) || buf == "{");
    std::free(heap);
  }
  {  // examples: nested inputs flattened, raw lists, ragged rejected
    const std::string ex = "{\"examples\":[{\"input\":[[1,2],[3,4]],\"label\":5},"
                           "{\"input\":[[5,6],[7,8]],\"label\":null}]}";
    char* heap = (char*)std::malloc(ex.size());
    std::memcpy(heap, ex.data(), ex.size());
    dnn::ParsedExamples E = dnn::parse_examples_json(heap, ex.size());
    std::free(heap);
    CHECK(E.n == 2 && E.dim == 4 && E.outer_len == 2 && E.labels[0] == 5 && E.labels[1] == -1);
    const std::string rag = "{\"examples\":[[1,2],[3]]}";
    CHECK(throws([&] { dnn::parse_examples_json(rag.data(), rag.size()); }));
  }

  // ---- Matrix codec: random round trips + truncated / corrupted buffers ----
  for (int t = 0; t < 50; ++t) {
    const long rows = rng() % 9, cols = rng() % 300;
    std::vector<double> a((size_t)(rows * cols));
    for (auto& x : a) x = U(rng);
    const std::string enc = dnn::encode_matrix(a.data(), rows, cols);
    dnn::DecodedMatrix d = dnn::decode_matrix((const uint8_t*)enc.data(), enc.size());
    CHECK(d.rows == rows && (rows == 0 || cols == 0 || d.cols == cols));
    CHECK(d.data == a || cols == 0);
    for (size_t cut = 1; cut < enc.size() && cut < 40; cut += 3) {  // truncations
      uint8_t* h = (uint8_t*)std::malloc(cut);
      std::memcpy(h, enc.data(), cut);
      try {
        dnn::decode_matrix(h, cut);
      } catch (const std::exception&) {
      }
      std::free(h);
    }
    std::string bad2 = enc;  // random corruption
    for (int k = 0; k < 5 && !bad2.empty(); ++k) bad2[rng() % bad2.size()] = (char)(rng() & 0xff);
    uint8_t* h = (uint8_t*)std::malloc(bad2.size() + 1);
    std::memcpy(h, bad2.data(), bad2.size());
    try {
      dnn::decode_matrix(h, bad2.size());
    } catch (const std::exception&) {
    }
    std::free(h);
  }

  // ---- schedules ----
  for (const char* k : {"gpipe", "1f1b", "1f1b_w", "zb"})
    for (int S = 1; S <= 8; ++S)
      for (int M = 1; M <= 12; M += 3) {
        for (int s = 0; s < S; ++s) CHECK(dnn::make_schedule(k, S, M, s).back().kind == dnn::OpKind::OPT);
        auto r = dnn::simulate_schedule(k, S, M, {1.0}, {2.0}, {0.5}, 0.1);
        CHECK(std::get<0>(r) > 0 && std::get<2>(r) >= 0 && std::get<2>(r) < 1);
      }
  CHECK(throws([] { dnn::make_schedule("nope", 2, 2, 0); }));
  CHECK(throws([] { dnn::make_schedule("gpipe", 2, 2, 5); }));

  std::printf("runtime selftest: %s (%d failures)\n", failures ? "FAIL" : "OK", failures);
  return failures ? 1 : 0;
}
