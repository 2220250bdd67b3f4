#include "json_weights.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace dnn {
namespace {

struct Cursor {
  const char* p;
  const char* e;
  const char* begin;

  [[noreturn]] void fail(const std::string& what) const {
    throw std::runtime_error("neuron JSON parse error at byte " + std::to_string(p - begin) +
                             ": " + what);
  }
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  char peek() {
    ws();
    return p < e ? *p : '\0';
  }
  void expect(char c) {
    ws();
    if (p >= e || *p != c) fail(std::string("expected '") + c + "'");
    ++p;
  }
  bool consume(char c) {
    ws();
    if (p < e && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
  std::string str() {
    expect('"');
    std::string out;
    while (p < e && *p != '"') {
      if (*p == '\\') {
        ++p;
        if (p >= e) fail("bad escape");
        switch (*p) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u':
            out += "\\u";  // kept verbatim: keys/activations are ASCII in this format
            break;
          default: out += *p;
        }
        ++p;
      } else {
        out += *p++;
      }
    }
    if (p >= e) fail("unterminated string");
    ++p;
    return out;
  }
  double num() {
    ws();
    double v = 0.0;
    auto r = std::from_chars(p, e, v);
    if (r.ec != std::errc()) {
      // JSON literals that NumPy/json.dump can emit for floats
      if (e - p >= 3 && !std::strncmp(p, "NaN", 3)) {
        p += 3;
        return std::nan("");
      }
      if (e - p >= 8 && !std::strncmp(p, "Infinity", 8)) {
        p += 8;
        return 1.0 / 0.0;
      }
      if (e - p >= 9 && !std::strncmp(p, "-Infinity", 9)) {
        p += 9;
        return -1.0 / 0.0;
      }
      fail("expected a number");
    }
    p = r.ptr;
    return v;
  }
  void skip() {  // skip any JSON value
    char c = peek();
    if (c == '"') {
      str();
    } else if (c == '{' || c == '[') {
      int depth = 0;
      while (p < e) {
        char ch = *p;
        if (ch == '"') {
          str();
          continue;
        }
        if (ch == '{' || ch == '[') ++depth;
        if (ch == '}' || ch == ']') {
          if (--depth == 0) {
            ++p;
            return;
          }
        }
        ++p;
      }
      fail("unterminated container");
    } else if (c == 't' || c == 'f' || c == 'n') {
      while (p < e && std::isalpha((unsigned char)*p)) ++p;
    } else {
      num();
    }
  }
};

// neurons array -> layer (appends rows)
void parse_neurons(Cursor& c, ParsedLayer& L) {
  c.expect('[');
  bool first = true;
  int count = 0;
  if (c.consume(']')) return;
  do {
    c.expect('{');
    std::string act = "linear";
    double bias = 0.0;
    size_t before = L.weights.size();
    bool have_w = false;
    if (!c.consume('}')) {
      do {
        std::string key = c.str();
        c.expect(':');
        if (key == "weights") {
          have_w = true;
          c.expect('[');
          if (!c.consume(']')) {
            do {
              // 2-D weight rows are flattened (schema allows only 1-D, be lenient)
              if (c.peek() == '[') {
                c.expect('[');
                if (!c.consume(']')) {
                  do L.weights.push_back((float)c.num());
                  while (c.consume(','));
                  c.expect(']');
                }
              } else {
                L.weights.push_back((float)c.num());
              }
            } while (c.consume(','));
            c.expect(']');
          }
        } else if (key == "bias") {
          bias = c.num();
        } else if (key == "activation") {
          act = c.str();
        } else {
          c.skip();
        }
      } while (c.consume(','));
      c.expect('}');
    }
    const int n_w = (int)(L.weights.size() - before);
    if (!have_w) c.fail("neuron without \"weights\"");
    if (first) {
      L.in_dim = n_w;
      L.activation = act;
      first = false;
    } else {
      if (n_w != L.in_dim)
        c.fail("ragged neuron weights in layer: " + std::to_string(n_w) + " vs " +
               std::to_string(L.in_dim));
      if (act != L.activation) L.mixed_activation = true;
    }
    L.bias.push_back((float)bias);
    ++count;
  } while (c.consume(','));
  c.expect(']');
  if (L.nodes == 0) L.nodes = count;
}

void parse_layers_array(Cursor& c, ParsedModel& M) {
  c.expect('[');
  if (c.consume(']')) return;
  do {
    ParsedLayer L;
    int declared_nodes = -1;
    c.expect('{');
    if (!c.consume('}')) {
      do {
        std::string key = c.str();
        c.expect(':');
        if (key == "type") L.type = c.str();
        else if (key == "nodes") declared_nodes = (int)c.num();
        else if (key == "neurons") parse_neurons(c, L);
        else c.skip();
      } while (c.consume(','));
      c.expect('}');
    }
    const int n_neurons = (int)L.bias.size();
    L.nodes = declared_nodes >= 0 ? declared_nodes : n_neurons;
    M.layers.push_back(std::move(L));
  } while (c.consume(','));
  c.expect(']');
}

void parse_model_object(Cursor& c, ParsedModel& M, bool top) {
  c.expect('{');
  std::vector<std::pair<long, ParsedLayer>> staged;
  if (!c.consume('}')) {
    do {
      std::string key = c.str();
      c.expect(':');
      if (key == "layers") {
        parse_layers_array(c, M);
      } else if (top && key == "model" && c.peek() == '{') {
        M.wrapped = true;
        parse_model_object(c, M, false);
      } else if (key == "layer_distribution") {
        M.has_distribution = true;
        M.layer_distribution.clear();
        c.expect('[');
        if (!c.consume(']')) {
          do M.layer_distribution.push_back((int)c.num());
          while (c.consume(','));
          c.expect(']');
        }
      } else if (key.rfind("layer_", 0) == 0 && c.peek() == '[') {
        ParsedLayer L;
        L.key = key;
        parse_neurons(c, L);
        char* endp = nullptr;
        long k = std::strtol(key.c_str() + 6, &endp, 10);
        if (!endp || *endp) c.fail("stage-file key must be layer_<int>: " + key);
        if (!L.bias.empty()) staged.emplace_back(k, std::move(L));  // grpc_node.py:49 skip
      } else {
        c.skip();
      }
    } while (c.consume(','));
    c.expect('}');
  }
  if (!staged.empty()) {
    std::stable_sort(staged.begin(), staged.end(),
                     [](const auto& a, const auto& b) { return a.first < b.first; });
    M.stage_file = true;
    for (auto& kv : staged) M.layers.push_back(std::move(kv.second));
  }
}

}  // namespace

ParsedModel parse_neuron_json(const char* data, size_t size) {
  Cursor c{data, data + size, data};
  ParsedModel M;
  parse_model_object(c, M, true);
  return M;
}

namespace {
// Flatten one (possibly nested) numeric array; returns the top-level length.
int flat_numbers(Cursor& c, std::vector<float>& out) {
  c.expect('[');
  int top = 0;
  if (c.consume(']')) return 0;
  do {
    if (c.peek() == '[') flat_numbers(c, out);
    else out.push_back((float)c.num());
    ++top;
  } while (c.consume(','));
  c.expect(']');
  return top;
}
}  // namespace

ParsedExamples parse_examples_json(const char* data, size_t size) {
  Cursor c{data, data + size, data};
  ParsedExamples E;
  c.expect('{');
  if (c.consume('}')) return E;
  do {
    std::string key = c.str();
    c.expect(':');
    if (key != "examples") {
      c.skip();
      continue;
    }
    c.expect('[');
    if (c.consume(']')) continue;
    do {
      const size_t before = E.x.size();
      int label = -1, outer = 0;
      if (c.peek() == '[') {
        E.raw_list = true;
        outer = flat_numbers(c, E.x);
      } else {
        c.expect('{');
        if (!c.consume('}')) {
          do {
            std::string k = c.str();
            c.expect(':');
            if (k == "input") outer = flat_numbers(c, E.x);
            else if (k == "label" && c.peek() != 'n') label = (int)c.num();
            else c.skip();
          } while (c.consume(','));
          c.expect('}');
        }
      }
      const int d = (int)(E.x.size() - before);
      if (E.n == 0) {
        E.dim = d;
        E.outer_len = outer;
      } else if (d != E.dim) {
        c.fail("example " + std::to_string(E.n) + " has " + std::to_string(d) +
               " values, expected " + std::to_string(E.dim));
      }
      E.labels.push_back(label);
      ++E.n;
    } while (c.consume(','));
    c.expect(']');
  } while (c.consume(','));
  c.expect('}');
  return E;
}

template <class R, class Fn>
static R with_mmap(const std::string& path, Fn fn) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    throw std::runtime_error("cannot stat " + path);
  }
  const size_t n = (size_t)st.st_size;
  if (n == 0) {
    ::close(fd);
    throw std::runtime_error("empty file " + path);
  }
  void* mem = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (mem == MAP_FAILED) throw std::runtime_error("mmap failed for " + path);
  madvise(mem, n, MADV_SEQUENTIAL);
  try {
    R r = fn((const char*)mem, n);
    munmap(mem, n);
    return r;
  } catch (...) {
    munmap(mem, n);
    throw;
  }
}

ParsedExamples parse_examples_json_file(const std::string& path) {
  return with_mmap<ParsedExamples>(path, [](const char* d, size_t n) { return parse_examples_json(d, n); });
}

ParsedModel parse_neuron_json_file(const std::string& path) {
  return with_mmap<ParsedModel>(path, [](const char* d, size_t n) { return parse_neuron_json(d, n); });
}

namespace {
struct Out {
  FILE* f;
  char buf[64];
  void s(const char* x) { std::fputs(x, f); }
  void s(const std::string& x) { std::fwrite(x.data(), 1, x.size(), f); }
  void fl(float v) {
    auto r = std::to_chars(buf, buf + sizeof(buf), (double)v);  // shortest round-trip of the
    std::fwrite(buf, 1, r.ptr - buf, f);                        // fp32 value as a double
  }
  void i(long v) { std::fprintf(f, "%ld", v); }
};

void write_neurons(Out& o, const LayerOut& L) {
  o.s("[");
  for (int n = 0; n < L.out; ++n) {
    o.s(n ? ",\n{\"weights\":[" : "\n{\"weights\":[");
    const float* row = L.w + (long)n * L.in;
    for (int k = 0; k < L.in; ++k) {
      if (k) o.s(",");
      o.fl(row[k]);
    }
    o.s("],\"bias\":");
    o.fl(L.b[n]);
    o.s(",\"activation\":\"");
    o.s(L.activation);
    o.s("\"}");
  }
  o.s("]");
}
}  // namespace

void write_neuron_json_file(const std::string& path, const std::vector<LayerOut>& layers,
                            const std::vector<int>& distribution, bool stage_file) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + path);
  static char iobuf[1 << 20];
  std::setvbuf(f, iobuf, _IOFBF, sizeof(iobuf));
  Out o{f, {}};
  if (stage_file) {
    o.s("{");
    for (size_t l = 0; l < layers.size(); ++l) {
      o.s(l ? ",\n\"layer_" : "\"layer_");
      o.i((long)l + 1);
      o.s("\":");
      write_neurons(o, layers[l]);
    }
    o.s("}\n");
  } else {
    o.s("{\"layers\":[");
    for (size_t l = 0; l < layers.size(); ++l) {
      const LayerOut& L = layers[l];
      o.s(l ? ",\n{\"type\":\"" : "\n{\"type\":\"");
      o.s(L.type);
      o.s("\",\"nodes\":");
      o.i(L.out);
      o.s(",\"neurons\":");
      write_neurons(o, L);
      o.s("}");
    }
    o.s("]");
    if (!distribution.empty()) {
      o.s(",\n\"layer_distribution\":[");
      for (size_t i = 0; i < distribution.size(); ++i) {
        if (i) o.s(",");
        o.i(distribution[i]);
      }
      o.s("]");
    }
    o.s("}\n");
  }
  const bool bad = std::ferror(f);
  std::fclose(f);
  if (bad) throw std::runtime_error("write error on " + path);
}

}  // namespace dnn
