#include "matrix_codec.hpp"

#include <cstring>
#include <stdexcept>

namespace dnn {
namespace {

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  uint64_t varint() {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      if (p >= e) throw std::runtime_error("Matrix decode: truncated varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
      shift += 7;
      if (shift > 63) throw std::runtime_error("Matrix decode: varint too long");
    }
  }
  void skip(int wire) {
    switch (wire) {
      case 0: varint(); break;
      case 1: advance(8); break;
      case 2: advance(varint()); break;
      case 5: advance(4); break;
      default: throw std::runtime_error("Matrix decode: unsupported wire type");
    }
  }
  void advance(uint64_t n) {
    if ((uint64_t)(e - p) < n) throw std::runtime_error("Matrix decode: truncated field");
    p += n;
  }
};

void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}

size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}

}  // namespace

DecodedMatrix decode_matrix(const uint8_t* buf, size_t n) {
  DecodedMatrix M;
  Reader r{buf, buf + n};
  long cols = -1;
  while (r.p < r.e) {
    const uint64_t tag = r.varint();
    const int field = (int)(tag >> 3), wire = (int)(tag & 7);
    if (field != 1 || wire != 2) {
      r.skip(wire);
      continue;
    }
    const uint64_t len = r.varint();
    if ((uint64_t)(r.e - r.p) < len) throw std::runtime_error("Matrix decode: truncated row");
    Reader row{r.p, r.p + len};
    r.p += len;
    const size_t before = M.data.size();
    while (row.p < row.e) {
      const uint64_t t = row.varint();
      const int f = (int)(t >> 3), w = (int)(t & 7);
      if (f == 1 && w == 2) {  // packed doubles
        const uint64_t bl = row.varint();
        if (bl % 8 || (uint64_t)(row.e - row.p) < bl)
          throw std::runtime_error("Matrix decode: bad packed double run");
        const size_t k = bl / 8;
        M.data.resize(M.data.size() + k);
        std::memcpy(M.data.data() + M.data.size() - k, row.p, bl);
        row.p += bl;
      } else if (f == 1 && w == 1) {  // unpacked double
        double v;
        if (row.e - row.p < 8) throw std::runtime_error("Matrix decode: truncated double");
        std::memcpy(&v, row.p, 8);
        row.p += 8;
        M.data.push_back(v);
      } else {
        row.skip(w);
      }
    }
    const long c = (long)(M.data.size() - before);
    if (cols < 0) cols = c;
    else if (c != cols)
      throw std::invalid_argument("Matrix decode: rows have different lengths (" +
                                  std::to_string(c) + " vs " + std::to_string(cols) + ")");
    ++M.rows;
  }
  M.cols = cols < 0 ? 0 : cols;
  return M;
}

std::string encode_matrix(const double* data, long rows, long cols) {
  std::string s;
  const uint64_t payload = (uint64_t)cols * 8;
  const uint64_t row_len = cols ? 1 + varint_len(payload) + payload : 0;
  s.reserve((size_t)rows * (1 + varint_len(row_len) + row_len));
  for (long i = 0; i < rows; ++i) {
    s.push_back(0x0A);
    put_varint(s, row_len);
    if (cols) {
      s.push_back(0x0A);
      put_varint(s, payload);
      s.append(reinterpret_cast<const char*>(data + i * cols), payload);
    }
  }
  return s;
}

std::string encode_matrix_f32(const float* data, long rows, long cols, long ld) {
  std::string s;
  const uint64_t payload = (uint64_t)cols * 8;
  const uint64_t row_len = cols ? 1 + varint_len(payload) + payload : 0;
  s.reserve((size_t)rows * (1 + varint_len(row_len) + row_len));
  std::vector<double> tmp((size_t)cols);
  for (long i = 0; i < rows; ++i) {
    s.push_back(0x0A);
    put_varint(s, row_len);
    if (cols) {
      for (long j = 0; j < cols; ++j) tmp[j] = data[i * ld + j];
      s.push_back(0x0A);
      put_varint(s, payload);
      s.append(reinterpret_cast<const char*>(tmp.data()), payload);
    }
  }
  return s;
}

}  // namespace dnn
