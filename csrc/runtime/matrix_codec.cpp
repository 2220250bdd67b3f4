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

// One row's values, visited in order: fn(ptr, count) for each packed run / unpacked double.
template <class F>
static void for_each_run(Reader row, F&& fn) {
  while (row.p < row.e) {
    const uint64_t t = row.varint();
    const int f = (int)(t >> 3), w = (int)(t & 7);
    if (f == 1 && w == 2) {  // packed doubles
      const uint64_t bl = row.varint();
      if (bl % 8 || (uint64_t)(row.e - row.p) < bl)
        throw std::runtime_error("Matrix decode: bad packed double run");
      fn(row.p, (size_t)(bl / 8));
      row.p += bl;
    } else if (f == 1 && w == 1) {  // unpacked double
      if (row.e - row.p < 8) throw std::runtime_error("Matrix decode: truncated double");
      fn(row.p, (size_t)1);
      row.p += 8;
    } else {
      row.skip(w);
    }
  }
}

// Rows of the Matrix, visited in order: fn(Reader over the row's bytes).
template <class F>
static void for_each_row(const uint8_t* buf, size_t n, F&& fn) {
  Reader r{buf, buf + n};
  while (r.p < r.e) {
    const uint64_t tag = r.varint();
    const int field = (int)(tag >> 3), wire = (int)(tag & 7);
    if (field != 1 || wire != 2) {
      r.skip(wire);
      continue;
    }
    const uint64_t len = r.varint();
    if ((uint64_t)(r.e - r.p) < len) throw std::runtime_error("Matrix decode: truncated row");
    fn(Reader{r.p, r.p + len});
    r.p += len;
  }
}

void scan_matrix(const uint8_t* buf, size_t n, long* rows, long* cols) {
  long nr = 0, nc = -1;
  for_each_row(buf, n, [&](Reader row) {
    long c = 0;
    for_each_run(row, [&](const uint8_t*, size_t k) { c += (long)k; });
    if (nc < 0) nc = c;
    else if (c != nc)
      throw std::invalid_argument("Matrix decode: rows have different lengths (" +
                                  std::to_string(c) + " vs " + std::to_string(nc) + ")");
    ++nr;
  });
  *rows = nr;
  *cols = nc < 0 ? 0 : nc;
}

void fill_matrix(const uint8_t* buf, size_t n, double* out, long cols) {
  long i = 0;
  for_each_row(buf, n, [&](Reader row) {
    double* dst = out + i * cols;
    for_each_run(row, [&](const uint8_t* p, size_t k) {
      std::memcpy(dst, p, k * 8);
      dst += k;
    });
    ++i;
  });
}

DecodedMatrix decode_matrix(const uint8_t* buf, size_t n) {
  DecodedMatrix M;
  scan_matrix(buf, n, &M.rows, &M.cols);
  M.data.resize((size_t)M.rows * (size_t)M.cols);
  if (!M.data.empty()) fill_matrix(buf, n, M.data.data(), M.cols);
  return M;
}

size_t encoded_size(long rows, long cols) {
  const uint64_t payload = (uint64_t)cols * 8;
  const uint64_t row_len = cols ? 1 + varint_len(payload) + payload : 0;
  return (size_t)rows * (1 + varint_len(row_len) + row_len);
}

static char* put_varint_raw(char* d, uint64_t v) {
  while (v >= 0x80) {
    *d++ = (char)(v | 0x80);
    v >>= 7;
  }
  *d++ = (char)v;
  return d;
}

void encode_matrix_into(const double* data, long rows, long cols, char* d) {
  const uint64_t payload = (uint64_t)cols * 8;
  const uint64_t row_len = cols ? 1 + varint_len(payload) + payload : 0;
  for (long i = 0; i < rows; ++i) {
    *d++ = 0x0A;
    d = put_varint_raw(d, row_len);
    if (cols) {
      *d++ = 0x0A;
      d = put_varint_raw(d, payload);
      std::memcpy(d, data + i * cols, payload);
      d += payload;
    }
  }
}

std::string encode_matrix(const double* data, long rows, long cols) {
  std::string s(encoded_size(rows, cols), '\0');
  encode_matrix_into(data, rows, cols, s.data());
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
