// Native protobuf wire codec for the reference's RPC payload
//   message Row    { repeated double values = 1; }   (proto3: packed)
//   message Matrix { repeated Row rows = 1; }
// (/root/reference/src/proto/dist_nn.proto:5-11).
//
// The reference converted every hop list<->protobuf in Python (grpc_node.py:107,113,126-127;
// run_grpc_inference.py:135-137,147) -- SURVEY §6.2 measured ~83 ms per 668x784 hop, >99% of
// chain time. This codec maps the wire bytes straight to/from a dense float64 row-major array
// and accepts both packed and unpacked encodings of `values`, so any standard protobuf client
// (including the reference's generated stubs) interoperates with our gRPC ingress.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace dnn {

struct DecodedMatrix {
  std::vector<double> data;  // [rows][cols]
  long rows = 0, cols = 0;
};

DecodedMatrix decode_matrix(const uint8_t* buf, size_t n);
std::string encode_matrix(const double* data, long rows, long cols);

// Zero-intermediate forms (the bindings write straight into the numpy array / bytes object):
// scan_matrix validates the wire bytes and returns the shape (ragged rows throw
// std::invalid_argument); fill_matrix then copies the values of the same bytes into
// out[rows][cols]. encoded_size + encode_matrix_into write the wire bytes into a caller buffer.
void scan_matrix(const uint8_t* buf, size_t n, long* rows, long* cols);
void fill_matrix(const uint8_t* buf, size_t n, double* out, long cols);
size_t encoded_size(long rows, long cols);
void encode_matrix_into(const double* data, long rows, long cols, char* dst);
std::string encode_matrix_f32(const float* data, long rows, long cols, long ld);

}  // namespace dnn
