// Rank 0's side of one device-side chain request (serve/fastpath.py FastChain.predict) as ONE
// native call: H2D of the request's bf16 rows, the stage's layer fused with the send
// (chain_gemv_send), and on the result stream the wait for the last stage's flag, one D2H of
// header + logits, the result slot's ack and an event; then a GIL-free spin on that event.
// Replaces ~10 Python-level launches and an event-polling loop per request.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../kernels/chain.hpp"

namespace dnn {

struct ChainRequest {
  hipStream_t stream, res_stream;
  void* x_dev;            // the stage's input buffer (device)
  const void* x_host;     // pinned host rows (bf16)
  size_t x_bytes;
  ChainGemvSend send;     // stage 0's (single) layer fused with its send
  const uint32_t* res_flag;  // rank 0's result flag of the slot (written by the last stage)
  uint32_t* res_err;      // wait outcome word inside the result slot's header
  const void* res_dev;    // result slot (header + fp32 rows)
  void* res_host;         // pinned host copy
  size_t res_bytes;
  uint32_t* last_ack;     // the last stage's ack word (IPC-mapped)
  double wait_timeout_s;  // device-side wait for the result flag
};

class ChainHost {
 public:
  explicit ChainHost(int slots);
  ~ChainHost();
  ChainHost(const ChainHost&) = delete;
  ChainHost& operator=(const ChainHost&) = delete;
  // Enqueue one request on slot `slot` (0 on success, a negative launch / copy error code).
  int enqueue(const ChainRequest& r, int slot);
  // Spin (no GIL held by the caller) until the slot's event completed: 0, or 1 after
  // timeout_s seconds.
  int wait(int slot, double timeout_s);

 private:
  std::vector<hipEvent_t> ev_;
};

}  // namespace dnn
