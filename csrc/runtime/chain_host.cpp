// Rank 0's native request path of the device-side serving chain (chain_host.hpp).
#include "chain_host.hpp"

#include <chrono>
#include <stdexcept>
#include <thread>

namespace dnn {

ChainHost::ChainHost(int slots) : ev_(slots, nullptr) {
  for (auto& e : ev_)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      throw std::runtime_error("ChainHost: hipEventCreateWithFlags failed");
}

ChainHost::~ChainHost() {
  for (auto e : ev_)
    if (e) (void)hipEventDestroy(e);
}

int ChainHost::enqueue(const ChainRequest& r, int slot) {
  if (slot < 0 || slot >= (int)ev_.size()) return -1;
  if (hipMemcpyAsync(r.x_dev, r.x_host, r.x_bytes, hipMemcpyHostToDevice, r.stream) !=
      hipSuccess)
    return -20;
  int rc = chain_gemv_send(r.send, r.stream);
  if (rc) return rc;
  rc = chain_wait(r.res_flag, r.send.seq, r.res_err, r.wait_timeout_s, r.res_stream);
  if (rc) return rc;
  if (hipMemcpyAsync(r.res_host, r.res_dev, r.res_bytes, hipMemcpyDeviceToHost,
                     r.res_stream) != hipSuccess)
    return -21;
  rc = chain_signal(r.last_ack, r.send.seq, r.res_stream);  // the result slot is free again
  if (rc) return rc;
  return hipEventRecord(ev_[slot], r.res_stream) == hipSuccess ? 0 : -22;
}

int ChainHost::wait(int slot, double timeout_s) {
  const auto t_end = std::chrono::steady_clock::now() +
                     std::chrono::duration<double>(timeout_s);
  for (long spins = 0;; ++spins) {
    const hipError_t q = hipEventQuery(ev_[slot]);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return -23;
    if (std::chrono::steady_clock::now() > t_end) return 1;
    if (spins > 20000) std::this_thread::sleep_for(std::chrono::microseconds(5));
  }
}

}  // namespace dnn
