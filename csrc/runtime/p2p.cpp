#include "p2p.hpp"

#include "kernels/elementwise.hpp"

#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>

namespace dnn {
namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

std::mutex mu;
std::map<std::string, void*> opened;  // handle bytes -> mapped base (opened once per process)

}  // namespace

std::pair<std::string, uint64_t> ipc_export(void* ptr) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  ck(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr)),
     "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  ck(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base)), "hipIpcGetMemHandle");
  return {std::string(reinterpret_cast<const char*>(&h), sizeof(h)),
          (uint64_t)(reinterpret_cast<char*>(ptr) - reinterpret_cast<char*>(base))};
}

void* ipc_import(const std::string& handle, uint64_t offset) {
  if (handle.size() != sizeof(hipIpcMemHandle_t))
    throw std::invalid_argument("ipc_import: bad handle size");
  std::lock_guard<std::mutex> g(mu);
  auto it = opened.find(handle);
  void* base = nullptr;
  if (it != opened.end()) {
    base = it->second;
  } else {
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle.data(), sizeof(h));
    ck(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    opened[handle] = base;
  }
  return static_cast<char*>(base) + offset;
}

void* alloc_uncached(size_t bytes) {
  void* p = nullptr;
  ck(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags");
  ck(hipMemset(p, 0, bytes), "hipMemset");
  return p;
}

void free_device(void* p) {
  if (p) (void)hipFree(p);
}

bool can_access_peer(int dev, int peer) {
  int ok = 0;
  if (dev == peer) return true;
  return hipDeviceCanAccessPeer(&ok, dev, peer) == hipSuccess && ok != 0;
}

void ipc_close_all() {
  std::lock_guard<std::mutex> g(mu);
  for (auto& kv : opened) (void)hipIpcCloseMemHandle(kv.second);
  opened.clear();
}

// Copies and flag writes are kernels (kernels/elementwise.hip p2p_copy / p2p_signal): the
// runtime's hipMemcpyAsync / hipStreamWriteValue32 into IPC-imported memory block the host.
void copy_async(void* dst, const void* src, size_t n, hipStream_t s) {
  if (p2p_copy(dst, src, n, s) != 0) throw std::runtime_error("p2p_copy failed");
}

void signal_u32(hipStream_t s, void* flag, uint32_t v) {
  if (p2p_signal(reinterpret_cast<uint32_t*>(flag), v, s) != 0)
    throw std::runtime_error("p2p_signal failed");
}

void wait_geq_u32(hipStream_t s, void* flag, uint32_t v) {
  ck(hipStreamWaitValue32(s, flag, v, hipStreamWaitValueGte, 0xFFFFFFFFu), "hipStreamWaitValue32");
}

}  // namespace dnn
