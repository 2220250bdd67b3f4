// Peer-to-peer pipeline transport primitives over xGMI: IPC-mapped peer buffers and
// stream-ordered flags (SURVEY §5 "fast path for tiny messages": the producer writes the
// activation straight into the consumer's input buffer and raises a flag the consumer's
// stream waits on -- no RCCL kernel, no receive-side copy).
//
//   exporter:  ipc_export(ptr) -> (handle bytes, offset inside its allocation)
//   importer:  ipc_import(handle, offset) -> a pointer to the same memory, usable by kernels,
//              copies and stream memory operations of this process (hipIpcOpenMemHandle with
//              lazy peer access; dmabuf IPC, HSA_ENABLE_IPC_MODE_LEGACY=0)
//   producer:  copy_async(peer_dst, src, n, stream); signal(stream, peer_flag, seq)
//   consumer:  wait_geq(stream, my_flag, seq)  (hipStreamWaitValue32: the stream, not the host,
//              waits)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <utility>

namespace dnn {

std::pair<std::string, uint64_t> ipc_export(void* ptr);
void* ipc_import(const std::string& handle, uint64_t offset);
void ipc_close_all();
// Device memory the L2 does not cache (hipDeviceMallocUncached), zeroed: the receive buffers
// of xGMI peer writes. A peer's stores land in this GPU's HBM without touching its L2s (one
// per XCD, not coherent with each other or with the peer), so a cached copy of the previous
// step's rows could otherwise be read back stale.
void* alloc_uncached(size_t bytes);
void free_device(void* p);
bool can_access_peer(int dev, int peer);
void copy_async(void* dst, const void* src, size_t n, hipStream_t s);
void signal_u32(hipStream_t s, void* flag, uint32_t v);
void wait_geq_u32(hipStream_t s, void* flag, uint32_t v);

}  // namespace dnn
