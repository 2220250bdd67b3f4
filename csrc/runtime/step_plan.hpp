// Native multi-rank training step: one C++ call per step for a rank that owns one pipeline
// stage (and possibly a data-parallel group).
//
// The reference chains its stages with one synchronous protobuf RPC per request and hop
// (/root/reference/src/grpc_node.py:120-135). Here a step is a precomputed list of operations
// that the engine builds ONCE from the pipeline schedule (parallel/pipeline.py) and replays
// per step with no Python in the loop:
//   SEG    replay a recorded Program segment (F3, B3, W, FIN, O, ...) on a stream
//   SEND / RECV / ALLREDUCE   RCCL point-to-point / collective on a communicator (the
//          ncclComm_t that torch.distributed already created for a process group; RCCL entry
//          points are resolved from the librccl the process has loaded -- same library, same
//          communicator objects, no second RCCL instance)
//   COPY / SIGNAL / WAITV     xGMI peer-write transport: a device copy into an IPC-mapped
//          peer buffer and stream-ordered 32-bit flags (hipStreamWriteValue32 /
//          hipStreamWaitValue32) carrying the step sequence number (value = seq + delta)
//   REC / WAIT  event record on one stream / another stream waits for it
//   GSTART / GEND  ncclGroupStart / ncclGroupEnd around the RCCL ops between them (one kernel
//          per group: its sends and receives progress together)
// Streams: index 0 is the caller's stream; the plan owns the others (per-direction comm
// streams, a data-parallel stream). Every run forks all plan streams from stream 0 first and
// joins them back at the end, so a step is ordered like one kernel on the caller's stream and
// the whole step can be captured into a HIP graph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "runtime/program.hpp"

namespace dnn {

// RCCL entry points (ncclResult_t as int, ncclComm_t as void*), resolved with dlopen(NOLOAD).
struct NcclApi {
  int (*send)(const void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*recv)(void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*all_reduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*reduce_scatter)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*all_gather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  int (*group_start)() = nullptr;
  int (*group_end)() = nullptr;
  int (*comm_count)(void*, int*) = nullptr;
  int (*comm_user_rank)(void*, int*) = nullptr;
  int (*async_error)(void*, int*) = nullptr;
  const char* (*error_string)(int) = nullptr;
  std::string path;
};

// Resolve from `path` (the librccl torch loaded); throws if it is not loaded or lacks a symbol.
const NcclApi& nccl_load(const std::string& path);
const NcclApi* nccl_api();  // nullptr until nccl_load succeeded

class StepPlan {
 public:
  // COPYSIG is never added from outside: add() merges a SIGNAL that directly follows a COPY
  // on the same stream into the COPY (one kernel: kernels/chain.hpp p2p_copy_signal_seq)
  enum Kind { SEG = 0, SEND, RECV, ALLREDUCE, REDUCE_SCATTER, ALL_GATHER, COPY, SIGNAL, WAITV,
              REC, WAIT, GSTART, GEND, COPYSIG };
  struct Op {
    Kind kind;
    int stream = 0;
    const Program* prog = nullptr;
    std::string seg;
    void* comm = nullptr;
    uint64_t a = 0, b = 0;  // buffers (send/recv/copy src, dst) or flag address
    uint64_t count = 0;     // elements (RCCL) / bytes (COPY)
    int dtype = 0, peer = 0;
    int64_t delta = 0;      // SIGNAL / WAITV value = seq + delta
    int event = 0, src = 0; // REC: event id on `stream`; WAIT: `stream` waits event id
    uint64_t flag = 0;      // COPYSIG: the merged SIGNAL's flag (value = seq + delta)
    int counter = -1;       // COPYSIG: its arrival counter slot
  };

  explicit StepPlan(int n_streams, int n_events);
  ~StepPlan();
  StepPlan(const StepPlan&) = delete;
  StepPlan& operator=(const StepPlan&) = delete;

  void add(const Op& op);
  void clear_ops() {
    ops_.clear();
    group_open_ = -1;
    n_counters_ = 0;  // (the counters are back at 0 after every completed run)
  }
  // One step on `main`; advances the sequence number first (seq() = 1 in the first step).
  void run(hipStream_t main);
  uint32_t seq() const { return seq_; }
  // Sets the step number (host mirror and the device counter the flag kernels read); not
  // during a capture.
  void set_seq(uint32_t s);
  // Flag waits that timed out (device error word; reading it synchronises the device).
  uint32_t flag_timeouts() const;
  // Host mirror := device step number (after graph replays advanced it on the device).
  void sync_seq();
  size_t size() const { return ops_.size(); }
  int n_streams() const { return (int)streams_.size() + 1; }
  // RCCL async-error poll over every communicator the plan uses (0 = healthy).
  int comm_error() const;
  // Seconds a WAITV spins before it gives up and raises the error word. Steady state: long
  // (DNN_FLAG_TIMEOUT, default 120 s) -- a wait that gives up lets the plan consume rows that
  // never arrived. The first-step verification (engine/trainer.py) sets a short one.
  double wait_timeout() const { return wait_timeout_; }
  void set_wait_timeout(double s) { wait_timeout_ = s; }

 private:
  hipStream_t stream(int i, hipStream_t main) const { return i == 0 ? main : streams_[i - 1]; }
  std::vector<hipStream_t> streams_;
  std::vector<hipEvent_t> events_;
  hipEvent_t fork_ = nullptr;
  std::vector<hipEvent_t> join_;
  std::vector<Op> ops_;
  uint32_t seq_ = 0;
  int group_open_ = -1;  // stream of the RCCL group being added, -1 = none
  double wait_timeout_;
  // [0] = step number read by the SIGNAL / WAITV kernels, [1] = wait-timeout error word
  uint32_t* dev_ = nullptr;
  // COPYSIG arrival counters (one per merged op, zero between runs); merging can be turned
  // off with DNN_PLAN_COPYSIG=0
  uint32_t* counters_ = nullptr;
  int n_counters_ = 0;
  static constexpr int MAX_COUNTERS = 4096;
};

}  // namespace dnn
