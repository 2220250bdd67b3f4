// Native step executor: a recorded, replayable list of kernel launches.
//
// The Python engine decides WHAT runs (shapes, tiles, buffer pointers, validation); a Program
// records those launches once -- every kernel binding in bindings.cpp appends a closure
// instead of launching while a Program is recording on the calling thread -- and then replays
// named segments of it ("F3" = forward of micro-batch 3, "B3", "W", "FIN", "O", ...) from C++
// with no Python per kernel. This is the C++ hot loop of SURVEY §7.1 (the reference's stage
// loop is /root/reference/src/grpc_node.py:100-135, one Python RPC handler per request).
//
// Unlike a HIP graph, a replay (a) interleaves with host-side communication issued between
// segments (pipeline send/recv, DP all-reduce buckets), and (b) can RELOCATE pointers: a
// registered region [base, base+size) is re-based at replay time, so e.g. the first stage can
// read each step's input directly from a resident dataset slice (zero-copy) although the
// launches were recorded against its staging buffer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace dnn {

class Program {
 public:
  // A recorded launch: returns 0 or a negative precondition/launch code.
  using Launch = std::function<int(hipStream_t, const Program&)>;

  void add(const char* what, Launch fn);
  // Start a named segment at the current end (closes the previous one).
  void mark(const std::string& name);
  void close();
  // Relocatable pointer region; returns its id.
  int region(uint64_t base, uint64_t size);
  void rebase(int id, uint64_t new_base);
  // Device pointer as of the current bases (identity outside every region).
  template <class T>
  T* fix(T* p) const {
    return reinterpret_cast<T*>(fix_addr(reinterpret_cast<uint64_t>(p)));
  }
  uint64_t fix_addr(uint64_t p) const;

  // Replay segments in order on `stream`; throws std::runtime_error naming the failed launch.
  void run(const std::vector<std::string>& names, hipStream_t stream) const;
  void run_all(hipStream_t stream) const;

  size_t size() const { return recs_.size(); }
  std::vector<std::string> segments() const;
  size_t segment_size(const std::string& name) const;
  void clear();

 private:
  struct Rec {
    const char* what;
    Launch fn;
  };
  struct Region {
    uint64_t base, size, cur;
  };
  void run_range(size_t b, size_t e, hipStream_t s, const char* seg) const;

  std::vector<Rec> recs_;
  std::unordered_map<std::string, std::pair<size_t, size_t>> segs_;
  std::vector<std::string> order_;
  std::string open_;
  size_t open_begin_ = 0;
  std::vector<Region> regions_;
};

// Program recording on this thread (nullptr = launch immediately).
Program*& recording_program();

// Optional roctx ranges around replayed segments (DNN_ROCTX=1): resolved from the libroctx64
// already loaded by the process, no link-time dependency.
void roctx_push(const char* name);
void roctx_pop();

}  // namespace dnn
