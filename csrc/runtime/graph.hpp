// HIP graph capture/replay of a launch-bound step (cdna guide §6: "capture launch-bound inner
// loops in hipGraphs"). The engine captures a whole single-stage training step -- every GEMM,
// loss, reduction and optimizer launch, ~20 kernels -- and replays it with one hipGraphLaunch.
#pragma once
#include <hip/hip_runtime.h>

#include <stddef.h>

namespace dnn {

class GraphExec {
 public:
  GraphExec() = default;
  ~GraphExec();
  GraphExec(const GraphExec&) = delete;
  GraphExec& operator=(const GraphExec&) = delete;

  void begin_capture(hipStream_t s);
  void end_capture();
  void replay(hipStream_t s);
  bool captured() const { return exec_ != nullptr; }
  size_t num_nodes() const { return nodes_; }
  void reset();

 private:
  hipStream_t capturing_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  size_t nodes_ = 0;
};

}  // namespace dnn
