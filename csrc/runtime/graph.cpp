#include "graph.hpp"

#include <stdexcept>
#include <string>

namespace dnn {

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

GraphExec::~GraphExec() { reset(); }

void GraphExec::reset() {
  if (exec_) hipGraphExecDestroy(exec_);
  if (graph_) hipGraphDestroy(graph_);
  exec_ = nullptr;
  graph_ = nullptr;
  nodes_ = 0;
}

void GraphExec::begin_capture(hipStream_t s) {
  if (capturing_) throw std::runtime_error("GraphExec: capture already in progress");
  if (!s) throw std::runtime_error("GraphExec: refuse to capture the legacy null stream");
  reset();
  // Relaxed mode: the capturing thread may still call non-stream-ordered APIs; every buffer the
  // captured step touches is allocated before capture begins.
  hip_check(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
  capturing_ = s;
}

void GraphExec::end_capture() {
  if (!capturing_) throw std::runtime_error("GraphExec: end_capture without begin_capture");
  hipStream_t s = capturing_;
  capturing_ = nullptr;
  hip_check(hipStreamEndCapture(s, &graph_), "hipStreamEndCapture");
  hip_check(hipGraphGetNodes(graph_, nullptr, &nodes_), "hipGraphGetNodes");
  hip_check(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "hipGraphInstantiate");
}

void GraphExec::replay(hipStream_t s) {
  if (!exec_) throw std::runtime_error("GraphExec: nothing captured");
  hip_check(hipGraphLaunch(exec_, s), "hipGraphLaunch");
}

}  // namespace dnn
