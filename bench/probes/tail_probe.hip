// Probe library for bench/probes/tail_probe.py: the fused classifier tail compiled on its own
// with -DDNN_TAIL_PROBE=<bits> (parts of the kernel removed, see mlp_tail.hip), launched
// through a C entry point so several variants can be timed side by side in one process.
#include "kernels/mlp_tail.hip"

extern "C" int tail_probe_launch(const dnn::TailParams* p, hipStream_t s) {
  return dnn::mlp_tail(*p, s);
}
