// Pipeline-parallel step schedules (per-stage ordered compute ops) and an event simulator.
//
// The reference runs its layer chain strictly synchronously, one request in flight
// (/root/reference/src/grpc_node.py:120-135, /root/reference/src/run_grpc_inference.py:199-211).
// Our stages exchange micro-batches instead; this file decides the order in which each stage
// runs forward (F), backward-dgrad (B), weight-gradient (W) and optimizer (O) work.
//
// Kinds:
//   "gpipe"  : all F, then all B (same micro order), then one batched W over every micro-batch
//   "1f1b"   : warm-up F's, steady F/B pairs, cool-down B's, then one batched W
//   "1f1b_lh": 1f1b with 3x the warm-up forwards: hides hop latency (multi-GPU default)
//   "1f1b_w" : as 1f1b but W_j runs right after B_j (per-micro-batch wgrad, slab accumulation)
//   "zb"     : 1f1b whose cool-down interleaves per-micro W's into the slots where the stage
//              would wait for the next gradient (zero-bubble style W deferral)
#pragma once
#include <string>
#include <tuple>
#include <vector>

namespace dnn {

enum class OpKind : int { FWD = 0, BWD = 1, WGRAD = 2, OPT = 3 };

struct SchedOp {
  OpKind kind;
  int micro;  // micro-batch index; -1 for W over all micro-batches / OPT
};

std::vector<SchedOp> make_schedule(const std::string& kind, int num_stages, int num_micro,
                                   int stage);

// Simulates one step with per-stage op costs (vectors of length num_stages, or length 1 =
// uniform) and a fixed per-hop transfer time. A batched W costs num_micro * t_wgrad.
// Returns (makespan, per-stage busy time, mean bubble fraction).
std::tuple<double, std::vector<double>, double> simulate_schedule(
    const std::string& kind, int num_stages, int num_micro, const std::vector<double>& t_fwd,
    const std::vector<double>& t_bwd, const std::vector<double>& t_wgrad, double t_comm);

}  // namespace dnn
