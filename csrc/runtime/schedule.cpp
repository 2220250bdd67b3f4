#include "schedule.hpp"

#include <algorithm>
#include <deque>
#include <stdexcept>

namespace dnn {

static void check_args(int S, int M, int s) {
  if (S < 1 || M < 1 || s < 0 || s >= S)
    throw std::invalid_argument("make_schedule: need num_stages>=1, num_micro>=1, 0<=stage<S");
}

std::vector<SchedOp> make_schedule(const std::string& kind, int S, int M, int s) {
  check_args(S, M, s);
  std::vector<SchedOp> ops;
  auto F = [&](int j) { ops.push_back({OpKind::FWD, j}); };
  auto B = [&](int j) { ops.push_back({OpKind::BWD, j}); };
  auto W = [&](int j) { ops.push_back({OpKind::WGRAD, j}); };

  if (kind == "gpipe") {
    for (int j = 0; j < M; ++j) F(j);
    for (int j = 0; j < M; ++j) B(j);
    W(-1);
  } else if (kind == "1f1b" || kind == "1f1b_w" || kind == "zb" || kind == "1f1b_lh") {
    const bool eager_w = kind == "1f1b_w";
    const bool zb = kind == "zb";
    // 1f1b_lh (latency hiding): 3x the warm-up forwards. Classic 1F1B keeps only S - s
    // micro-batches in flight on stage s, which covers the round trip to the last stage only
    // when hops are free; with a hop of about one micro-batch's compute that round trip is
    // ~3x longer, and the extra in-flight micro-batches (their rows are allocated anyway) keep
    // both link directions busy: per micro-batch max(compute, hop) instead of up to
    // compute + 2 hops (parallel/plan_sim.py, tests/test_step_plan_sim_cpu.py).
    const int warm = std::min((kind == "1f1b_lh" ? 3 : 1) * (S - s - 1), M);
    std::deque<int> pending_w;
    int f = 0, b = 0;
    for (; f < warm; ++f) F(f);
    // steady state: one forward, one backward
    for (; f < M; ++f) {
      F(f);
      B(b);
      if (eager_w) W(b);
      else if (zb) pending_w.push_back(b);
      ++b;
    }
    // cool-down: remaining backwards; zb fills the gradient waits with deferred W's
    for (; b < M; ++b) {
      B(b);
      if (eager_w) W(b);
      else if (zb) {
        pending_w.push_back(b);
        W(pending_w.front());
        pending_w.pop_front();
      }
    }
    if (zb) {
      while (!pending_w.empty()) {
        W(pending_w.front());
        pending_w.pop_front();
      }
    } else if (!eager_w) {
      W(-1);
    }
  } else {
    throw std::invalid_argument("unknown schedule kind '" + kind +
                                "' (gpipe | 1f1b | 1f1b_lh | 1f1b_w | zb)");
  }
  ops.push_back({OpKind::OPT, -1});
  return ops;
}

static double pick(const std::vector<double>& v, int s) {
  if (v.empty()) return 0.0;
  return v.size() == 1 ? v[0] : v.at(s);
}

std::tuple<double, std::vector<double>, double> simulate_schedule(
    const std::string& kind, int S, int M, const std::vector<double>& t_fwd,
    const std::vector<double>& t_bwd, const std::vector<double>& t_wgrad, double t_comm) {
  std::vector<std::vector<SchedOp>> prog(S);
  for (int s = 0; s < S; ++s) prog[s] = make_schedule(kind, S, M, s);
  const double NA = -1.0;
  std::vector<std::vector<double>> fend(S, std::vector<double>(M, NA));
  std::vector<std::vector<double>> bend(S, std::vector<double>(M, NA));
  std::vector<size_t> pc(S, 0);
  std::vector<double> clock(S, 0.0), busy(S, 0.0);
  size_t remaining = 0;
  for (auto& p : prog) remaining += p.size();

  while (remaining) {
    bool progress = false;
    for (int s = 0; s < S; ++s) {
      while (pc[s] < prog[s].size()) {
        const SchedOp& op = prog[s][pc[s]];
        double ready = clock[s], cost = 0.0;
        if (op.kind == OpKind::FWD) {
          if (s > 0) {
            if (fend[s - 1][op.micro] < 0) break;
            ready = std::max(ready, fend[s - 1][op.micro] + t_comm);
          }
          cost = pick(t_fwd, s);
        } else if (op.kind == OpKind::BWD) {
          if (s < S - 1) {
            if (bend[s + 1][op.micro] < 0) break;
            ready = std::max(ready, bend[s + 1][op.micro] + t_comm);
          }
          cost = pick(t_bwd, s);
        } else if (op.kind == OpKind::WGRAD) {
          cost = pick(t_wgrad, s) * (op.micro < 0 ? M : 1);
        }
        const double end = ready + cost;
        if (op.kind == OpKind::FWD) fend[s][op.micro] = end;
        if (op.kind == OpKind::BWD) bend[s][op.micro] = end;
        clock[s] = end;
        busy[s] += cost;
        ++pc[s];
        --remaining;
        progress = true;
      }
    }
    if (!progress) throw std::runtime_error("simulate_schedule: schedule deadlocks");
  }
  const double makespan = *std::max_element(clock.begin(), clock.end());
  double bubble = 0.0;
  for (int s = 0; s < S; ++s) bubble += makespan > 0 ? 1.0 - busy[s] / makespan : 0.0;
  return {makespan, busy, bubble / S};
}

}  // namespace dnn
