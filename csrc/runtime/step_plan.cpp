#include "runtime/step_plan.hpp"
#include "runtime/p2p.hpp"
#include "kernels/chain.hpp"
#include "kernels/elementwise.hpp"

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include <mutex>
#include <set>
#include <stdexcept>

namespace dnn {
namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

NcclApi g_api;
bool g_loaded = false;
std::mutex g_mu;

template <class F>
void sym(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  if (!f) throw std::runtime_error(std::string("librccl: missing symbol ") + name);
}

}  // namespace

const NcclApi& nccl_load(const std::string& path) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_loaded) {
    if (path != g_api.path) throw std::runtime_error("nccl_load: a different librccl is bound");
    return g_api;
  }
  // NOLOAD: bind to the RCCL instance that created the communicators (torch's), never a
  // second copy whose internal state would not know them
  void* h = dlopen(path.c_str(), RTLD_LAZY | RTLD_NOLOAD);
  if (!h) throw std::runtime_error("nccl_load: " + path + " is not loaded in this process");
  NcclApi a;
  sym(h, "ncclSend", a.send);
  sym(h, "ncclRecv", a.recv);
  sym(h, "ncclAllReduce", a.all_reduce);
  sym(h, "ncclReduceScatter", a.reduce_scatter);
  sym(h, "ncclAllGather", a.all_gather);
  sym(h, "ncclGroupStart", a.group_start);
  sym(h, "ncclGroupEnd", a.group_end);
  sym(h, "ncclCommCount", a.comm_count);
  sym(h, "ncclCommUserRank", a.comm_user_rank);
  sym(h, "ncclCommGetAsyncError", a.async_error);
  sym(h, "ncclGetErrorString", a.error_string);
  a.path = path;
  g_api = a;
  g_loaded = true;
  return g_api;
}

const NcclApi* nccl_api() { return g_loaded ? &g_api : nullptr; }

static double default_wait_timeout_s() {
  const char* e = std::getenv("DNN_FLAG_TIMEOUT");
  return e ? std::atof(e) : 120.0;
}

StepPlan::StepPlan(int n_streams, int n_events) : wait_timeout_(default_wait_timeout_s()) {
  if (n_streams < 1 || n_events < 0) throw std::invalid_argument("StepPlan: bad sizes");
  for (int i = 1; i < n_streams; ++i) {
    hipStream_t s;
    ck(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    streams_.push_back(s);
    hipEvent_t e;
    ck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    join_.push_back(e);
  }
  for (int i = 0; i < n_events; ++i) {
    hipEvent_t e;
    ck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    events_.push_back(e);
  }
  ck(hipEventCreateWithFlags(&fork_, hipEventDisableTiming), "hipEventCreate");
  ck(hipMalloc(&dev_, 2 * sizeof(uint32_t)), "hipMalloc");
  ck(hipMemset(dev_, 0, 2 * sizeof(uint32_t)), "hipMemset");
  ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
}

void StepPlan::set_seq(uint32_t s) {
  if (s == seq_) return;
  seq_ = s;
  ck(hipMemcpy(dev_, &s, sizeof(s), hipMemcpyHostToDevice), "hipMemcpy");
}

void StepPlan::sync_seq() {
  ck(hipMemcpy(&seq_, dev_, sizeof(seq_), hipMemcpyDeviceToHost), "hipMemcpy");
}

uint32_t StepPlan::flag_timeouts() const {
  uint32_t e = 0;
  ck(hipMemcpy(&e, dev_ + 1, sizeof(e), hipMemcpyDeviceToHost), "hipMemcpy");
  return e;
}


StepPlan::~StepPlan() {
  for (auto e : events_) (void)hipEventDestroy(e);
  for (auto e : join_) (void)hipEventDestroy(e);
  if (fork_) (void)hipEventDestroy(fork_);
  for (auto s : streams_) (void)hipStreamDestroy(s);
  if (dev_) (void)hipFree(dev_);
  if (counters_) (void)hipFree(counters_);
}

void StepPlan::add(const Op& op) {
  if (op.stream < 0 || op.stream > (int)streams_.size())
    throw std::out_of_range("StepPlan op: stream index");
  if ((op.kind == REC || op.kind == WAIT) && (op.event < 0 || op.event >= (int)events_.size()))
    throw std::out_of_range("StepPlan op: event id");
  if (op.kind == SEG && (!op.prog || op.seg.empty()))
    throw std::invalid_argument("StepPlan op: SEG needs a program and a segment");
  const bool rccl = op.kind == SEND || op.kind == RECV || op.kind == ALLREDUCE ||
                    op.kind == REDUCE_SCATTER || op.kind == ALL_GATHER;
  if (rccl && (!op.comm || !nccl_api()))
    throw std::invalid_argument("StepPlan op: RCCL op without a communicator / nccl_load");
  if ((op.kind == SIGNAL || op.kind == WAITV) && !op.a)
    throw std::invalid_argument("StepPlan op: flag address");
  if (op.kind == GSTART || op.kind == GEND) {
    if (!nccl_api()) throw std::invalid_argument("StepPlan op: RCCL group without nccl_load");
    // a group holds RCCL ops of ONE stream only, and groups do not nest
    if (op.kind == GSTART && group_open_ >= 0)
      throw std::invalid_argument("StepPlan op: nested RCCL group");
    if (op.kind == GEND && group_open_ != op.stream)
      throw std::invalid_argument("StepPlan op: GEND without GSTART on its stream");
    group_open_ = op.kind == GSTART ? op.stream : -1;
  } else if (group_open_ >= 0 && (!(op.kind == SEND || op.kind == RECV) ||
                                  op.stream != group_open_)) {
    throw std::invalid_argument("StepPlan op: only SEND / RECV of the group's stream in a group");
  }
  if (op.kind == COPYSIG) throw std::invalid_argument("StepPlan op: COPYSIG is internal");
  // a flag that follows its copy on the same stream rides in the copy's launch
  static const bool merge = [] {
    const char* e = std::getenv("DNN_PLAN_COPYSIG");
    return !(e && e[0] == '0');
  }();
  if (merge && op.kind == SIGNAL && !ops_.empty() && ops_.back().kind == COPY &&
      ops_.back().stream == op.stream && n_counters_ < MAX_COUNTERS) {
    if (!counters_) {
      ck(hipMalloc(&counters_, MAX_COUNTERS * sizeof(uint32_t)), "hipMalloc");
      ck(hipMemset(counters_, 0, MAX_COUNTERS * sizeof(uint32_t)), "hipMemset");
      ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
    }
    Op& c = ops_.back();
    c.kind = COPYSIG;
    c.flag = op.a;
    c.delta = op.delta;
    c.counter = n_counters_++;
    return;
  }
  ops_.push_back(op);
}

static void nck(int rc, const char* what) {
  if (rc != 0) {
    const NcclApi* a = nccl_api();
    throw std::runtime_error(std::string(what) + " failed: " +
                             (a ? a->error_string(rc) : "rccl") + " (" + std::to_string(rc) + ")");
  }
}

// DNN_PLAN_TRACE=1: host timestamp of every op before it is issued (stderr) -- finds an
// issue call that blocks the host thread (a plan must never wait on the GPU while enqueuing).
static bool plan_trace() {
  static const bool on = [] {
    const char* e = std::getenv("DNN_PLAN_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}

void StepPlan::run(hipStream_t main) {
  if (group_open_ >= 0) throw std::runtime_error("StepPlan::run: RCCL group left open");
  ++seq_;
  if (p2p_seq_advance(dev_, main) != 0) throw std::runtime_error("p2p_seq_advance failed");
  ck(hipEventRecord(fork_, main), "hipEventRecord");
  for (auto s : streams_) ck(hipStreamWaitEvent(s, fork_, 0), "hipStreamWaitEvent");
  std::vector<std::string> one(1);
  const NcclApi* nc = nccl_api();
  const bool trace = plan_trace();
  int idx = 0;
  for (const Op& o : ops_) {
    hipStream_t s = stream(o.stream, main);
    if (trace) {
      const auto t = std::chrono::steady_clock::now().time_since_epoch();
      std::fprintf(stderr, "plan seq %llu op %d kind %d stream %d t_us %lld\n",
                   (unsigned long long)seq_, idx, (int)o.kind, o.stream,
                   (long long)std::chrono::duration_cast<std::chrono::microseconds>(t).count());
    }
    ++idx;
    switch (o.kind) {
      case SEG:
        one[0] = o.seg;
        o.prog->run(one, s);
        break;
      case SEND:
        nck(nc->send(reinterpret_cast<const void*>(o.a), o.count, o.dtype, o.peer, o.comm, s),
            "ncclSend");
        break;
      case RECV:
        nck(nc->recv(reinterpret_cast<void*>(o.a), o.count, o.dtype, o.peer, o.comm, s),
            "ncclRecv");
        break;
      case ALLREDUCE:  // in place, sum
        nck(nc->all_reduce(reinterpret_cast<const void*>(o.a), reinterpret_cast<void*>(o.a),
                           o.count, o.dtype, 0, o.comm, s),
            "ncclAllReduce");
        break;
      case REDUCE_SCATTER:  // a = full input, b = this rank's chunk (count elements)
        nck(nc->reduce_scatter(reinterpret_cast<const void*>(o.a), reinterpret_cast<void*>(o.b),
                               o.count, o.dtype, 0, o.comm, s),
            "ncclReduceScatter");
        break;
      case ALL_GATHER:  // a = this rank's chunk (count elements), b = full output
        nck(nc->all_gather(reinterpret_cast<const void*>(o.a), reinterpret_cast<void*>(o.b),
                           o.count, o.dtype, o.comm, s),
            "ncclAllGather");
        break;
      case COPY:  // kernels, not hipMemcpyAsync / hipStreamWriteValue32 (runtime/p2p.cpp)
        copy_async(reinterpret_cast<void*>(o.b), reinterpret_cast<const void*>(o.a), o.count, s);
        break;
      case COPYSIG:
        if (p2p_copy_signal_seq(reinterpret_cast<void*>(o.b), reinterpret_cast<const void*>(o.a),
                                o.count, reinterpret_cast<uint32_t*>(o.flag), dev_,
                                (int)o.delta, counters_ + o.counter, s) != 0)
          throw std::runtime_error("p2p_copy_signal_seq failed");
        break;
      case SIGNAL:  // flag = device step number + delta (kernels: capturable, non-blocking)
        if (p2p_signal_seq(reinterpret_cast<uint32_t*>(o.a), dev_, (int)o.delta, s) != 0)
          throw std::runtime_error("p2p_signal_seq failed");
        break;
      case WAITV:
        if (p2p_wait_seq(reinterpret_cast<const uint32_t*>(o.a), dev_, (int)o.delta, dev_ + 1,
                         wait_timeout_, s) != 0)
          throw std::runtime_error("p2p_wait_seq failed");
        break;
      case REC:
        ck(hipEventRecord(events_[o.event], s), "hipEventRecord");
        break;
      case WAIT:
        ck(hipStreamWaitEvent(s, events_[o.event], 0), "hipStreamWaitEvent");
        break;
      case GSTART:
        nck(nc->group_start(), "ncclGroupStart");
        break;
      case GEND:
        nck(nc->group_end(), "ncclGroupEnd");
        break;
    }
  }
  for (size_t i = 0; i < streams_.size(); ++i) {
    ck(hipEventRecord(join_[i], streams_[i]), "hipEventRecord");
    ck(hipStreamWaitEvent(main, join_[i], 0), "hipStreamWaitEvent");
  }
}

int StepPlan::comm_error() const {
  const NcclApi* nc = nccl_api();
  if (!nc) return 0;
  std::set<void*> seen;
  for (const Op& o : ops_) {
    if (!o.comm || !seen.insert(o.comm).second) continue;
    int err = 0;
    const int rc = nc->async_error(o.comm, &err);
    if (rc != 0) return rc;
    if (err != 0) return err;
  }
  return 0;
}

}  // namespace dnn
