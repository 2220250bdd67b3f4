#include "runtime/program.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <stdexcept>

namespace dnn {

Program*& recording_program() {
  static thread_local Program* p = nullptr;
  return p;
}

void Program::add(const char* what, Launch fn) { recs_.push_back({what, std::move(fn)}); }

void Program::close() {
  if (!open_.empty()) {
    segs_[open_] = {open_begin_, recs_.size()};
    order_.push_back(open_);
    open_.clear();
  }
}

void Program::mark(const std::string& name) {
  close();
  if (segs_.count(name)) throw std::invalid_argument("segment recorded twice: " + name);
  open_ = name;
  open_begin_ = recs_.size();
}

int Program::region(uint64_t base, uint64_t size) {
  for (const Region& r : regions_)
    if (base < r.base + r.size && r.base < base + size)
      throw std::invalid_argument("overlapping relocation regions");
  regions_.push_back({base, size, base});
  return (int)regions_.size() - 1;
}

void Program::rebase(int id, uint64_t new_base) {
  if (id < 0 || id >= (int)regions_.size()) throw std::out_of_range("bad region id");
  regions_[id].cur = new_base;
}

uint64_t Program::fix_addr(uint64_t p) const {
  for (const Region& r : regions_)
    if (p >= r.base && p < r.base + r.size) return r.cur + (p - r.base);
  return p;
}

static bool roctx_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("DNN_ROCTX");
    return e && e[0] == '1';
  }();
  return on;
}

void Program::run_range(size_t b, size_t e, hipStream_t s, const char* seg) const {
  const bool tx = roctx_enabled();
  if (tx) roctx_push(seg);
  for (size_t i = b; i < e; ++i) {
    const int rc = recs_[i].fn(s, *this);
    if (rc != 0) {
      if (tx) roctx_pop();
      throw std::runtime_error(std::string("replay of ") + recs_[i].what + " in segment " + seg +
                               " failed with code " + std::to_string(rc));
    }
  }
  if (tx) roctx_pop();
}

void Program::run(const std::vector<std::string>& names, hipStream_t stream) const {
  for (const std::string& n : names) {
    auto it = segs_.find(n);
    if (it == segs_.end()) throw std::out_of_range("no recorded segment " + n);
    run_range(it->second.first, it->second.second, stream, n.c_str());
  }
}

void Program::run_all(hipStream_t stream) const { run_range(0, recs_.size(), stream, "all"); }

std::vector<std::string> Program::segments() const { return order_; }

size_t Program::segment_size(const std::string& name) const {
  auto it = segs_.find(name);
  if (it == segs_.end()) throw std::out_of_range("no recorded segment " + name);
  return it->second.second - it->second.first;
}

void Program::clear() {
  recs_.clear();
  segs_.clear();
  order_.clear();
  open_.clear();
  regions_.clear();
}

// ---- roctx ------------------------------------------------------------------------------
namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    void* h = dlopen("libroctx64.so.4", RTLD_LAZY | RTLD_NOLOAD);
    if (!h) h = dlopen("libroctx64.so", RTLD_LAZY | RTLD_NOLOAD);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_LAZY);
    if (h) {
      push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    }
  }
};
const Roctx& roctx() {
  static const Roctx r;
  return r;
}
}  // namespace

void roctx_push(const char* name) {
  if (roctx().push) roctx().push(name);
}
void roctx_pop() {
  if (roctx().pop) roctx().pop();
}

}  // namespace dnn
