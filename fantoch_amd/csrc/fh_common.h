// fh_common.h -- shared host/device helpers for the fantoch_hip engine.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/fantoch_hip.h"

namespace fh {

// --- dots (fantoch/src/id.rs:21-27) -------------------------
__host__ __device__ inline uint64_t make_dot(uint32_t src, uint64_t seq) {
  return (uint64_t(src) << 56) | seq;
}
__host__ __device__ inline uint32_t dot_src(uint64_t d) { return uint32_t(d >> 56); }
__host__ __device__ inline uint64_t dot_seq(uint64_t d) { return d & 0x00FFFFFFFFFFFFFFull; }

// --- errors -----------------------------------------------------------------
struct Error : std::runtime_error {
  fh_status code;
  Error(fh_status c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define FH_HIP(expr)                                                          \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess)                                                     \
      throw ::fh::Error(_e == hipErrorOutOfMemory ? FH_EOOM : FH_EHIP,        \
                        std::string(#expr) + ": " + hipGetErrorString(_e) +   \
                            " (" __FILE__ ":" + std::to_string(__LINE__) +    \
                            ")");                                             \
  } while (0)

#define FH_CHECK(cond, code, msg)                                             \
  do {                                                                        \
    if (!(cond)) throw ::fh::Error((code), (msg));                            \
  } while (0)

// Host: wait for a completion word `*done == seq` that a kernel stores into
// mapped host memory, spinning on the word and querying the stream now and
// then (query() returns the stream's hipStreamQuery status).  A failed
// launch raises its HIP error; a stream that finished without the word
// raises FH_EINVARIANT; work that has not finished after deadline_ms raises
// FH_EHIP ("<what> did not complete within ...") instead of spinning
// forever on a kernel that never ends.
template <class Q>
void poll_completion(const volatile uint32_t *done, uint32_t seq, Q query, double deadline_ms,
                     const char *what = "graph_small: the pass") {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1; *done != seq; i++) {
    if ((i & 1023) != 0) continue;
    const hipError_t st = query();
    if (st == hipErrorNotReady) {
      if ((i & 65535) == 0 &&
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() >
              deadline_ms)
        throw Error(FH_EHIP, std::string(what) + " did not complete within " +
                                 std::to_string(uint64_t(deadline_ms)) +
                                 " ms (the handle is no longer usable)");
      continue;
    }
    FH_HIP(st);
    FH_CHECK(*done == seq, FH_EINVARIANT, std::string(what) + " ended without its completion word");
  }
}

// --- device buffer ----------------------------------------------------------
template <class T>
struct DBuf {
  T *p = nullptr;
  size_t cap = 0;
  DBuf() = default;
  DBuf(const DBuf &) = delete;
  DBuf &operator=(const DBuf &) = delete;
  ~DBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  // Ensure capacity for n elements (contents not preserved).
  T *ensure(size_t n) {
    if (n <= cap && p) return p;
    release();
    size_t c = n < 16 ? 16 : n;
    FH_HIP(hipMalloc(reinterpret_cast<void **>(&p), c * sizeof(T)));
    cap = c;
    return p;
  }
  T *get() const { return p; }
  void swap(DBuf &o) {
    std::swap(p, o.p);
    std::swap(cap, o.cap);
  }
};

// The fused engine keeps every staged command's dot in a device-resident
// command log; the single-view latest table stores log positions tagged with
// kLogFlag (top byte 0, so never a dot; >= 2^48, so never an in-batch
// "index + 1" dependency).  Dots are read from the log when results are read.
constexpr uint64_t kLogFlag = uint64_t(1) << 48;
__host__ __device__ inline bool is_log_ref(uint64_t x) { return (x >> 56) == 0 && x >= kLogFlag; }

inline unsigned grid_for(size_t n, unsigned block, unsigned cap = 8192) {
  size_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return unsigned(g);
}

// Number of significant bits of (x - 1), at least 1: bits needed for ids < x.
inline int bits_for(uint64_t x) {
  int b = 1;
  while (b < 64 && (uint64_t(1) << b) < x) b++;
  return b;
}

// Roofline probe: HIP events around every launch of the named kernels on the
// stream they run on, plus the algorithmic bytes each launch moves.
struct ProbeSlot {
  std::string name;
  std::vector<hipEvent_t> ev;
  size_t next = 0;
  double bytes = 0;
};
struct Probe {
  std::vector<ProbeSlot> slots;
  // comma-separated kernel names ("" = off)
  void set(const std::string &csv) {
    for (auto &sl : slots)
      for (auto e : sl.ev) (void)hipEventDestroy(e);
    slots.clear();
    size_t a = 0;
    while (a < csv.size()) {
      size_t b = csv.find(',', a);
      if (b == std::string::npos) b = csv.size();
      if (b > a) slots.push_back(ProbeSlot{csv.substr(a, b - a)});
      a = b + 1;
    }
  }
  ProbeSlot *find(const char *name) {
    for (auto &sl : slots)
      if (sl.name == name) return &sl;
    return nullptr;
  }
  hipEvent_t take(ProbeSlot &sl) {
    if (sl.next >= sl.ev.size()) {
      hipEvent_t e;
      FH_HIP(hipEventCreate(&e));
      sl.ev.push_back(e);
    }
    return sl.ev[sl.next++];
  }
  void reset() {
    for (auto &sl : slots) {
      sl.next = 0;
      sl.bytes = 0;
    }
  }
  ~Probe() { set(""); }
};
extern thread_local Probe *t_probe;

// Launch `k` on stream `s`; when the thread's probe targets `name`, the launch
// carries a start/stop event pair via hipExtLaunchKernel, so the recorded
// interval is the kernel's own dispatch begin/end (the interval rocprofv3's
// kernel trace reports), not an event-marker bracket around it.
template <class F, class... Args>
inline void probed_launch(const char *name, double bytes, F k, dim3 grid, dim3 block,
                          hipStream_t s, Args... args) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (t_probe) {
    if (ProbeSlot *sl = t_probe->find(name)) {
      sl->bytes += bytes;
      e0 = t_probe->take(*sl);
      e1 = t_probe->take(*sl);
    }
  }
  hipExtLaunchKernelGGL(k, grid, block, 0, s, e0, e1, 0, args...);
  FH_HIP(hipGetLastError());
}

// Device selection per SURVEY §8b (shard -> device, or env override).
int pick_device(const fh_config *cfg, uint64_t shard_id);

// Thread-local last error.
void set_last_error(const std::string &m);

}  // namespace fh

// C-ABI wrappers: map exceptions to fh_status + thread-local message.
#define FH_API_BEGIN try {
#define FH_API_END                                                                \
  return FH_OK;                                                                   \
  }                                                                               \
  catch (const fh::Error &e) {                                                    \
    fh::set_last_error(e.what());                                                 \
    return e.code;                                                                \
  }                                                                               \
  catch (const std::bad_alloc &) {                                                \
    fh::set_last_error("host allocation failed");                                 \
    return FH_EOOM;                                                               \
  }                                                                               \
  catch (const std::exception &e) {                                               \
    fh::set_last_error(e.what());                                                 \
    return FH_EINVARIANT;                                                         \
  }

