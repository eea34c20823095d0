// hoststage.h -- host side of the PCIe legs: validation and conversion of
// staged streams on several host threads, uploads through a ring of pinned
// chunks (the fill of chunk i+1 overlaps the DMA of chunk i), and read-backs
// through the same ring.
//
// SURVEY §8(d)(ii) asks for the PCIe-inclusive rate next to the device-
// resident one: a drop-in that feeds commands from the host
// (fantoch/src/run/task/executor.rs:150-175) sees staging + run + read-back.
// Pageable hipMemcpy runs through the runtime's own bounce buffers at a
// fraction of the link's rate, and single-threaded validation loops over
// 300M log entries dominated the round-5 stage (1,037 ms per 100M commands).
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fh_common.h"

namespace fh {

// Host threads for staging: OMP_NUM_THREADS when set (the GPU box sets it to
// its CPU share), else the hardware's, at most 16 either way.
inline size_t host_threads() {
  static const size_t n = [] {
    size_t t = std::thread::hardware_concurrency();
    if (const char *e = std::getenv("OMP_NUM_THREADS")) t = size_t(std::max(1L, atol(e)));
    return std::max<size_t>(1, std::min<size_t>(16, t ? t : 1));
  }();
  return n;
}

// The first error a worker raised (workers must not throw across a thread).
struct ParErr {
  std::atomic<bool> set{false};
  std::mutex m;
  fh_status code = FH_OK;
  std::string msg;
  void raise(fh_status c, const std::string &s) {
    std::lock_guard<std::mutex> g(m);
    if (set.load()) return;
    code = c;
    msg = s;
    set.store(true);
  }
  void rethrow() const {
    if (set.load()) throw Error(code, msg);
  }
};

// f(part, lo, hi) over `parts` contiguous slices of [0, n), on up to
// host_threads() threads (the caller takes slice 0).  Exceptions thrown by f
// are carried to the caller.
template <class F>
void par_for(size_t n, size_t min_per_part, F f) {
  if (n == 0) return;
  const size_t parts = std::max<size_t>(1, std::min(host_threads(), n / std::max<size_t>(1, min_per_part)));
  ParErr err;
  auto body = [&](size_t p) {
    const size_t lo = n * p / parts, hi = n * (p + 1) / parts;
    try {
      f(p, lo, hi);
    } catch (const Error &e) {
      err.raise(e.code, e.what());
    } catch (const std::exception &e) {
      err.raise(FH_EINVARIANT, e.what());
    }
  };
  if (parts == 1) {
    body(0);
  } else {
    std::vector<std::thread> ts;
    ts.reserve(parts - 1);
    for (size_t p = 1; p < parts; p++) ts.emplace_back(body, p);
    body(0);
    for (auto &t : ts) t.join();
  }
  err.rethrow();
}

// A ring of pinned host chunks for uploads and read-backs on one stream.
class PinnedRing {
 public:
  static constexpr size_t kChunk = size_t(32) << 20;
  static constexpr int kBufs = 4;
  PinnedRing() = default;
  PinnedRing(const PinnedRing &) = delete;
  PinnedRing &operator=(const PinnedRing &) = delete;
  ~PinnedRing() {
    for (int i = 0; i < kBufs; i++) {
      if (ev_[i]) {
        (void)hipEventSynchronize(ev_[i]);
        (void)hipEventDestroy(ev_[i]);
      }
      if (buf_[i]) (void)hipHostFree(buf_[i]);
    }
  }

  // count elements of T to device dst: fill(out, first, cnt) writes elements
  // [first, first + cnt) of the source into out (called on several threads
  // with disjoint ranges)
  template <class T, class F>
  void upload(T *ddst, size_t count, F fill, hipStream_t s) {
    const size_t per = kChunk / sizeof(T);
    for (size_t i0 = 0; i0 < count; i0 += per) {
      const size_t c = std::min(per, count - i0);
      T *h = reinterpret_cast<T *>(take(s));
      par_for(c, size_t(1) << 16, [&](size_t, size_t lo, size_t hi) { fill(h + lo, i0 + lo, hi - lo); });
      FH_HIP(hipMemcpyAsync(ddst + i0, h, c * sizeof(T), hipMemcpyHostToDevice, s));
      give(s);
    }
  }
  // a plain copy of host memory
  template <class T>
  void upload_copy(T *ddst, const T *src, size_t count, hipStream_t s) {
    upload(ddst, count, [&](T *out, size_t first, size_t cnt) {
      std::memcpy(out, src + first, cnt * sizeof(T));
    }, s);
  }
  // count elements of T from device src to host dst: the DMA of chunk i+1 is
  // in flight while host threads copy chunk i out of its pinned buffer
  template <class T>
  void download(T *hdst, const T *dsrc, size_t count, hipStream_t s) {
    const size_t per = kChunk / sizeof(T);
    std::vector<std::pair<size_t, int>> inflight;  // (first element, buffer)
    auto drain = [&](size_t keep) {
      while (inflight.size() > keep) {
        const auto [i0, k] = inflight.front();
        inflight.erase(inflight.begin());
        FH_HIP(hipEventSynchronize(ev_[k]));
        const size_t c = std::min(per, count - i0);
        const T *h = reinterpret_cast<const T *>(buf_[k]);
        par_for(c, size_t(1) << 16, [&](size_t, size_t lo, size_t hi) {
          std::memcpy(hdst + i0 + lo, h + lo, (hi - lo) * sizeof(T));
        });
        pending_[k] = false;
      }
    };
    for (size_t i0 = 0; i0 < count; i0 += per) {
      drain(kBufs - 1);
      const size_t c = std::min(per, count - i0);
      const int k = next_;
      alloc(k);
      FH_HIP(hipMemcpyAsync(buf_[k], dsrc + i0, c * sizeof(T), hipMemcpyDeviceToHost, s));
      FH_HIP(hipEventRecord(ev_[k], s));
      pending_[k] = true;
      next_ = (next_ + 1) % kBufs;
      inflight.push_back({i0, k});
    }
    drain(0);
  }

 private:
  void alloc(int k) {
    if (!buf_[k]) {
      FH_HIP(hipHostMalloc(reinterpret_cast<void **>(&buf_[k]), kChunk, hipHostMallocDefault));
      FH_HIP(hipEventCreateWithFlags(&ev_[k], hipEventDisableTiming));
    }
    if (pending_[k]) {
      FH_HIP(hipEventSynchronize(ev_[k]));
      pending_[k] = false;
    }
  }
  uint8_t *take(hipStream_t) {
    cur_ = next_;
    next_ = (next_ + 1) % kBufs;
    alloc(cur_);
    return buf_[cur_];
  }
  void give(hipStream_t s) {
    FH_HIP(hipEventRecord(ev_[cur_], s));
    pending_[cur_] = true;
  }
  uint8_t *buf_[kBufs] = {};
  hipEvent_t ev_[kBufs] = {};
  bool pending_[kBufs] = {};
  int next_ = 0, cur_ = 0;
};

}  // namespace fh
