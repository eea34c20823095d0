// dotindex.h -- dots on the device: the executed set and dot -> vertex id.
//
// Shared by the executors (graph_api.hip: GraphExecutor, pred.hip: Caesar's
// PredecessorsExecutor).  An AEClock<ProcessId> (threshold crate, used at
// executor/graph/mod.rs:50 and executor/pred/mod.rs:29-30) is a contiguous
// frontier per process plus exceptions, kept on the host and mirrored to the
// device per batch (frontier[256] + sorted exception dots).  Vertex dots
// resolve through a device sort of the vertex dots and binary search.
#pragma once

#include <unordered_set>

#include "fh_common.h"

namespace fh {

__device__ __forceinline__ bool executed_dev(uint64_t d, const uint64_t *__restrict__ frontier,
                                             const uint64_t *__restrict__ exc, uint32_t nexc) {
  if ((d & 0x00FFFFFFFFFFFFFFull) <= frontier[d >> 56]) return true;
  uint32_t lo = 0, hi = nexc;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (exc[mid] < d)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < nexc && exc[lo] == d;
}

// vertex id of dot d (sd = sorted vertex dots, sv = their ids), -1 if absent
__device__ __forceinline__ int64_t find_vid(uint64_t d, const uint64_t *__restrict__ sd,
                                            const uint32_t *__restrict__ sv, uint32_t V) {
  uint32_t lo = 0, hi = V;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sd[mid] < d)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < V && sd[lo] == d) ? int64_t(sv[lo]) : -1;
}

// *err |= 1 if two sorted vertex dots are equal (an already indexed dot)
__global__ void k_dup_check(uint32_t V, const uint64_t *__restrict__ sd, uint32_t *err);

// AEClock<ProcessId>: per-process contiguous frontier + exception set.
struct AEClock {
  uint64_t frontier[256] = {0};
  std::unordered_set<uint64_t> exc;
  uint64_t version = 0;  // bumped on every change (device mirrors re-upload)
  bool contains(uint64_t d) const {
    return (d & 0x00FFFFFFFFFFFFFFull) <= frontier[d >> 56] || exc.count(d);
  }
  // AEClock::add: true if d was not in the set
  bool add(uint64_t d) {
    const uint32_t s = uint32_t(d >> 56);
    const uint64_t q = d & 0x00FFFFFFFFFFFFFFull;
    if (q <= frontier[s]) return false;
    version++;
    if (q == frontier[s] + 1) {
      frontier[s] = q;
      while (!exc.empty()) {
        auto it = exc.find(make_dot(s, frontier[s] + 1));
        if (it == exc.end()) break;
        exc.erase(it);
        frontier[s]++;
      }
      return true;
    }
    if (exc.insert(d).second) return true;
    version--;  // already an exception: unchanged
    return false;
  }
};

}  // namespace fh
