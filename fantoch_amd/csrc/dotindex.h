// dotindex.h -- dots on the device: the executed set and dot -> vertex id.
//
// Shared by the executors (graph_api.hip: GraphExecutor, pred.hip: Caesar's
// PredecessorsExecutor).  An AEClock<ProcessId> (threshold crate, used at
// executor/graph/mod.rs:50 and executor/pred/mod.rs:29-30) is a contiguous
// frontier per process plus exceptions, kept on the host and mirrored to the
// device per batch (frontier[256] + sorted exception dots).  Vertex dots
// resolve through a device sort of the vertex dots and binary search.
#pragma once

#include <algorithm>
#include <memory>
#include <unordered_set>
#include <vector>

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
// Exceptions within kWin sequence numbers above a process's frontier are
// bits of a per-process ring (bit q mod kWin); farther ones go to a hash
// set.  Executions arrive almost in sequence order, so an add is a few bit
// operations (the hash set alone cost 36-87 ns per add on locally reordered
// C4 streams: most of a 1,000-command batch's host time).
struct AEClock {
  static constexpr uint64_t kWin = 4096;  // ring bits per process
  uint64_t frontier[256] = {0};
  uint64_t version = 0;  // bumped on every change (device mirrors re-upload)

  bool contains(uint64_t d) const {
    const uint32_t s = uint32_t(d >> 56);
    const uint64_t q = d & 0x00FFFFFFFFFFFFFFull;
    if (q <= frontier[s]) return true;
    if (q - frontier[s] <= kWin && nbits[s] && test(s, q)) return true;
    return !far.empty() && far.count(d) != 0;
  }
  // AEClock::add: true if d was not in the set
  bool add(uint64_t d) {
    const uint32_t s = uint32_t(d >> 56);
    const uint64_t q = d & 0x00FFFFFFFFFFFFFFull;
    if (q <= frontier[s]) return false;
    if (q - frontier[s] <= kWin) {
      if (nbits[s] && test(s, q)) return false;
      if (!far.empty() && far.count(d)) return false;  // went far before the frontier moved
      version++;
      if (q == frontier[s] + 1) {
        frontier[s] = q;
        advance(s);
      } else {
        words(s)[(q % kWin) >> 6] |= uint64_t(1) << (q & 63);
        nbits[s]++;
      }
      return true;
    }
    if (!far.insert(d).second) return false;
    version++;
    return true;
  }
  // add for a list of dots (one executor pass's executed dots): bits first,
  // then each touched process's frontier advances once, by whole runs
  void add_all(const uint64_t *dots, size_t n) {
    if (n > kBulk) {
      add_bulk(dots, n);
      return;
    }
    bool changed = false;
    uint64_t touched[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < n; i++) {
      const uint64_t d = dots[i];
      const uint32_t s = uint32_t(d >> 56);
      const uint64_t q = d & 0x00FFFFFFFFFFFFFFull;
      if (q <= frontier[s]) continue;
      if (q - frontier[s] <= kWin) {
        uint64_t &w = words(s)[(q % kWin) >> 6];
        const uint64_t b = uint64_t(1) << (q & 63);
        if (w & b) continue;
        if (!far.empty() && far.count(d)) continue;
        w |= b;
        nbits[s]++;
        touched[s >> 6] |= uint64_t(1) << (s & 63);
        changed = true;
      } else if (far.insert(d).second) {
        touched[s >> 6] |= uint64_t(1) << (s & 63);
        changed = true;
      }
    }
    for (uint32_t g = 0; g < 4; g++)
      for (uint64_t m = touched[g]; m; m &= m - 1) advance(g * 64 + uint32_t(__builtin_ctzll(m)));
    if (changed) version++;
  }
  // add_all for a large pass (a 1M-command batch spans ~200K sequence numbers
  // per process, most of them beyond the ring while the frontier has not
  // moved yet: the hash set took ~55 ns per dot, 55 ms per pass).  Per
  // process, a dense bitmap over (frontier, the batch's largest sequence]:
  // the batch's dots and the old exceptions in that range are set there, the
  // frontier advances over the leading ones, and the remaining bits go back
  // to the ring (or the hash set beyond it).  O(n + span / 64).
  static constexpr size_t kBulk = size_t(1) << 14;
  static constexpr uint64_t kMaxSpan = uint64_t(1) << 28;  // bits per process
  void add_bulk(const uint64_t *dots, size_t n) {
    uint64_t hi[256] = {0};
    for (size_t i = 0; i < n; i++) {
      const uint32_t s = uint32_t(dots[i] >> 56);
      const uint64_t q = dots[i] & 0x00FFFFFFFFFFFFFFull;
      if (q > frontier[s] && q > hi[s]) hi[s] = q;
    }
    bool dense[256] = {false};
    for (uint32_t s = 0; s < 256; s++)
      if (hi[s] && hi[s] - frontier[s] <= kMaxSpan) {
        dense[s] = true;
        bulk[s].assign((hi[s] - frontier[s] + 63) / 64, 0);
      }
    bool changed = false;
    for (size_t i = 0; i < n; i++) {
      const uint32_t s = uint32_t(dots[i] >> 56);
      const uint64_t q = dots[i] & 0x00FFFFFFFFFFFFFFull;
      if (q <= frontier[s]) continue;
      if (!dense[s]) {
        changed |= add(dots[i]);
        continue;
      }
      const uint64_t b = q - frontier[s] - 1;
      bulk[s][b >> 6] |= uint64_t(1) << (b & 63);
    }
    for (uint32_t s = 0; s < 256; s++) {
      if (!dense[s]) continue;
      std::vector<uint64_t> &bm = bulk[s];
      const uint64_t f = frontier[s], h = hi[s];
      uint64_t batch_bits = 0, overlap = 0;
      for (uint64_t w : bm) batch_bits += uint64_t(__builtin_popcountll(w));
      // the old exceptions in (f, h] join the bitmap
      if (nbits[s]) {
        uint64_t *w = ring[s].get();
        for (uint64_t x = 0; x < kWin / 64; x++)
          for (uint64_t m = w[x]; m; m &= m - 1) {
            const uint64_t i = x * 64 + uint64_t(__builtin_ctzll(m));
            const uint64_t q = f + 1 + ((i - (f + 1)) & (kWin - 1));
            if (q > h) continue;
            const uint64_t b = q - f - 1;
            overlap += (bm[b >> 6] >> (b & 63)) & 1;
            bm[b >> 6] |= uint64_t(1) << (b & 63);
            w[x] &= ~(uint64_t(1) << (i & 63));
            nbits[s]--;
          }
      }
      if (!far.empty())
        for (auto it = far.begin(); it != far.end();) {
          const uint64_t q = *it & 0x00FFFFFFFFFFFFFFull;
          if ((*it >> 56) == s && q <= h) {
            const uint64_t b = q - f - 1;
            overlap += (bm[b >> 6] >> (b & 63)) & 1;
            bm[b >> 6] |= uint64_t(1) << (b & 63);
            it = far.erase(it);
          } else {
            ++it;
          }
        }
      changed |= batch_bits > overlap;
      // the frontier over the leading ones
      uint64_t lead = 0, x = 0;
      while (x < bm.size() && bm[x] == ~uint64_t(0)) {
        lead += 64;
        x++;
      }
      if (x < bm.size()) lead += uint64_t(__builtin_ctzll(~bm[x]));
      lead = std::min(lead, h - f);
      const uint64_t fn = f + lead;
      // the rest back to the ring (slot q mod kWin, valid for q - fn <= kWin)
      // or the hash set
      for (uint64_t y = lead >> 6; y < bm.size(); y++)
        for (uint64_t m = bm[y]; m; m &= m - 1) {
          const uint64_t b = y * 64 + uint64_t(__builtin_ctzll(m));
          if (b < lead) continue;
          const uint64_t q = f + 1 + b;
          if (q - fn <= kWin) {
            words(s)[(q % kWin) >> 6] |= uint64_t(1) << (q & 63);
            nbits[s]++;
          } else {
            far.insert(make_dot(s, q));
          }
        }
      frontier[s] = fn;
      advance(s);
      bm.clear();
    }
    if (changed) version++;
  }
  // Raise s's frontier to seq (>= the current one): exceptions at or below it
  // go, and exceptions right above it fold in
  void raise_frontier(uint32_t s, uint64_t seq) {
    if (seq <= frontier[s]) return;
    // ring bits at or below seq go; the ones above it keep their slots (the
    // new window (seq, seq + kWin] covers them)
    const uint64_t hi = std::min(seq, frontier[s] + kWin);
    for (uint64_t q = frontier[s] + 1; q <= hi && nbits[s]; q++) clear(s, q);
    for (auto it = far.begin(); it != far.end();) {
      if ((*it >> 56) == s && (*it & 0x00FFFFFFFFFFFFFFull) <= seq)
        it = far.erase(it);
      else
        ++it;
    }
    frontier[s] = seq;
    advance(s);
    version++;
  }
  // every exception dot, sorted
  void exceptions(std::vector<uint64_t> &out) const {
    out.clear();
    for (uint32_t s = 0; s < 256; s++) {
      if (!nbits[s]) continue;
      // the ring's slot i holds q = the one in (frontier, frontier + kWin]
      // with q mod kWin = i
      const uint64_t *w = ring[s].get();
      const uint64_t f = frontier[s];
      for (uint64_t x = 0; x < kWin / 64; x++)
        for (uint64_t m = w[x]; m; m &= m - 1) {
          const uint64_t i = x * 64 + uint64_t(__builtin_ctzll(m));
          out.push_back(make_dot(s, f + 1 + ((i - (f + 1)) & (kWin - 1))));
        }
    }
    out.insert(out.end(), far.begin(), far.end());
    std::sort(out.begin(), out.end());
  }
  size_t exception_count() const {
    size_t c = far.size();
    for (uint32_t s = 0; s < 256; s++) c += nbits[s];
    return c;
  }

 private:
  std::unique_ptr<uint64_t[]> ring[256];
  uint32_t nbits[256] = {0};
  std::unordered_set<uint64_t> far;
  std::vector<uint64_t> bulk[256];  // add_bulk's per-process bitmaps
  uint64_t *words(uint32_t s) {
    if (!ring[s]) ring[s].reset(new uint64_t[kWin / 64]());
    return ring[s].get();
  }
  bool test(uint32_t s, uint64_t q) const { return (ring[s][(q % kWin) >> 6] >> (q & 63)) & 1; }
  void clear(uint32_t s, uint64_t q) {
    uint64_t &w = ring[s][(q % kWin) >> 6];
    const uint64_t b = uint64_t(1) << (q & 63);
    if (w & b) {
      w &= ~b;
      nbits[s]--;
    }
  }
  // fold the exceptions right above the frontier into it
  void advance(uint32_t s) {
    for (;;) {
      const uint64_t q = frontier[s] + 1;
      if (nbits[s]) {
        // the run of set bits from q's slot to the end of its word
        uint64_t &w = ring[s][(q % kWin) >> 6];
        const uint64_t x = ~(w >> (q & 63));  // ones above the word's top: len <= 64 - (q & 63)
        const uint64_t len = x ? uint64_t(__builtin_ctzll(x)) : 64;
        if (len) {
          const uint64_t mask = (len == 64 ? ~uint64_t(0) : ((uint64_t(1) << len) - 1)) << (q & 63);
          w &= ~mask;
          nbits[s] -= uint32_t(len);
          frontier[s] += len;
          continue;
        }
      }
      if (!far.empty()) {
        auto it = far.find(make_dot(s, q));
        if (it != far.end()) {
          far.erase(it);
          frontier[s] = q;
          continue;
        }
      }
      return;
    }
  }
};

}  // namespace fh
