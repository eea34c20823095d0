// aeclock_check.cpp -- host-only differential test of the executed clock
// (AEClock, csrc/dotindex.h) against a plain set of dots: single adds,
// bulk adds (add_all, one executor pass), frontier raises, exceptions near
// the frontier (bit rings) and far above it (hash set).  Built and run by
// tests/test_aeclock.py; prints "ok" or the first mismatch.
#include <cstdint>
#include <cstdio>
#include <random>
#include <set>
#include <vector>

#include "dotindex.h"

using fh::AEClock;
using fh::make_dot;

static uint64_t seq_of(uint64_t d) { return d & 0x00FFFFFFFFFFFFFFull; }

int main() {
  std::mt19937_64 rng(0xAEC10C);
  for (int trial = 0; trial < 100; trial++) {
    AEClock c;
    std::set<uint64_t> ref;
    // spans below and above the ring (4096 sequence numbers per process)
    const uint64_t span = trial % 3 == 0 ? 20000 : trial % 3 == 1 ? 300 : 5000;
    for (int i = 0; i < 3000; i++) {
      const uint32_t s = 1 + uint32_t(rng() % 3);
      const uint64_t d = make_dot(s, 1 + rng() % span);
      const int op = int(rng() % 40);
      if (op == 0) {
        // (the set already holds 1..frontier)
        const uint64_t f0 = c.frontier[s], seq = f0 + rng() % (trial % 2 ? 6000 : 50);
        c.raise_frontier(s, seq);
        for (uint64_t x = f0 + 1; x <= seq; x++) ref.insert(make_dot(s, x));
      } else if (op < 10) {
        std::vector<uint64_t> batch{d};
        for (int k = 0; k < 30; k++) batch.push_back(make_dot(1 + uint32_t(rng() % 3), 1 + rng() % span));
        const uint64_t v0 = c.version;
        bool fresh = false;
        for (uint64_t x : batch) fresh |= ref.insert(x).second;
        c.add_all(batch.data(), batch.size());
        if (fresh != (c.version != v0)) {
          printf("add_all version trial %d\n", trial);
          return 1;
        }
      } else {
        const bool a = c.add(d), b = ref.insert(d).second;
        if (a != b) {
          printf("add trial %d op %d\n", trial, i);
          return 1;
        }
      }
      const uint64_t p = make_dot(1 + uint32_t(rng() % 3), 1 + rng() % (span + 100));
      if (c.contains(p) != (ref.count(p) != 0)) {
        printf("contains trial %d op %d\n", trial, i);
        return 1;
      }
    }
    // the frontier is the contiguous prefix; exceptions are the rest, sorted
    for (uint32_t s = 1; s <= 3; s++) {
      for (uint64_t x = 1; x <= c.frontier[s]; x++)
        if (!ref.count(make_dot(s, x))) {
          printf("frontier hole trial %d\n", trial);
          return 1;
        }
      if (ref.count(make_dot(s, c.frontier[s] + 1))) {
        printf("frontier not advanced trial %d\n", trial);
        return 1;
      }
    }
    std::vector<uint64_t> got, want;
    c.exceptions(got);
    for (uint64_t d : ref)
      if (seq_of(d) > c.frontier[d >> 56]) want.push_back(d);
    if (got != want || c.exception_count() != want.size()) {
      printf("exceptions trial %d: %zu vs %zu\n", trial, got.size(), want.size());
      return 1;
    }
  }
  // large passes (add_all above AEClock::kBulk dots: the bitmap path), over
  // clocks that already hold ring and hash-set exceptions, with some dots
  // beyond the bitmap span (the per-dot path)
  for (int trial = 0; trial < 12; trial++) {
    AEClock c;
    std::set<uint64_t> ref;
    const uint64_t span = trial % 2 ? 300000 : 40000;
    for (int round = 0; round < 4; round++) {
      // a few single adds first: ring and far exceptions
      for (int i = 0; i < 200; i++) {
        const uint32_t s = 1 + uint32_t(rng() % 3);
        const uint64_t d = make_dot(s, c.frontier[s] + 1 + rng() % 9000);
        c.add(d);
        ref.insert(d);
      }
      std::vector<uint64_t> batch;
      const size_t nb = AEClock::kBulk + 1 + rng() % 30000;
      for (size_t k = 0; k < nb; k++) {
        const uint32_t s = 1 + uint32_t(rng() % 3);
        // mostly the next `span` sequence numbers (a whole pass), some repeats
        uint64_t q = c.frontier[s] + 1 + rng() % span;
        if (rng() % 1000 == 0) q = (uint64_t(1) << 29) + rng() % 1000;  // beyond the bitmap span
        batch.push_back(make_dot(s, q));
      }
      // and a contiguous run from each frontier, so the frontier moves
      for (uint32_t s = 1; s <= 3; s++)
        for (uint64_t q = c.frontier[s] + 1; q <= c.frontier[s] + span / 2; q++)
          batch.push_back(make_dot(s, q));
      const uint64_t v0 = c.version;
      bool fresh = false;
      for (uint64_t x : batch) fresh |= ref.insert(x).second;
      c.add_all(batch.data(), batch.size());
      if (fresh != (c.version != v0)) {
        printf("bulk version trial %d\n", trial);
        return 1;
      }
      for (int i = 0; i < 2000; i++) {
        const uint64_t p = make_dot(1 + uint32_t(rng() % 3), 1 + rng() % (c.frontier[1] + 2 * span));
        if (c.contains(p) != (ref.count(p) != 0)) {
          printf("bulk contains trial %d\n", trial);
          return 1;
        }
      }
      for (uint32_t s = 1; s <= 3; s++)
        if (ref.count(make_dot(s, c.frontier[s] + 1)) ||
            (c.frontier[s] && !ref.count(make_dot(s, c.frontier[s])))) {
          printf("bulk frontier trial %d\n", trial);
          return 1;
        }
      std::vector<uint64_t> got, want;
      c.exceptions(got);
      for (uint64_t d : ref)
        if (seq_of(d) > c.frontier[d >> 56]) want.push_back(d);
      if (got != want || c.exception_count() != want.size()) {
        printf("bulk exceptions trial %d: %zu vs %zu\n", trial, got.size(), want.size());
        return 1;
      }
    }
  }
  printf("ok\n");
  return 0;
}
