// workload.cpp -- seeded synthetic command streams (fh_workload_*).
//
// Semantics follow fantoch's client workload (fantoch/src/client/workload.rs,
// key_gen.rs) with a counter-based RNG so any range of the stream can be
// generated independently (and in parallel) and every consumer -- the GPU
// engine, the oracle, the CPU baseline -- sees the same commands:
//  - command i is submitted by process p = 1 + (i mod n) with sequence
//    i / n + 1 (DotGen::next_id, fantoch/src/id.rs:88-91; process ids 1..n,
//    fantoch/src/util.rs:115-122);
//  - keys are unique within a command (Workload::gen_unique_keys,
//    workload.rs:182-191), all ops are writes (read_only_percentage = 0,
//    workload.rs:50-51);
//  - Zipf{s, key_count}: ranks 1..key_count (zipf crate, key_gen.rs:102-108)
//    mapped to ids 0..key_count-1, sampled through an alias table;
//  - ConflictRate{r}: with probability r% the shared "CONFLICT" key (id 0),
//    otherwise the client's own key (key_gen.rs:87-99); clients submit
//    round-robin;
//  - ConflictPool{r, pool}: key 0 as ConflictRate, remaining keys uniform in
//    a pool of hot keys (BASELINE config C3; the reference rejects
//    ConflictRate 100% with >1 key, workload.rs:43-48);
//  - replica views: member j of command i's fast quorum is process
//    1 + ((p-1+j) mod n) (the coordinator plus the next fq-1 processes,
//    standing in for BaseProcess::fast_quorum's distance order,
//    fantoch/src/protocol/base.rs:82-87,153-157); it sees the command at time
//    (i+d)*W + d with d = 0 for the coordinator and d uniform in [0, W)
//    otherwise (the analogue of the simulator's reorder_messages,
//    fantoch/src/sim/runner.rs:513-518).
#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "fh_common.h"

namespace fh {
namespace {

inline uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
inline uint64_t rnd(uint64_t seed, uint64_t i, uint64_t tag) {
  return splitmix(splitmix(seed ^ (i * 0xD6E8FEB86659FD93ull)) + tag * 0xA0761D6478BD642Full);
}

struct Alias {
  std::vector<uint32_t> prob;   // 32-bit fixed-point acceptance threshold
  std::vector<uint32_t> alias;
};

const Alias &zipf_alias(double s, uint64_t k) {
  static std::mutex mu;
  static std::map<std::pair<double, uint64_t>, Alias> cache;
  std::lock_guard<std::mutex> g(mu);
  auto key = std::make_pair(s, k);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  std::vector<double> w(k);
  double sum = 0;
  for (uint64_t r = 0; r < k; r++) {
    w[r] = std::pow(double(r + 1), -s);
    sum += w[r];
  }
  // Vose's alias method
  std::vector<double> p(k);
  std::vector<uint32_t> small, large;
  for (uint64_t r = 0; r < k; r++) {
    p[r] = w[r] / sum * double(k);
    (p[r] < 1.0 ? small : large).push_back(uint32_t(r));
  }
  Alias a;
  a.prob.assign(k, 0xFFFFFFFFu);
  a.alias.resize(k);
  for (uint64_t r = 0; r < k; r++) a.alias[r] = uint32_t(r);
  while (!small.empty() && !large.empty()) {
    uint32_t l = small.back();
    small.pop_back();
    uint32_t g2 = large.back();
    large.pop_back();
    a.prob[l] = uint32_t(std::min(4294967295.0, std::floor(p[l] * 4294967296.0)));
    a.alias[l] = g2;
    p[g2] = (p[g2] + p[l]) - 1.0;
    (p[g2] < 1.0 ? small : large).push_back(g2);
  }
  return cache.emplace(key, std::move(a)).first->second;
}

uint64_t key_space_of(const fh_workload &w) {
  switch (w.kind) {
    case 0:
      return w.key_count;
    case 1:
      return 1 + uint64_t(w.clients);
    case 2:
      return 1 + uint64_t(w.pool_size) + uint64_t(w.clients);
    default:
      return 0;
  }
}

void validate(const fh_workload &w) {
  FH_CHECK(w.n >= 1 && w.n <= 255, FH_EINVAL, "workload: n must be in [1, 255]");
  FH_CHECK(w.keys_per_cmd >= 1 && w.keys_per_cmd <= 8, FH_EINVAL,
           "workload: keys_per_cmd must be in [1, 8]");
  FH_CHECK(w.kind <= 2, FH_EINVAL, "workload: unknown key generator");
  if (w.kind == 0) {
    FH_CHECK(w.key_count >= w.keys_per_cmd && w.key_count < (uint64_t(1) << 31), FH_EINVAL,
             "workload: zipf key_count out of range");
    FH_CHECK(w.zipf_s > 0, FH_EINVAL, "workload: zipf coefficient must be > 0");
  } else {
    FH_CHECK(w.conflict_rate <= 100 && w.clients >= 1, FH_EINVAL,
             "workload: bad conflict rate / clients");
    if (w.kind == 1) {
      // workload.rs:39-48
      FH_CHECK(!(w.conflict_rate == 100 && w.keys_per_cmd > 1), FH_EINVAL,
               "invalid workload; can't generate more than one key when the conflict_rate is 100");
      FH_CHECK(w.keys_per_cmd <= 2, FH_EINVAL,
               "invalid workload; can't generate more than two keys with the conflict_rate key "
               "generator");
    } else {
      FH_CHECK(w.pool_size + 1 >= w.keys_per_cmd, FH_EINVAL, "workload: pool too small");
    }
  }
  FH_CHECK(w.views <= w.n && w.views <= 16, FH_EINVAL, "workload: views must be <= n");
}

inline uint64_t gen_key(const fh_workload &w, const Alias *za, uint64_t i, uint32_t slot,
                        uint32_t attempt) {
  const uint64_t r = rnd(w.seed, i, 1 + slot * 64 + attempt);
  switch (w.kind) {
    case 0: {
      const uint64_t bucket = ((r >> 32) * w.key_count) >> 32;
      return (uint32_t(r) < za->prob[bucket]) ? bucket : za->alias[bucket];
    }
    case 1: {
      const uint64_t client = i % w.clients;
      return (r % 100) < w.conflict_rate ? 0 : 1 + client;
    }
    default: {
      const uint64_t client = i % w.clients;
      if (slot == 0) return (r % 100) < w.conflict_rate ? 0 : 1 + w.pool_size + client;
      return 1 + (r % w.pool_size);
    }
  }
}

void gen_range(const fh_workload &w, const Alias *za, uint64_t first, size_t lo, size_t hi,
               uint64_t *dot, uint64_t *key_id, uint8_t *fq_proc, uint64_t *fq_time) {
  const uint32_t k = w.keys_per_cmd;
  const uint64_t W = w.window ? w.window : 1;
  for (size_t c = lo; c < hi; c++) {
    const uint64_t i = first + c;
    const uint32_t p = 1 + uint32_t(i % w.n);
    if (dot) dot[c] = make_dot(p, i / w.n + 1);
    if (key_id) {
      uint64_t *ks = key_id + c * k;
      for (uint32_t s = 0; s < k; s++) {
        uint64_t key = 0;
        for (uint32_t a = 0;; a++) {
          key = gen_key(w, za, i, s, a);
          bool dup = false;
          for (uint32_t t = 0; t < s; t++) dup |= ks[t] == key;
          if (!dup) break;
        }
        ks[s] = key;
      }
    }
    if (w.views && (fq_proc || fq_time)) {
      for (uint32_t j = 0; j < w.views; j++) {
        const uint64_t d = j == 0 ? 0 : rnd(w.seed, i, 1000 + j) % W;
        if (fq_proc) fq_proc[c * w.views + j] = uint8_t(1 + (p - 1 + j) % w.n);
        if (fq_time) fq_time[c * w.views + j] = (i + d) * W + d;
      }
    }
  }
}

// Replica `r` (process r + 1) sees member j of command i with
// j = (r - (p_i - 1)) mod n when j < views, at time (i + d)·W + d (gen_range).
// Its arrival order is (T = i + d, d) ascending: a counting sort over the
// bucket T, filled in decreasing i so that within a bucket d ascends.
uint32_t member_delay(const fh_workload &w, uint64_t i, uint32_t j) {
  const uint64_t W = w.window ? w.window : 1;
  return j == 0 ? 0u : uint32_t(rnd(w.seed, i, 1000 + j) % W);
}

// `keep` (may be null): batch-local index of each command in the output, or
// ~0u for commands left out (a key shard of the stream)
void gen_log(const fh_workload &w, uint64_t first, size_t count, uint32_t r, uint32_t *out,
             size_t cap, const uint32_t *keep = nullptr) {
  const uint64_t W = w.window ? w.window : 1;
  std::vector<uint32_t> cnt(count + W + 1, 0);
  auto member = [&](size_t c, uint32_t *j) {
    if (keep && keep[c] == ~0u) return false;
    const uint64_t i = first + c;
    const uint32_t p = uint32_t(i % w.n);  // p_i - 1
    *j = (r + w.n - p) % w.n;
    return *j < w.views;
  };
  for (size_t c = 0; c < count; c++) {
    uint32_t j;
    if (member(c, &j)) cnt[c + member_delay(w, first + c, j) + 1]++;
  }
  for (size_t t = 1; t < cnt.size(); t++) cnt[t] += cnt[t - 1];
  FH_CHECK(cnt.back() <= cap, FH_EINVARIANT, "log capacity");
  for (size_t c = count; c-- > 0;) {
    uint32_t j;
    if (member(c, &j)) out[cnt[c + member_delay(w, first + c, j)]++] = keep ? keep[c] : uint32_t(c);
  }
}

template <class F>
void parallel_chunks(size_t count, F f) {
  size_t threads = std::min<size_t>(16, std::max<size_t>(1, count / (1 << 16)));
  unsigned hc = std::thread::hardware_concurrency();
  if (hc) threads = std::min<size_t>(threads, hc);
  std::vector<std::thread> ts;
  const size_t chunk = (count + threads - 1) / threads;
  for (size_t t = 0; t < threads; t++) {
    const size_t lo = t * chunk, hi = std::min(count, lo + chunk);
    if (lo >= hi) break;
    ts.emplace_back(f, t, lo, hi);
  }
  for (auto &t : ts) t.join();
}

}  // namespace
}  // namespace fh

extern "C" {

fh_status fh_workload_generate_shard(const fh_workload *w, uint64_t first, size_t count,
                                     uint32_t nshards, uint32_t shard, size_t *n_out,
                                     uint64_t *dot, uint64_t *key_id, uint64_t *log_off,
                                     uint32_t *log_cmd) {
  FH_API_BEGIN
  FH_CHECK(w && n_out, FH_EINVAL, "null argument");
  fh::validate(*w);
  FH_CHECK(nshards >= 1 && shard < nshards, FH_EINVAL, "workload: shard must be < nshards");
  FH_CHECK(count < (size_t(1) << 32), FH_EINVAL, "workload: count must be < 2^32");
  const fh::Alias *za = w->kind == 0 ? &fh::zipf_alias(w->zipf_s, w->key_count) : nullptr;
  const uint32_t k = w->keys_per_cmd;
  // pass 1: membership (owner of the command's first key) and per-chunk counts
  std::vector<uint32_t> keep(count);
  std::vector<size_t> per(17, 0);
  fh::parallel_chunks(count, [&](size_t t, size_t lo, size_t hi) {
    std::vector<uint64_t> ks(k);
    size_t m = 0;
    for (size_t c = lo; c < hi; c++) {
      fh::gen_range(*w, za, first + c, 0, 1, nullptr, ks.data(), nullptr, nullptr);
      const bool mine = ks[0] % nshards == shard;
      keep[c] = mine ? 1u : ~0u;
      m += mine;
    }
    per[t + 1] = m;
  });
  for (size_t t = 1; t < per.size(); t++) per[t] += per[t - 1];
  *n_out = per.back();
  if (!dot && !key_id && !log_off && !log_cmd) return FH_OK;  // size query
  FH_CHECK(dot && key_id, FH_EINVAL, "null argument");
  // pass 2: the shard's commands, global dots and keys, in stream order
  fh::parallel_chunks(count, [&](size_t t, size_t lo, size_t hi) {
    size_t o = per[t];
    for (size_t c = lo; c < hi; c++) {
      if (keep[c] == ~0u) continue;
      keep[c] = uint32_t(o);
      fh::gen_range(*w, za, first + c, 0, 1, dot + o, key_id + o * k, nullptr, nullptr);
      o++;
    }
  });
  if (!log_off && !log_cmd) return FH_OK;
  FH_CHECK(log_off && log_cmd && w->views >= 1, FH_EINVAL, "logs need views and both arrays");
  // replicas' logs restricted to the shard's commands
  std::vector<size_t> lp(w->n, 0);
  for (size_t c = 0; c < count; c++) {
    if (keep[c] == ~0u) continue;
    const uint32_t p = uint32_t((first + c) % w->n);
    for (uint32_t j = 0; j < w->views; j++) lp[(p + j) % w->n]++;
  }
  log_off[0] = 0;
  for (uint32_t r = 0; r < w->n; r++) log_off[r + 1] = log_off[r] + lp[r];
  std::vector<std::thread> ts;
  std::vector<std::string> errs(w->n);
  for (uint32_t r = 0; r < w->n; r++)
    ts.emplace_back([&, r] {
      try {
        fh::gen_log(*w, first, count, r, log_cmd + log_off[r], lp[r], keep.data());
      } catch (const std::exception &e) {
        errs[r] = e.what();
      }
    });
  for (auto &t : ts) t.join();
  for (auto &e : errs) FH_CHECK(e.empty(), FH_EINVARIANT, e);
  FH_API_END
}

fh_status fh_workload_generate_logs(const fh_workload *w, uint64_t first, size_t count,
                                    uint64_t *log_off, uint32_t *log_cmd) {
  FH_API_BEGIN
  FH_CHECK(w && log_off && log_cmd, FH_EINVAL, "null argument");
  fh::validate(*w);
  FH_CHECK(w->views >= 1, FH_EINVAL, "workload: logs need replica views (views >= 1)");
  FH_CHECK(count < (size_t(1) << 32), FH_EINVAL, "workload: count must be < 2^32");
  // replica r holds exactly the commands whose fast quorum includes r + 1
  std::vector<size_t> per(w->n, 0);
  for (uint32_t r = 0; r < w->n; r++) {
    // commands i with (r - (i mod n)) mod n < views
    for (uint32_t j = 0; j < w->views; j++) {
      const uint32_t p = (r + w->n - j) % w->n;  // p_i - 1 for member j
      // count of i in [first, first + count) with i mod n == p
      const uint64_t lo = first, hi = first + count;
      auto upto = [&](uint64_t x) { return x / w->n + (x % w->n > p ? 1 : 0); };
      per[r] += size_t(upto(hi) - upto(lo));
    }
  }
  log_off[0] = 0;
  for (uint32_t r = 0; r < w->n; r++) log_off[r + 1] = log_off[r] + per[r];
  std::vector<std::thread> ts;
  std::vector<std::string> errs(w->n);
  for (uint32_t r = 0; r < w->n; r++)
    ts.emplace_back([&, r] {
      try {
        fh::gen_log(*w, first, count, r, log_cmd + log_off[r], per[r]);
      } catch (const std::exception &e) {
        errs[r] = e.what();
      }
    });
  for (auto &t : ts) t.join();
  for (auto &e : errs) FH_CHECK(e.empty(), FH_EINVARIANT, e);
  FH_API_END
}

uint64_t fh_workload_key_space(const fh_workload *w) { return w ? fh::key_space_of(*w) : 0; }

fh_status fh_workload_generate(const fh_workload *w, uint64_t first, size_t count, uint64_t *dot,
                               uint64_t *key_id, uint8_t *fq_proc, uint64_t *fq_time) {
  FH_API_BEGIN
  FH_CHECK(w, FH_EINVAL, "null workload");
  fh::validate(*w);
  const fh::Alias *za = w->kind == 0 ? &fh::zipf_alias(w->zipf_s, w->key_count) : nullptr;
  size_t threads = std::min<size_t>(16, std::max<size_t>(1, count / (1 << 16)));
  unsigned hc = std::thread::hardware_concurrency();
  if (hc) threads = std::min<size_t>(threads, hc);
  if (threads <= 1) {
    fh::gen_range(*w, za, first, 0, count, dot, key_id, fq_proc, fq_time);
  } else {
    std::vector<std::thread> ts;
    const size_t chunk = (count + threads - 1) / threads;
    for (size_t t = 0; t < threads; t++) {
      const size_t lo = t * chunk, hi = std::min(count, lo + chunk);
      if (lo >= hi) break;
      ts.emplace_back(fh::gen_range, std::cref(*w), za, first, lo, hi, dot, key_id, fq_proc,
                      fq_time);
    }
    for (auto &t : ts) t.join();
  }
  FH_API_END
}

}  // extern "C"
