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
// Partial replication (shards >= 2, BASELINE config C5): shard h holds the
// processes n·h + 1 ... n·h + n (fantoch/src/util.rs:115-122) and the keys
// with key % shards == h.
//  - the command's target shard t is the shard of its first key (the client
//    submits to it, fantoch/src/client/workload.rs:172-176); its coordinator
//    there is process n·t + 1 + (i mod n), and the dot is that process's next
//    id (DotGen::next_id, id.rs:88-91), so Dot::target_shard (id.rs:59-61)
//    is t;
//  - every shard h the command touches runs its own collect (the forwarded
//    submit, protocol/partial.rs:8-34, then atlas.rs:214-328): its
//    coordinator is n·h + 1 + (i mod n) (closest_process, the same local
//    index) and its fast quorum the next fq-1 processes of shard h, each with
//    a delay seeded by (i, h, j) -- shards see the command in independent
//    orders;
//  - a command's committed deps are the union of its shards' reports
//    (MShardCommit, atlas.rs:559-639).
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
  FH_CHECK(w.shards <= 64 && uint64_t(w.n) * std::max(1u, w.shards) <= 255, FH_EINVAL,
           "workload: shards <= 64 and n * shards <= 255 (ProcessId is a u8)");
}

inline uint32_t nshards(const fh_workload &w) { return w.shards > 1 ? w.shards : 1; }

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

// the command's keys (unique within the command)
inline void gen_keys(const fh_workload &w, const Alias *za, uint64_t i, uint64_t *ks) {
  for (uint32_t s = 0; s < w.keys_per_cmd; s++) {
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

// Delay of view j of command i in shard h (0 for the shard's coordinator);
// h = 0 is the unsharded stream's seeding.
inline uint32_t member_delay(const fh_workload &w, uint64_t i, uint32_t h, uint32_t j) {
  const uint64_t W = w.window ? w.window : 1;
  return j == 0 ? 0u : uint32_t(rnd(w.seed, i, 1000 + 64 * uint64_t(h) + j) % W);
}

// Partial replication: the dot of command i is the next id of its target
// shard's coordinator, so sequences count the earlier commands with the same
// (target shard, coordinator index).  seq[n·shards] holds those counts for the
// commands before `first + lo` and is advanced over the range.
void gen_range(const fh_workload &w, const Alias *za, uint64_t first, size_t lo, size_t hi,
               uint64_t *dot, uint64_t *key_id, uint8_t *fq_proc, uint64_t *fq_time,
               uint64_t *seq) {
  const uint32_t k = w.keys_per_cmd, S = nshards(w);
  const uint64_t W = w.window ? w.window : 1;
  uint64_t ks[8];
  for (size_t c = lo; c < hi; c++) {
    const uint64_t i = first + c;
    const uint32_t l = uint32_t(i % w.n);
    gen_keys(w, za, i, ks);
    if (key_id)
      for (uint32_t s = 0; s < k; s++) key_id[c * k + s] = ks[s];
    if (S == 1) {
      if (dot) dot[c] = make_dot(1 + l, i / w.n + 1);
      if (w.views && (fq_proc || fq_time)) {
        for (uint32_t j = 0; j < w.views; j++) {
          const uint64_t d = member_delay(w, i, 0, j);
          if (fq_proc) fq_proc[c * w.views + j] = uint8_t(1 + (l + j) % w.n);
          if (fq_time) fq_time[c * w.views + j] = (i + d) * W + d;
        }
      }
      continue;
    }
    const uint32_t t = uint32_t(ks[0] % S);
    const uint64_t q = ++seq[t * w.n + l];
    if (dot) dot[c] = make_dot(w.n * t + 1 + l, q);
    // views per key slot: those of the slot's shard, [(c·k + s)·views + j]
    if (w.views && (fq_proc || fq_time)) {
      for (uint32_t s = 0; s < k; s++) {
        const uint32_t h = uint32_t(ks[s] % S);
        for (uint32_t j = 0; j < w.views; j++) {
          const uint64_t d = member_delay(w, i, h, j);
          const size_t x = (c * k + s) * w.views + j;
          if (fq_proc) fq_proc[x] = uint8_t(w.n * h + 1 + (l + j) % w.n);
          if (fq_time) fq_time[x] = (i + d) * W + d;
        }
      }
    }
  }
}

// Per-(target shard, coordinator index) command counts over [lo, hi) of the
// stream (partial replication's dot sequences).
void seq_counts(const fh_workload &w, const Alias *za, uint64_t lo, uint64_t hi, uint64_t *cnt) {
  const uint32_t S = nshards(w);
  uint64_t ks[8];
  for (uint64_t i = lo; i < hi; i++) {
    gen_keys(w, za, i, ks);
    cnt[uint32_t(ks[0] % S) * w.n + uint32_t(i % w.n)]++;
  }
}

// Replica `r` (process r + 1) sees member j of command i with
// j = (r - (p_i - 1)) mod n when j < views, at time (i + d)·W + d (gen_range).
// Its arrival order is (T = i + d, d) ascending: a counting sort over the
// bucket T, filled in decreasing i so that within a bucket d ascends.

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
    if (member(c, &j)) cnt[c + member_delay(w, first + c, 0, j) + 1]++;
  }
  for (size_t t = 1; t < cnt.size(); t++) cnt[t] += cnt[t - 1];
  FH_CHECK(cnt.back() <= cap, FH_EINVARIANT, "log capacity");
  for (size_t c = count; c-- > 0;) {
    uint32_t j;
    if (member(c, &j)) out[cnt[c + member_delay(w, first + c, 0, j)]++] = keep ? keep[c] : uint32_t(c);
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

// [0, count) in up to 16 chunks of >= 2^16 commands (generation threads)
std::vector<size_t> chunk_bounds(size_t count) {
  size_t threads = std::min<size_t>(16, std::max<size_t>(1, count / (1 << 16)));
  unsigned hc = std::thread::hardware_concurrency();
  if (hc) threads = std::min<size_t>(threads, hc);
  std::vector<size_t> b(threads + 1);
  for (size_t t = 0; t <= threads; t++) b[t] = count * t / threads;
  return b;
}

// Partial replication: per generation chunk, the (target shard, coordinator)
// counts of every command before it -- the sequences its dots continue from.
std::vector<std::vector<uint64_t>> seq_bases(const fh_workload &w, const Alias *za,
                                             uint64_t first, const std::vector<size_t> &bounds) {
  const size_t T = bounds.size() - 1, C = size_t(w.n) * nshards(w);
  // commands before `first`, then each chunk's own counts
  const std::vector<size_t> pre = chunk_bounds(first);
  const size_t P = pre.size() - 1;
  std::vector<std::vector<uint64_t>> cnt(P + T, std::vector<uint64_t>(C, 0));
  std::vector<std::thread> ts;
  for (size_t t = 0; t < P; t++)
    ts.emplace_back([&, t] { seq_counts(w, za, pre[t], pre[t + 1], cnt[t].data()); });
  for (size_t t = 0; t < T; t++)
    ts.emplace_back([&, t] {
      seq_counts(w, za, first + bounds[t], first + bounds[t + 1], cnt[P + t].data());
    });
  for (auto &t : ts) t.join();
  std::vector<std::vector<uint64_t>> base(T, std::vector<uint64_t>(C, 0));
  std::vector<uint64_t> run(C, 0);
  for (size_t t = 0; t < P; t++)
    for (size_t x = 0; x < C; x++) run[x] += cnt[t][x];
  for (size_t t = 0; t < T; t++) {
    base[t] = run;
    for (size_t x = 0; x < C; x++) run[x] += cnt[P + t][x];
  }
  return base;
}

}  // namespace
}  // namespace fh

extern "C" {

fh_status fh_workload_key_histogram(const fh_workload *w, uint64_t first, size_t count,
                                    uint64_t *hist) {
  FH_API_BEGIN
  FH_CHECK(w && hist, FH_EINVAL, "null argument");
  fh::validate(*w);
  const uint64_t K = fh::key_space_of(*w);
  FH_CHECK(K >= 1 && K < (uint64_t(1) << 32), FH_EINVAL, "workload: key space");
  const fh::Alias *za = w->kind == 0 ? &fh::zipf_alias(w->zipf_s, w->key_count) : nullptr;
  const uint32_t k = w->keys_per_cmd;
  const std::vector<size_t> bounds = fh::chunk_bounds(count);
  const size_t T = bounds.size() - 1;
  // per-thread 32-bit counts (a chunk holds < 2^32 commands), summed once
  std::vector<std::vector<uint32_t>> part(T, std::vector<uint32_t>(K, 0));
  std::vector<std::thread> ts;
  for (size_t t = 0; t < T; t++)
    ts.emplace_back([&, t] {
      std::vector<uint64_t> ks(k);
      for (size_t c = bounds[t]; c < bounds[t + 1]; c++) {
        fh::gen_range(*w, za, first + c, 0, 1, nullptr, ks.data(), nullptr, nullptr, nullptr);
        part[t][ks[0]]++;
      }
    });
  for (auto &t : ts) t.join();
  for (uint64_t x = 0; x < K; x++) {
    uint64_t s = 0;
    for (size_t t = 0; t < T; t++) s += part[t][x];
    hist[x] = s;
  }
  FH_API_END
}

fh_status fh_workload_generate_shard(const fh_workload *w, uint64_t first, size_t count,
                                     uint32_t nshards, uint32_t shard, size_t *n_out,
                                     uint64_t *dot, uint64_t *key_id, uint64_t *log_off,
                                     uint32_t *log_cmd) {
  return fh_workload_generate_shard_owned(w, first, count, nullptr, nshards, shard, n_out, dot,
                                          key_id, log_off, log_cmd);
}

fh_status fh_workload_generate_shard_owned(const fh_workload *w, uint64_t first, size_t count,
                                           const uint32_t *owner, uint32_t nshards,
                                           uint32_t shard, size_t *n_out, uint64_t *dot,
                                           uint64_t *key_id, uint64_t *log_off,
                                           uint32_t *log_cmd) {
  FH_API_BEGIN
  FH_CHECK(w && n_out, FH_EINVAL, "null argument");
  fh::validate(*w);
  FH_CHECK(nshards >= 1 && shard < nshards, FH_EINVAL, "workload: shard must be < nshards");
  FH_CHECK(fh::nshards(*w) == 1, FH_EINVAL,
           "workload: key shards of a partially replicated stream: use element logs");
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
      fh::gen_range(*w, za, first + c, 0, 1, nullptr, ks.data(), nullptr, nullptr, nullptr);
      const bool mine = (owner ? owner[ks[0]] : uint32_t(ks[0] % nshards)) == shard;
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
      fh::gen_range(*w, za, first + c, 0, 1, dot + o, key_id + o * k, nullptr, nullptr, nullptr);
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
  FH_CHECK(fh::nshards(*w) == 1, FH_EINVAL,
           "workload: a partially replicated stream's replicas log elements "
           "(fh_workload_generate_element_logs)");
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
  const std::vector<size_t> bounds = fh::chunk_bounds(count);
  const size_t T = bounds.size() - 1;
  std::vector<std::vector<uint64_t>> seq(T);
  if (fh::nshards(*w) > 1) seq = fh::seq_bases(*w, za, first, bounds);
  std::vector<std::thread> ts;
  for (size_t t = 0; t < T; t++)
    ts.emplace_back(fh::gen_range, std::cref(*w), za, first, bounds[t], bounds[t + 1], dot, key_id,
                    fq_proc, fq_time, seq[t].empty() ? nullptr : seq[t].data());
  for (auto &t : ts) t.join();
  FH_API_END
}

fh_status fh_workload_generate_element_logs(const fh_workload *w, uint64_t first, size_t count,
                                            uint64_t *log_off, uint32_t *log_elem) {
  FH_API_BEGIN
  FH_CHECK(w && log_off && log_elem, FH_EINVAL, "null argument");
  fh::validate(*w);
  FH_CHECK(w->views >= 1, FH_EINVAL, "workload: logs need replica views (views >= 1)");
  const uint32_t k = w->keys_per_cmd, V = w->views, n = w->n, S = fh::nshards(*w);
  const uint32_t nlog = n * S, per = k * V;
  FH_CHECK(uint64_t(count) * per < (uint64_t(1) << 31), FH_EINVAL,
           "workload: element positions must be < 2^31");
  // the arrival sort below keeps each element's delay (< window) in a byte
  FH_CHECK(w->window <= 256, FH_EINVAL, "workload: element logs need window <= 256");
  const fh::Alias *za = w->kind == 0 ? &fh::zipf_alias(w->zipf_s, w->key_count) : nullptr;
  const std::vector<size_t> bounds = fh::chunk_bounds(count);
  const size_t T = bounds.size() - 1;
  // element (c, s, j) -> its replica's log: shard h of key slot s, the
  // shard's process (i + j) mod n
  auto each = [&](size_t lo, size_t hi, auto f) {
    uint64_t ks[8];
    for (size_t c = lo; c < hi; c++) {
      const uint64_t i = first + c;
      const uint32_t l = uint32_t(i % n);
      fh::gen_keys(*w, za, i, ks);
      for (uint32_t s = 0; s < k; s++) {
        const uint32_t h = uint32_t(ks[s] % S);
        for (uint32_t j = 0; j < V; j++)
          f(n * h + (l + j) % n, uint32_t((c * V + j) * k + s), fh::member_delay(*w, i, h, j));
      }
    }
  };
  std::vector<std::vector<uint64_t>> cnt(T, std::vector<uint64_t>(nlog, 0));
  {
    std::vector<std::thread> ts;
    for (size_t t = 0; t < T; t++)
      ts.emplace_back([&, t] { each(bounds[t], bounds[t + 1], [&](uint32_t r, uint32_t, uint32_t) {
                                 cnt[t][r]++;
                               }); });
    for (auto &t : ts) t.join();
  }
  // log r's entries of chunk t start at its offset plus the earlier chunks'
  log_off[0] = 0;
  for (uint32_t r = 0; r < nlog; r++) {
    uint64_t tot = 0;
    for (size_t t = 0; t < T; t++) tot += cnt[t][r];
    log_off[r + 1] = log_off[r] + tot;
  }
  FH_CHECK(log_off[nlog] == uint64_t(count) * per, FH_EINVARIANT, "element log count");
  std::vector<uint8_t> dly(count * per);
  {
    std::vector<std::vector<uint64_t>> pos(T, std::vector<uint64_t>(nlog));
    for (uint32_t r = 0; r < nlog; r++) {
      uint64_t o = log_off[r];
      for (size_t t = 0; t < T; t++) {
        pos[t][r] = o;
        o += cnt[t][r];
      }
    }
    std::vector<std::thread> ts;
    for (size_t t = 0; t < T; t++)
      ts.emplace_back([&, t] {
        each(bounds[t], bounds[t + 1], [&](uint32_t r, uint32_t p, uint32_t d) {
          const uint64_t o = pos[t][r]++;
          log_elem[o] = p;
          dly[o] = uint8_t(d);
        });
      });
    for (auto &t : ts) t.join();
  }
  // each log in arrival order (time (c + d)·W + d, then position: one
  // command's elements at a replica arrive together, slot order): the
  // entries are in command order, displaced by less than the window, so an
  // insertion sort is near linear
  std::vector<std::thread> ts;
  const uint32_t nt = std::min<uint32_t>(nlog, 16);
  for (uint32_t t = 0; t < nt; t++)
    ts.emplace_back([&, t] {
      for (uint32_t r = t; r < nlog; r += nt) {
        const uint64_t a = log_off[r], b = log_off[r + 1];
        auto key = [&](uint64_t x) {
          return ((uint64_t(log_elem[x] / per) + dly[x]) << 8) | dly[x];
        };
        for (uint64_t x = a + 1; x < b; x++) {
          const uint32_t p = log_elem[x];
          const uint8_t d = dly[x];
          const uint64_t kx = key(x);
          uint64_t y = x;
          while (y > a) {
            const uint64_t ky = key(y - 1);
            if (ky < kx || (ky == kx && log_elem[y - 1] < p)) break;
            log_elem[y] = log_elem[y - 1];
            dly[y] = dly[y - 1];
            y--;
          }
          log_elem[y] = p;
          dly[y] = d;
        }
      }
    });
  for (auto &t : ts) t.join();
  FH_API_END
}

}  // extern "C"
