// multi.cpp -- fh_multi_*: the fused engine over several GPUs of one node
// from one process (SURVEY §8b "fh_multi_create / fh_multi_run", §8e).
//
// Key-shard partition: owner(key) from fh_key_owners_balanced over the
// staged stream's per-key work estimates (command counts weighted up for
// hot keys; G = engines; key mod G left the largest of 8 shards at 1.37x the
// mean under Zipf 0.99).  With one key
// per command every dependency joins two commands of one key (each
// replica's KeyDeps chains a key's commands, keys/sequential.rs:72-104), so
// a shard's dependency graph is closed: the shards order independently and
// concurrently (one host thread per device, each engine on its own stream),
// no data-path exchange.  Every shard keeps the global dots and its
// replicas' arrival logs restricted to its commands.  Results merge back to
// the stream's command order; per-key sequences come from each key's owner;
// the execution order is the shards' orders concatenated (shards share no
// dependency, so any interleaving is an execution order).
//
// Multi-key commands across shards (partial replication, C5) need the
// dependency union across owners and cross-shard SCC exchange; those go
// through fh_dep_union + the partial-replication executor (PartialShard,
// fh_graph_*_sharded), not this entry: FH_ENOTIMPL for keys_per_cmd > 1.
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fh_common.h"

struct fh_multi {
  fh_config cfg{};
  std::vector<int> devices;
  std::vector<fh_engine *> eng;
  std::vector<std::vector<uint32_t>> cmds;  // per shard: global command indices
  std::vector<uint32_t> owner;              // key -> shard of the last staging
  fh_stream_desc desc{};
  size_t n = 0;
  bool staged = false, ran = false;
  ~fh_multi() {
    for (auto *e : eng)
      if (e) fh_engine_destroy(e);
  }
};

namespace {

void check_status(fh_status st) {
  if (st != FH_OK) throw fh::Error(st, fh_last_error());
}

// run f(shard) on one thread per shard; rethrow the first error
template <class F>
void per_shard(fh_multi *h, F f) {
  std::vector<std::thread> ts;
  std::vector<std::string> err(h->eng.size());
  std::vector<fh_status> code(h->eng.size(), FH_OK);
  for (size_t g = 0; g < h->eng.size(); g++)
    ts.emplace_back([&, g] {
      try {
        FH_HIP(hipSetDevice(h->devices[g]));
        f(g);
      } catch (const fh::Error &e) {
        err[g] = e.what();
        code[g] = e.code;
      } catch (const std::exception &e) {
        err[g] = e.what();
        code[g] = FH_EINVARIANT;
      }
    });
  for (auto &t : ts) t.join();
  for (size_t g = 0; g < err.size(); g++)
    if (code[g] != FH_OK) throw fh::Error(code[g], "shard " + std::to_string(g) + ": " + err[g]);
}

}  // namespace

extern "C" {

fh_status fh_multi_create(const fh_config *cfg, size_t ndev, const int32_t *devices,
                          fh_multi **out) {
  FH_API_BEGIN
  FH_CHECK(cfg && out && ndev >= 1 && ndev <= 64, FH_EINVAL, "bad argument");
  auto *h = new fh_multi();
  try {
    h->cfg = *cfg;
    for (size_t g = 0; g < ndev; g++) {
      fh_config c = *cfg;
      c.device = devices ? devices[g] : int32_t(g);
      h->devices.push_back(c.device);
      fh_engine *e = nullptr;
      check_status(fh_engine_create(&c, &e));
      h->eng.push_back(e);
    }
  } catch (...) {
    delete h;
    throw;
  }
  *out = h;
  FH_API_END
}

fh_status fh_multi_destroy(fh_multi *h) {
  FH_API_BEGIN
  delete h;
  FH_API_END
}

fh_status fh_multi_stage_logs(fh_multi *h, const fh_stream_desc *desc, const uint64_t *dot,
                              const uint64_t *key_id, const uint64_t *log_off,
                              const uint32_t *log_cmd) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  // whatever happens below, the previous staging is gone: run() and
  // results() refuse until a staging completes
  h->staged = false;
  h->ran = false;
  FH_CHECK(desc && dot && key_id && log_off && log_cmd, FH_EINVAL, "null argument");
  FH_CHECK(desc->keys_per_cmd == 1, FH_ENOTIMPL,
           "fh_multi: key shards need one key per command (closed per-shard graphs)");
  FH_CHECK(desc->views >= 1 && desc->nproc >= 1, FH_EINVAL, "fh_multi: replica views only");
  const size_t G = h->eng.size(), n = desc->n, np = desc->nproc;
  // validate and partition into locals; h->cmds / h->n change only after
  // every shard staged
  FH_CHECK(log_off[0] == 0 && log_off[np] == n * desc->views, FH_EINVAL,
           "logs: every command must appear in exactly `views` replica logs");
  for (size_t r = 0; r < np; r++)
    FH_CHECK(log_off[r + 1] >= log_off[r], FH_EINVAL, "logs: offsets");
  for (uint64_t q = 0; q < log_off[np]; q++)
    FH_CHECK(log_cmd[q] < n, FH_EINVAL, "logs: command index >= n");
  const size_t K = h->cfg.key_space;
  std::vector<uint64_t> hist(K, 0);
  for (size_t i = 0; i < n; i++) {
    FH_CHECK(key_id[i] < K, FH_EINVAL, "key id >= key_space");
    hist[key_id[i]]++;
  }
  // packed by estimated work, not by count: a hot key's commands cost more
  // (longer same-key scans in the search, larger ready groups in the tile
  // kernel), count x (1 + 14 x share), x16 -- fantoch_amd/workload.py
  // key_weights, measured on the C4 stream's 8 shards
  std::vector<uint64_t> wt(K);
  for (size_t x = 0; x < K; x++) {
    const double h = double(hist[x]);
    wt[x] = uint64_t(16.0 * h * (1.0 + 14.0 * h / double(std::max<size_t>(n, 1))) + 0.5);
  }
  std::vector<uint32_t> owner(K);
  check_status(fh_key_owners_balanced(wt.data(), K, uint32_t(G), owner.data()));
  std::vector<uint32_t> shard_of(n), local(n);
  std::vector<std::vector<uint32_t>> cmds(G);
  for (size_t i = 0; i < n; i++) {
    const uint32_t g = owner[key_id[i]];
    shard_of[i] = g;
    local[i] = uint32_t(cmds[g].size());
    cmds[g].push_back(uint32_t(i));
  }
  per_shard(h, [&](size_t g) {
    const auto &c = cmds[g];
    std::vector<uint64_t> d(c.size()), k(c.size()), off(np + 1, 0);
    for (size_t j = 0; j < c.size(); j++) {
      d[j] = dot[c[j]];
      k[j] = key_id[c[j]];
    }
    std::vector<uint32_t> lc;
    lc.reserve(c.size() * desc->views);
    for (size_t r = 0; r < np; r++) {
      for (uint64_t q = log_off[r]; q < log_off[r + 1]; q++)
        if (shard_of[log_cmd[q]] == g) lc.push_back(local[log_cmd[q]]);
      off[r + 1] = lc.size();
    }
    fh_stream_desc sd = *desc;
    sd.n = c.size();
    check_status(fh_engine_stage_logs(h->eng[g], &sd, 1, d.data(), k.data(), off.data(),
                                      lc.data()));
  });
  h->cmds.swap(cmds);
  h->owner.swap(owner);
  h->desc = *desc;
  h->n = n;
  h->staged = true;
  FH_API_END
}

fh_status fh_multi_rewind(fh_multi *h) {
  FH_API_BEGIN
  FH_CHECK(h && h->staged, FH_EINVAL, "nothing staged");
  for (auto *e : h->eng) check_status(fh_engine_rewind(e));
  FH_API_END
}

fh_status fh_multi_sync(fh_multi *h) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  for (auto *e : h->eng) check_status(fh_engine_sync(e));
  FH_API_END
}

fh_status fh_multi_run(fh_multi *h, float *device_ms) {
  FH_API_BEGIN
  FH_CHECK(h && h->staged, FH_EINVAL, "nothing staged");
  std::vector<float> ms(h->eng.size(), 0.f);
  per_shard(h, [&](size_t g) { check_status(fh_engine_run(h->eng[g], device_ms ? &ms[g] : nullptr)); });
  if (device_ms) *device_ms = *std::max_element(ms.begin(), ms.end());
  h->ran = true;
  FH_API_END
}

fh_status fh_multi_results(fh_multi *h, uint32_t *dep_off, uint64_t *dep_dot, size_t dep_cap,
                           size_t *dep_len, uint64_t *scc_label, uint32_t *exec_rank,
                           uint32_t *key_off, uint64_t *key_seq) {
  FH_API_BEGIN
  FH_CHECK(h && h->ran, FH_EINVAL, "no run to read results from");
  const size_t G = h->eng.size(), n = h->n, K = h->cfg.key_space;
  struct R {
    std::vector<uint32_t> off, rank, koff;
    std::vector<uint64_t> deps, lab, seq;
  };
  std::vector<R> r(G);
  per_shard(h, [&](size_t g) {
    const size_t m = h->cmds[g].size();
    R &x = r[g];
    x.off.resize(m + 1);
    x.koff.resize(K + 1);
    size_t len = 0;
    check_status(fh_engine_results(h->eng[g], x.off.data(), nullptr, 0, &len, nullptr, nullptr,
                                   x.koff.data(), nullptr));
    x.deps.resize(len + 1);
    x.lab.resize(m + 1);
    x.rank.resize(m + 1);
    x.seq.resize(x.koff[K] + 1);
    check_status(fh_engine_results(h->eng[g], x.off.data(), x.deps.data(), len, &len,
                                   x.lab.data(), x.rank.data(), x.koff.data(), x.seq.data()));
  });
  // committed deps in the stream's command order
  size_t total = 0;
  for (auto &x : r) total += x.off.back();
  if (dep_len) *dep_len = total;
  if (dep_dot) FH_CHECK(dep_cap >= total, FH_ECAP, "dep output capacity too small");
  std::vector<uint32_t> cnt(n + 1, 0);
  std::vector<std::pair<uint32_t, uint32_t>> where(n);  // (shard, local)
  for (size_t g = 0; g < G; g++)
    for (size_t j = 0; j < h->cmds[g].size(); j++) {
      const uint32_t i = h->cmds[g][j];
      where[i] = {uint32_t(g), uint32_t(j)};
      cnt[i] = r[g].off[j + 1] - r[g].off[j];
    }
  std::vector<uint32_t> off(n + 1, 0);
  for (size_t i = 0; i < n; i++) off[i + 1] = off[i] + cnt[i];
  if (dep_off) std::memcpy(dep_off, off.data(), (n + 1) * sizeof(uint32_t));
  std::vector<uint32_t> base(G + 1, 0);
  for (size_t g = 0; g < G; g++) base[g + 1] = base[g] + uint32_t(h->cmds[g].size());
  for (size_t i = 0; i < n; i++) {
    const auto [g, j] = where[i];
    if (dep_dot)
      std::copy(r[g].deps.begin() + r[g].off[j], r[g].deps.begin() + r[g].off[j + 1],
                dep_dot + off[i]);
    if (scc_label) scc_label[i] = r[g].lab[j];
    if (exec_rank) exec_rank[i] = base[g] + r[g].rank[j];
  }
  // per-key sequences: key k's comes from its owner
  if (key_off || key_seq) {
    std::vector<uint32_t> ko(K + 1, 0);
    for (size_t k = 0; k < K; k++) {
      const R &x = r[h->owner[k]];
      ko[k + 1] = ko[k] + (x.koff[k + 1] - x.koff[k]);
    }
    if (key_off) std::memcpy(key_off, ko.data(), (K + 1) * sizeof(uint32_t));
    if (key_seq)
      for (size_t k = 0; k < K; k++) {
        const R &x = r[h->owner[k]];
        std::copy(x.seq.begin() + x.koff[k], x.seq.begin() + x.koff[k + 1], key_seq + ko[k]);
      }
  }
  FH_API_END
}

fh_status fh_multi_shard_size(fh_multi *h, size_t shard, size_t *n) {
  FH_API_BEGIN
  FH_CHECK(h && n && shard < h->eng.size(), FH_EINVAL, "bad argument");
  *n = h->cmds.size() > shard ? h->cmds[shard].size() : 0;
  FH_API_END
}

fh_status fh_multi_owners(fh_multi *h, uint32_t *owner) {
  FH_API_BEGIN
  FH_CHECK(h && owner && h->staged, FH_EINVAL, "bad argument");
  std::copy(h->owner.begin(), h->owner.end(), owner);
  FH_API_END
}

fh_status fh_key_owners_balanced(const uint64_t *hist, size_t key_space, uint32_t nshards,
                                 uint32_t *owner) {
  FH_API_BEGIN
  FH_CHECK(hist && owner && nshards >= 1 && key_space >= 1, FH_EINVAL, "bad argument");
  std::vector<uint32_t> ord(key_space);
  for (size_t x = 0; x < key_space; x++) ord[x] = uint32_t(x);
  std::stable_sort(ord.begin(), ord.end(),
                   [&](uint32_t a, uint32_t b) { return hist[a] > hist[b]; });
  // min-heap of (load, shard)
  using E = std::pair<uint64_t, uint32_t>;
  std::vector<E> heap;
  for (uint32_t g = 0; g < nshards; g++) heap.push_back({0, g});
  auto gt = [](const E &a, const E &b) { return a > b; };
  std::make_heap(heap.begin(), heap.end(), gt);
  for (uint32_t x : ord) {
    std::pop_heap(heap.begin(), heap.end(), gt);
    E &e = heap.back();
    owner[x] = e.second;
    e.first += hist[x];
    std::push_heap(heap.begin(), heap.end(), gt);
  }
  FH_API_END
}

}  // extern "C"
