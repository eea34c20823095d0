// stream_bench.cpp -- streaming throughput of the executor path (fh_graph_*)
// at a given batch size: a C4-shaped stream (Zipf 0.99 over 2^20 keys, 1 key
// per command, Atlas n=5 f=1 replica views, window 64) is committed by the
// fused engine (fh_engine: per-replica KeyDeps + union), then fed to one
// fh_graph in stream order, `batch` Adds per fh_graph_add_batch, draining
// after every call -- what GraphExecutor::handle + fetch_actions do per
// ExecutionInfo (executor.rs:76-145; the runners drain after every handle,
// run/task/executor.rs:150-175).  Timed: the add + drain loop (host arrays
// in, executed dots out: PCIe included), from a fresh graph.
//
// Usage: tools/stream_bench <batch> <commands> [<batch> <commands> ...]
// Prints one JSON line per pair.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fantoch_hip.h"

#define CK(x)                                                                 \
  do {                                                                        \
    fh_status s_ = (x);                                                       \
    if (s_ != FH_OK) {                                                        \
      fprintf(stderr, "%s failed: %d %s\n", #x, int(s_), fh_last_error());   \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 3 || (argc - 1) % 2) {
    fprintf(stderr, "usage: %s <batch> <commands> [...]\n", argv[0]);
    return 2;
  }
  size_t nmax = 0;
  for (int a = 2; a < argc; a += 2) nmax = std::max<size_t>(nmax, strtoull(argv[a], nullptr, 10));
  fh_workload w{};
  w.seed = 0xFA170C4000000004ull;
  w.n = 5;
  w.keys_per_cmd = 1;
  w.kind = 0;
  w.clients = 1024;
  w.zipf_s = 0.99;
  w.key_count = 1u << 20;
  w.views = 3;
  w.window = 64;
  const uint64_t K = fh_workload_key_space(&w);
  std::vector<uint64_t> dot(nmax), key(nmax), loff(w.n + 1);
  std::vector<uint32_t> lcmd(nmax * w.views);
  CK(fh_workload_generate(&w, 0, nmax, dot.data(), key.data(), nullptr, nullptr));
  CK(fh_workload_generate_logs(&w, 0, nmax, loff.data(), lcmd.data()));
  // committed deps of the whole prefix (the engine: deps only)
  fh_config cfg{};
  cfg.n = 5;
  cfg.f = 1;
  cfg.shard_count = 1;
  cfg.device = 0;
  cfg.key_space = K;
  fh_engine *e = nullptr;
  CK(fh_engine_create(&cfg, &e));
  CK(fh_engine_set_deps_only(e, 1));
  fh_stream_desc d{};
  d.n = nmax;
  d.keys_per_cmd = 1;
  d.views = w.views;
  d.nproc = w.n;
  CK(fh_engine_stage_logs(e, &d, 1, dot.data(), key.data(), loff.data(), lcmd.data()));
  CK(fh_engine_run(e, nullptr));
  std::vector<uint32_t> doff(nmax + 1);
  size_t nd = 0;
  CK(fh_engine_results(e, doff.data(), nullptr, 0, &nd, nullptr, nullptr, nullptr, nullptr));
  std::vector<uint64_t> deps(nd + 1);
  CK(fh_engine_results(e, doff.data(), deps.data(), deps.size(), &nd, nullptr, nullptr, nullptr,
                       nullptr));
  CK(fh_engine_destroy(e));
  std::vector<uint32_t> koff(nmax + 1);
  for (size_t i = 0; i <= nmax; i++) koff[i] = uint32_t(i);
  for (int a = 1; a < argc; a += 2) {
    const size_t B = strtoull(argv[a], nullptr, 10), n = strtoull(argv[a + 1], nullptr, 10);
    fh_graph *g = nullptr;
    CK(fh_graph_create(1, 0, &cfg, &g));
    std::vector<uint32_t> bko(B + 1), bdo(B + 1);
    std::vector<uint64_t> out(n + 1), lab(n + 1);
    size_t executed = 0, calls = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < n; i += B) {
      const size_t m = std::min(B, n - i);
      for (size_t j = 0; j <= m; j++) {
        bko[j] = uint32_t(j);
        bdo[j] = doff[i + j] - doff[i];
      }
      CK(fh_graph_add_batch(g, m, dot.data() + i, bko.data(), key.data() + i, bdo.data(),
                            deps.data() + doff[i]));
      size_t len = 0;
      CK(fh_graph_drain(g, out.data() + executed, nullptr, n - executed, &len));
      executed += len;
      calls++;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // the prefix's last commands may wait for deps on commands past it
    size_t pending = 0;
    CK(fh_graph_pending(g, &pending));
    printf("{\"batch\": %zu, \"commands\": %zu, \"executed\": %zu, \"pending\": %zu, "
           "\"seconds\": %.4f, \"commands_per_s\": %.1f, \"us_per_batch\": %.2f}\n",
           B, n, executed, pending, s, double(n) / s, s * 1e6 / double(calls));
    fflush(stdout);
    CK(fh_graph_destroy(g));
  }
  return 0;
}
