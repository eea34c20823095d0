// graph_api.hip -- the GraphExecutor drop-in (fh_graph_*).
//
// DependencyGraph semantics (fantoch_ps/src/executor/graph/mod.rs:45-679) for
// batches of GraphExecutionInfo::Add: vertices = carried pending vertices
// (earlier arrivals) + the batch; dependency dots resolve to vertex ids by a
// device sort of the vertex dots and binary search; a dependency that is
// neither a vertex nor executed is missing (the vertex stays pending, exactly
// like TarjanSCCFinder's MissingDependencies, tarjan.rs:150-170, and the
// PendingIndex retry, mod.rs:558-644); SCCs, execution order and per-key
// order come from GraphCore on the device.  The executed clock is an
// AEClock<ProcessId> (frontier + exceptions, threshold crate) kept on the
// host and mirrored to the device per batch.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "dotindex.h"
#include "execlog.h"
#include "graph_core.h"
#include "graph_small.h"

namespace fh {

#define GRID_STRIDE(i, n) \
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += gridDim.x * blockDim.x)

__global__ void k_dup_check(uint32_t V, const uint64_t *__restrict__ sd, uint32_t *err) {
  GRID_STRIDE(j, V) {
    if (j > 0 && sd[j] == sd[j - 1]) atomicOr(err, 1u);
  }
}

namespace {

constexpr unsigned B = 256;

// per vertex: count resolved edges, flag missing dependencies
// (tarjan.rs:131-170: self and executed deps are ignored)
__global__ void k_resolve_count(uint32_t V, const uint64_t *__restrict__ dot,
                                const uint32_t *__restrict__ doff, const uint64_t *__restrict__ ddot,
                                const uint64_t *__restrict__ sd, const uint32_t *__restrict__ sv,
                                const uint64_t *__restrict__ frontier,
                                const uint64_t *__restrict__ exc, uint32_t nexc,
                                uint32_t *__restrict__ cnt, uint8_t *__restrict__ blocked0) {
  GRID_STRIDE(v, V) {
    uint32_t c = 0;
    bool missing = false;
    const uint64_t self = dot[v];
    for (uint32_t e = doff[v]; e < doff[v + 1]; e++) {
      const uint64_t d = ddot[e];
      if (d == self || executed_dev(d, frontier, exc, nexc)) continue;
      if (find_vid(d, sd, sv, V) >= 0)
        c++;
      else
        missing = true;
    }
    cnt[v] = c;
    blocked0[v] = missing;
  }
}

__global__ void k_resolve_fill(uint32_t V, const uint64_t *__restrict__ dot,
                               const uint32_t *__restrict__ doff, const uint64_t *__restrict__ ddot,
                               const uint64_t *__restrict__ sd, const uint32_t *__restrict__ sv,
                               const uint64_t *__restrict__ frontier,
                               const uint64_t *__restrict__ exc, uint32_t nexc,
                               const uint32_t *__restrict__ off, uint32_t *__restrict__ dst) {
  GRID_STRIDE(v, V) {
    uint32_t o = off[v];
    const uint64_t self = dot[v];
    for (uint32_t e = doff[v]; e < doff[v + 1]; e++) {
      const uint64_t d = ddot[e];
      if (d == self || executed_dev(d, frontier, exc, nexc)) continue;
      const int64_t u = find_vid(d, sd, sv, V);
      if (u >= 0) dst[o++] = uint32_t(u);
    }
  }
}

// The batch's rows, uploaded as one block, appended after the carried
// prefix (offsets rebased past it); the executed-clock mirror rides along
// when it changed (nf = 256 frontier words, then ne exceptions).
__global__ void k_append(Upload u, AppendDst a) {
  const uint32_t m = append_items(u);
  GRID_STRIDE(i, m) append_item(u, a, i);
}

// executed vertices in execution order: their dots and SCC labels
// (ocar: per executed vertex, carried from an earlier pass -- vid below the
// carried prefix P -- so the host looks up pending metadata only for those)
__global__ void k_gather_exec(uint32_t m, const uint32_t *__restrict__ order,
                              const uint64_t *__restrict__ dot, const uint64_t *__restrict__ label,
                              uint32_t P, uint64_t *__restrict__ odot, uint64_t *__restrict__ olab,
                              uint8_t *__restrict__ ocar) {
  GRID_STRIDE(j, m) {
    const uint32_t v = order[j];
    odot[j] = dot[v];
    olab[j] = label[v];
    ocar[j] = v < P ? 1 : 0;
  }
}

// pending compaction: per vertex kept (1), its key and dep counts
__global__ void k_keep_counts(uint32_t V, const uint8_t *__restrict__ blocked,
                              const uint32_t *__restrict__ koff, const uint32_t *__restrict__ doff,
                              uint32_t *__restrict__ kv, uint32_t *__restrict__ kk,
                              uint32_t *__restrict__ kd) {
  GRID_STRIDE(v, V) {
    const bool keep = blocked[v] != 0;
    kv[v] = keep;
    kk[v] = keep ? koff[v + 1] - koff[v] : 0u;
    kd[v] = keep ? doff[v + 1] - doff[v] : 0u;
  }
}

__global__ void k_keep_copy(uint32_t V, const uint8_t *__restrict__ blocked,
                            const uint64_t *__restrict__ dot, const uint32_t *__restrict__ koff,
                            const uint32_t *__restrict__ key32, const uint32_t *__restrict__ doff,
                            const uint64_t *__restrict__ ddot, const uint32_t *__restrict__ pv,
                            const uint32_t *__restrict__ pk, const uint32_t *__restrict__ pd,
                            uint64_t *__restrict__ ndot, uint32_t *__restrict__ nkoff,
                            uint32_t *__restrict__ nkey32, uint32_t *__restrict__ ndoff,
                            uint64_t *__restrict__ nddot) {
  GRID_STRIDE(v, V) {
    if (!blocked[v]) continue;
    const uint32_t o = pv[v];
    ndot[o] = dot[v];
    nkoff[o] = pk[v];
    ndoff[o] = pd[v];
    for (uint32_t e = koff[v], q = pk[v]; e < koff[v + 1]; e++, q++) nkey32[q] = key32[e];
    for (uint32_t e = doff[v], q = pd[v]; e < doff[v + 1]; e++, q++) nddot[q] = ddot[e];
  }
}

// the missing dependencies (neither executed nor a vertex) of the vertices
// that have one, appended to a list (order and repeats do not matter)
__global__ void k_missing_list(uint32_t V, const uint8_t *__restrict__ blocked0,
                               const uint64_t *__restrict__ dot, const uint32_t *__restrict__ doff,
                               const uint64_t *__restrict__ ddot, const uint64_t *__restrict__ sd,
                               const uint32_t *__restrict__ sv,
                               const uint64_t *__restrict__ frontier,
                               const uint64_t *__restrict__ exc, uint32_t nexc, uint32_t cap,
                               uint32_t *__restrict__ n_out, uint64_t *__restrict__ out) {
  GRID_STRIDE(v, V) {
    if (!blocked0[v]) continue;
    const uint64_t self = dot[v];
    for (uint32_t e = doff[v]; e < doff[v + 1]; e++) {
      const uint64_t d = ddot[e];
      if (d == self || executed_dev(d, frontier, exc, nexc) || find_vid(d, sd, sv, V) >= 0)
        continue;
      const uint32_t q = atomicAdd(n_out, 1u);
      if (q < cap) out[q] = d;
    }
  }
}

// DBuf growth that keeps the first `keep` elements (the carried prefix)
template <class T>
static T *grow_keep(DBuf<T> &b, size_t need, size_t keep, hipStream_t s) {
  if (b.get() && need <= b.cap) return b.get();
  DBuf<T> n;
  n.ensure(need + need / 2);
  if (keep && b.get())
    FH_HIP(hipMemcpyAsync(n.get(), b.get(), keep * sizeof(T), hipMemcpyDeviceToDevice, s));
  FH_HIP(hipStreamSynchronize(s));
  b.swap(n);
  return b.get();
}

}  // namespace

struct GraphDevice {
  uint32_t process_id;
  uint64_t shard_id;
  fh_config cfg;
  int device = 0;
  hipStream_t stream = nullptr;
  int key_bits = 1;
  AEClock clock;
  // Carried pending vertices.  The device keeps them between batches in
  // arrival order (dots, key lists, dependency lists: set `cur` of two, the
  // pass compacts the survivors into the other), so a batch uploads only its
  // own commands.  The host keeps what the control paths need per pending
  // dot (request replies, the watchdog, metrics): Command::shards() bitmask,
  // the dependencies with their Dependency::shards bitmasks, the add time and
  // the arrival sequence.
  struct PInfo {
    uint64_t seq, cshard, time;
    std::vector<uint64_t> deps, dshards;
  };
  std::unordered_map<uint64_t, PInfo> pend;
  std::map<uint64_t, uint64_t> porder;  // arrival seq -> dot
  uint64_t next_seq = 0;
  struct DSet {
    DBuf<uint64_t> dot, ddot;
    DBuf<uint32_t> koff, key32, doff;
    uint32_t P = 0, KP = 0, DP = 0;
  } ds[2];
  int cur = 0;
  std::vector<uint64_t> exc_sorted;  // the clock's exceptions as on the device
  uint64_t exc_version = ~uint64_t(0);
  // partial replication (graph/mod.rs:139-157, 279-375; index.rs:145-211):
  // requested = dots already indexed as a missing non-local dependency
  // (PendingIndex keys that produced a request), out_requests = requests()
  // not yet taken, buffered = buffered_in_requests, replies = out_request_replies
  std::unordered_set<uint64_t> requested;
  std::set<std::pair<uint64_t, uint64_t>> out_requests;  // (target shard, dot)
  std::map<uint64_t, std::set<uint64_t>> buffered;       // from shard -> dots
  struct Reply {
    uint64_t to, dot, cshard;
    uint8_t kind;  // FH_REPLY_INFO / FH_REPLY_EXECUTED
    std::vector<uint64_t> deps, dshards;
  };
  std::vector<Reply> replies;
  // drain queue
  std::deque<std::pair<uint64_t, uint64_t>> ready;
  std::vector<uint64_t> missing_now;
  // time (SysTime::millis of the caller, fh_graph_set_time): vertices are
  // stamped when added (Vertex::new, tarjan.rs:335-351)
  uint64_t now_ms = 0;
  // executor metrics not yet taken (ExecutorMetricsKind, executor/mod.rs:
  // 122-129): ChainSize per executed SCC, ExecutionDelay per command
  // (save_scc, graph/mod.rs:490-525)
  std::vector<uint64_t> m_chain, m_delay;
  // the executed clock changed since the last pass (a pending retry with no
  // new vertex and no missing dependency executed since has nothing to do)
  bool clock_changed = false;
  uint64_t passes = 0, skipped = 0;
  // device buffers
  DBuf<uint64_t> d_sd, d_sd2, d_frontier, d_exc, d_xdot, d_xlab, d_miss;
  DBuf<uint8_t> d_xcar;
  uint8_t *h_up = nullptr;      // the batch's upload block: mapped pinned host memory
  uint8_t *h_up_dev = nullptr;  // its device address (k_append reads it)
  size_t h_up_cap = 0;
  DBuf<uint32_t> d_cnt, d_off, d_dst, d_sv, d_sv2, d_err, d_kv, d_kk, d_kd, d_pv, d_pk, d_pd;
  DBuf<uint8_t> d_blocked0;
  SortWorkspace sort_ws;
  ScanWorkspace scan_ws;
  GraphCore core;

  GraphDevice(uint32_t pid, uint64_t sid, const fh_config &c) : process_id(pid), shard_id(sid), cfg(c) {
    FH_CHECK(c.key_space >= 1 && c.key_space <= (uint64_t(1) << 31), FH_EINVAL,
             "key_space must be in [1, 2^31]");
    key_bits = bits_for(c.key_space);
    device = pick_device(&c, sid);
    FH_HIP(hipSetDevice(device));
    FH_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    core.stream = stream;
    d_err.ensure(4);
    d_frontier.ensure(256);
    for (auto &d : ds) {
      d.koff.ensure(16);
      d.doff.ensure(16);
      FH_HIP(hipMemsetAsync(d.koff.get(), 0, sizeof(uint32_t), stream));
      FH_HIP(hipMemsetAsync(d.doff.get(), 0, sizeof(uint32_t), stream));
    }
    FH_HIP(hipStreamSynchronize(stream));
  }
  ~GraphDevice() {
    (void)hipSetDevice(device);
    // the stream first: a pass that missed its deadline may still write the
    // mapped blocks
    if (stream) (void)hipStreamSynchronize(stream);
    if (h_small) (void)hipHostFree(h_small);
    if (h_up) (void)hipHostFree(h_up);
    if (stream) (void)hipStreamDestroy(stream);
  }

  // PendingIndex::index (index.rs:171-205) as called by index_pending
  // (mod.rs:527-556) on the first find of each added vertex: a dependency
  // missing when its child is added (not executed, not a carried vertex, not
  // an earlier vertex of this batch) and not replicated by this shard is
  // requested from dep.dot.target_shard(n) the first time it is indexed.  In
  // partial replication the first find collects every missing dependency of
  // the reachable set (tarjan.rs:161-169); the reachable vertices' own missing
  // deps were indexed on their own first finds (missing is monotone: missing
  // -> present -> executed), so the direct deps of each added vertex suffice.
  void index_requests(size_t n, const uint64_t *dot, const uint32_t *dep_off,
                      const uint64_t *dep_dot, const uint64_t *dep_shards) {
    if (cfg.shard_count <= 1 || !dep_shards || n == 0) return;
    std::unordered_map<uint64_t, size_t> pos;
    pos.reserve(n);
    for (size_t i = 0; i < n; i++) pos.emplace(dot[i], i);
    const uint32_t nproc = cfg.n ? cfg.n : 1;
    for (size_t i = 0; i < n; i++) {
      for (uint32_t e = dep_off[i]; e < dep_off[i + 1]; e++) {
        const uint64_t d = dep_dot[e];
        if (d == dot[i] || clock.contains(d) || carried(d)) continue;
        auto it = pos.find(d);
        if (it != pos.end() && it->second < i) continue;
        // "shards should be set if it's not a noop" (index.rs:190-194)
        FH_CHECK(dep_shards[e] != 0, FH_EINVARIANT,
                 "PendingIndex::index: missing dependency without a shard set");
        if ((dep_shards[e] >> shard_id) & 1) continue;  // is_mine
        if (!requested.insert(d).second) continue;     // already indexed
        const uint64_t target = ((d >> 56) - 1) / nproc;  // Dot::target_shard (id.rs:59-61)
        out_requests.emplace(target, d);
      }
    }
  }

  // process_requests (mod.rs:297-375): Info for an indexed vertex, Executed
  // for an executed dot, otherwise buffer until the next cleanup.
  // a carried (pending) vertex; batch vertices enter `pend` only after the
  // pass that indexes them
  bool carried(uint64_t d) const { return pend.count(d) != 0 && pend.at(d).seq < batch_seq0; }
  uint64_t batch_seq0 = ~uint64_t(0);

  void process_requests(uint64_t from, const uint64_t *dots, size_t n) {
    for (size_t i = 0; i < n; i++) {
      const uint64_t d = dots[i];
      auto it = pend.find(d);
      if (it != pend.end()) {
        const PInfo &pi = it->second;
        // panic if the shard that requested this vertex replicates it (:313-322)
        FH_CHECK(from >= 64 || !((pi.cshard >> from) & 1), FH_EINVARIANT,
                 "Graph::process_requests: requested dot is replicated by the requesting shard");
        Reply r{from, d, pi.cshard, FH_REPLY_INFO, pi.deps, pi.dshards};
        replies.push_back(std::move(r));
      } else if (clock.contains(d)) {
        replies.push_back(Reply{from, d, 0, FH_REPLY_EXECUTED, {}, {}});
      } else {
        buffered[from].insert(d);
      }
    }
  }

  // cleanup -> check_pending_requests (mod.rs:168-179, 673-678)
  void retry_buffered() {
    auto b = std::move(buffered);
    buffered.clear();
    for (auto &kv : b) {
      std::vector<uint64_t> v(kv.second.begin(), kv.second.end());
      process_requests(kv.first, v.data(), v.size());
    }
  }

  void add_batch(size_t n, const uint64_t *dot, const uint32_t *key_off, const uint64_t *key_id,
                 const uint32_t *dep_off, const uint64_t *dep_dot,
                 const uint64_t *cmd_shards = nullptr, const uint64_t *dep_shards = nullptr) {
    FH_CHECK(n == 0 || (dot && key_off && dep_off), FH_EINVAL, "null argument");
    t_enter = std::chrono::steady_clock::now();
    FH_HIP(hipSetDevice(device));
    // check_pending (mod.rs:558-644) retries only the children of dots that
    // were just executed: a retry with no new vertex where none of the
    // pending set's missing dependencies executed since the last pass
    // changes nothing
    if (n == 0) {
      bool resolved = false;
      if (clock_changed)
        for (uint64_t d : missing_now)
          if (clock.contains(d)) {
            resolved = true;
            break;
          }
      clock_changed = false;
      if (!resolved) {
        skipped++;
        return;
      }
    }
    passes++;
    clock_changed = false;
    // vertices: carried pending (earlier arrivals, already on the device)
    // then the batch (the only upload)
    DSet &W = ds[cur];
    const size_t P = W.P;
    const size_t V = P + n;
    FH_CHECK(V < (size_t(1) << 30), FH_EINVAL, "too many vertices");
    FH_CHECK(P == pend.size(), FH_EINVARIANT, "graph: device / host pending sets disagree");
    const size_t KB = n ? key_off[n] : 0, DB = n ? dep_off[n] : 0;
    FH_CHECK(size_t(W.KP) + KB < (size_t(1) << 32) && size_t(W.DP) + DB < (size_t(1) << 32),
             FH_EINVAL, "too many keys / dependencies");
    for (size_t e = 0; e < KB; e++)
      FH_CHECK(key_id[e] < cfg.key_space, FH_EINVAL, "key id >= key_space");
    if (V == 0) return;
    uint64_t *ddot_v = grow_keep(W.dot, V + 1, P, stream);
    uint32_t *dko = grow_keep(W.koff, V + 2, P + 1, stream);
    uint32_t *dk = grow_keep(W.key32, W.KP + KB + 1, W.KP, stream);
    uint32_t *ddo = grow_keep(W.doff, V + 2, P + 1, stream);
    uint64_t *dd = grow_keep(W.ddot, W.DP + DB + 1, W.DP, stream);
    // executed clock mirror: re-sorted and re-sent only when the clock
    // changed since the last pass
    const bool clk = clock.version != exc_version;
    if (clk) {
      clock.exceptions(exc_sorted);
      d_exc.ensure(exc_sorted.size() + 1);
    }
    // the device mirror is current only once the append that writes it is
    // enqueued (a throw before then leaves exc_version stale: re-sent next
    // pass)
    const uint64_t clk_version = clock.version;
    // one pinned block, one copy, one append launch (separate pageable
    // copies cost several microseconds each: the floor of a small batch)
    Upload u{};
    u.n = uint32_t(n);
    u.nk = uint32_t(KB);
    u.nd = uint32_t(DB);
    u.nf = clk ? 256u : 0u;
    u.ne = clk ? uint32_t(exc_sorted.size()) : 0u;
    if (n || clk) {
      const size_t o_dot = 0, o_dep = o_dot + n * 8, o_clk = o_dep + DB * 8,
                   o_key = o_clk + (size_t(u.nf) + u.ne) * 8, o_ko = o_key + KB * 4,
                   o_do = o_ko + (n + 1) * 4, bytes = o_do + (n + 1) * 4;
      if (h_up_cap < bytes) {
        if (h_up) FH_HIP(hipHostFree(h_up));
        h_up = nullptr;
        h_up_cap = 0;
        FH_HIP(hipHostMalloc(reinterpret_cast<void **>(&h_up), bytes * 2, hipHostMallocMapped));
        FH_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&h_up_dev), h_up, 0));
        h_up_cap = bytes * 2;
      }
      // k_append reads the mapped block itself (no copy operation; the pass
      // ends with a stream synchronize before the block is rewritten)
      uint8_t *dup = h_up_dev;
      if (n) {
        std::memcpy(h_up + o_dot, dot, n * 8);
        if (DB) std::memcpy(h_up + o_dep, dep_dot, DB * 8);
        uint32_t *hk = reinterpret_cast<uint32_t *>(h_up + o_key);
        for (size_t e = 0; e < KB; e++) hk[e] = uint32_t(key_id[e]);
        std::memcpy(h_up + o_ko, key_off, (n + 1) * 4);
        std::memcpy(h_up + o_do, dep_off, (n + 1) * 4);
      }
      if (clk) {
        std::memcpy(h_up + o_clk, clock.frontier, 256 * 8);
        if (u.ne) std::memcpy(h_up + o_clk + 256 * 8, exc_sorted.data(), size_t(u.ne) * 8);
      }
      u.dot = reinterpret_cast<const uint64_t *>(dup + o_dot);
      u.dep = reinterpret_cast<const uint64_t *>(dup + o_dep);
      u.clk = reinterpret_cast<const uint64_t *>(dup + o_clk);
      u.key = reinterpret_cast<const uint32_t *>(dup + o_key);
      u.koff = reinterpret_cast<const uint32_t *>(dup + o_ko);
      u.doff = reinterpret_cast<const uint32_t *>(dup + o_do);
    }
    const std::vector<uint64_t> &exc = exc_sorted;
    uint64_t *dexc = d_exc.ensure(exc.size() + 1);
    const AppendDst adst{ddot_v + P, dko + P, dk + W.KP, ddo + P, dd + W.DP, W.KP, W.DP,
                         d_frontier.get(), dexc};
    // FH_GRAPH_SMALL=0 (tests): every pass through the general path
    static const bool small_on = [] {
      const char *e = getenv("FH_GRAPH_SMALL");
      return !(e && *e == '0');
    }();
    if (small_on && V <= size_t(kSmallV) && size_t(W.DP) + DB <= size_t(kSmallE)) {
      // k_graph_small appends the rows itself
      small_pass(n, dot, dep_off, dep_dot, cmd_shards, dep_shards, V, KB, DB, ddot_v, dko, dk,
                 ddo, dd, dexc, uint32_t(exc.size()), u, adst);
      exc_version = clk_version;
      return;
    }
    const auto t_up = std::chrono::steady_clock::now();
    if (n || clk) {
      k_append<<<grid_for(std::max({u.n ? u.n + 1 : 0u, u.nk, u.nd, u.nf + u.ne}), B), B, 0,
                 stream>>>(u, adst);
      FH_HIP(hipGetLastError());
    }
    exc_version = clk_version;
    // dot -> vid index
    uint64_t *sd = nullptr;
    uint32_t *sv = nullptr;
    sort_pairs<uint64_t, uint32_t>(ddot_v, nullptr, d_sd.ensure(V), d_sv.ensure(V),
                                   d_sd2.ensure(V), d_sv2.ensure(V), V, 64, sort_ws, stream, &sd,
                                   &sv);
    FH_HIP(hipMemsetAsync(d_err.get(), 0, 2 * sizeof(uint32_t), stream));
    k_dup_check<<<grid_for(V, B), B, 0, stream>>>(uint32_t(V), sd, d_err.get());
    uint32_t *cnt = d_cnt.ensure(V + 1);
    uint8_t *b0 = d_blocked0.ensure(V + 1);
    k_resolve_count<<<grid_for(V, B), B, 0, stream>>>(uint32_t(V), ddot_v, ddo, dd, sd, sv,
                                                       d_frontier.get(), dexc,
                                                       uint32_t(exc.size()), cnt, b0);
    uint32_t *off = d_off.ensure(V + 1);
    exclusive_scan_u32(cnt, off, V, scan_ws, stream);
    uint32_t E = 0, dup = 0;
    FH_HIP(hipMemcpyAsync(&E, off + V, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    FH_HIP(hipMemcpyAsync(&dup, d_err.get(), sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    FH_HIP(hipStreamSynchronize(stream));
    // mod.rs:235-240: indexing an already indexed dot panics (state unchanged:
    // the carried prefix is untouched, the appended rows are ignored)
    FH_CHECK(dup == 0, FH_EINVARIANT, "Graph::handle_add tried to index already indexed dot");
    batch_seq0 = next_seq;
    index_requests(n, dot, dep_off, dep_dot, dep_shards);
    batch_seq0 = ~uint64_t(0);
    uint32_t *dst = d_dst.ensure(E + 1);
    k_resolve_fill<<<grid_for(V, B), B, 0, stream>>>(uint32_t(V), ddot_v, ddo, dd, sd, sv,
                                                      d_frontier.get(), dexc,
                                                      uint32_t(exc.size()), off, dst);
    GraphInput gin;
    gin.V = uint32_t(V);
    gin.off = off;
    gin.dst = dst;
    gin.blocked0 = b0;
    gin.dot = ddot_v;
    gin.k = 0;
    gin.key_off = dko;
    gin.key32 = dk;
    gin.key_bits = key_bits;
    gin.want_per_key = false;  // the executor's monitor is fed from the drain order
    GraphOutput out;
    const auto t_run0 = std::chrono::steady_clock::now();
    core.run(gin, out);
    const auto t_run1 = std::chrono::steady_clock::now();
    // which batch vertices stay pending: only those get host metadata (a
    // batch vertex executed in this pass needs none: its execution delay is 0)
    std::vector<uint8_t> bflag(n);
    if (n && out.blocked)
      FH_HIP(hipMemcpyAsync(bflag.data(), out.blocked + P, n, hipMemcpyDeviceToHost, stream));
    // executed vertices to the host: dots and labels in execution order
    const uint32_t nexec = out.nexec;
    std::vector<uint64_t> xdot(nexec), xlab(nexec);
    std::vector<uint8_t> xcar(nexec);
    if (nexec) {
      uint64_t *xd = d_xdot.ensure(nexec), *xl = d_xlab.ensure(nexec);
      uint8_t *xc = d_xcar.ensure(nexec);
      k_gather_exec<<<grid_for(nexec, B), B, 0, stream>>>(nexec, out.exec_order, ddot_v,
                                                           out.scc_label, uint32_t(P), xd, xl, xc);
      FH_HIP(hipMemcpyAsync(xcar.data(), xc, nexec, hipMemcpyDeviceToHost, stream));
      FH_HIP(hipMemcpyAsync(xdot.data(), xd, nexec * sizeof(uint64_t), hipMemcpyDeviceToHost,
                            stream));
      FH_HIP(hipMemcpyAsync(xlab.data(), xl, nexec * sizeof(uint64_t), hipMemcpyDeviceToHost,
                            stream));
    }
    // the missing dependencies of the vertices that stay pending
    const uint32_t P2 = uint32_t(V - nexec);
    uint32_t nmiss = 0;
    uint64_t *miss = nullptr;
    if (P2) {
      const uint32_t mcap = uint32_t(std::min<size_t>(W.DP + DB, size_t(1) << 30));
      miss = d_miss.ensure(mcap + 1);
      k_missing_list<<<grid_for(V, B), B, 0, stream>>>(uint32_t(V), b0, ddot_v, ddo, dd, sd, sv,
                                                        d_frontier.get(), dexc,
                                                        uint32_t(exc.size()), mcap,
                                                        d_err.get() + 1, miss);
      nmiss = fetch_u32(d_err.get() + 1, stream);
      nmiss = std::min(nmiss, mcap);
    }
    std::vector<uint64_t> mlist(nmiss);
    if (nmiss)
      FH_HIP(hipMemcpyAsync(mlist.data(), miss, nmiss * sizeof(uint64_t), hipMemcpyDeviceToHost,
                            stream));
    // the survivors, compacted in arrival order into the other set
    DSet &N = ds[1 - cur];
    if (P2) {
      uint32_t *kv = d_kv.ensure(V), *kk = d_kk.ensure(V), *kd = d_kd.ensure(V);
      uint32_t *pv = d_pv.ensure(V + 1), *pk = d_pk.ensure(V + 1), *pd = d_pd.ensure(V + 1);
      k_keep_counts<<<grid_for(V, B), B, 0, stream>>>(uint32_t(V), out.blocked, dko, ddo, kv, kk,
                                                       kd);
      exclusive_scan_u32(kv, pv, V, scan_ws, stream);
      exclusive_scan_u32(kk, pk, V, scan_ws, stream);
      exclusive_scan_u32(kd, pd, V, scan_ws, stream);
      uint32_t tot[3];
      FH_HIP(hipMemcpyAsync(&tot[0], pv + V, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
      FH_HIP(hipMemcpyAsync(&tot[1], pk + V, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
      FH_HIP(hipMemcpyAsync(&tot[2], pd + V, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
      FH_HIP(hipStreamSynchronize(stream));
      FH_CHECK(tot[0] == P2, FH_EINVARIANT, "graph: pending count disagrees with the pass");
      uint64_t *ndot = N.dot.ensure(P2 + 1), *nddot = N.ddot.ensure(tot[2] + 1);
      uint32_t *nkoff = N.koff.ensure(P2 + 2), *nkey = N.key32.ensure(tot[1] + 1);
      uint32_t *ndoff = N.doff.ensure(P2 + 2);
      k_keep_copy<<<grid_for(V, B), B, 0, stream>>>(uint32_t(V), out.blocked, ddot_v, dko, dk,
                                                     ddo, dd, pv, pk, pd, ndot, nkoff, nkey,
                                                     ndoff, nddot);
      FH_HIP(hipMemcpyAsync(nkoff + P2, &tot[1], sizeof(uint32_t), hipMemcpyHostToDevice, stream));
      FH_HIP(hipMemcpyAsync(ndoff + P2, &tot[2], sizeof(uint32_t), hipMemcpyHostToDevice, stream));
      N.KP = tot[1];
      N.DP = tot[2];
    } else {
      N.koff.ensure(16);
      N.doff.ensure(16);
      FH_HIP(hipMemsetAsync(N.koff.get(), 0, sizeof(uint32_t), stream));
      FH_HIP(hipMemsetAsync(N.doff.get(), 0, sizeof(uint32_t), stream));
      N.KP = N.DP = 0;
    }
    N.P = P2;
    W.P = W.KP = W.DP = 0;
    cur = 1 - cur;
    FH_HIP(hipStreamSynchronize(stream));
    const auto t_res = std::chrono::steady_clock::now();
    finish_pass(n, dot, dep_off, dep_dot, cmd_shards, dep_shards, xdot, xlab, bflag, mlist, P2,
                xcar.data());
    static const bool debug = getenv("FH_GRAPH_DEBUG") != nullptr;
    if (debug) {
      const auto t_end = std::chrono::steady_clock::now();
      auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      fprintf(stderr,
              "fh graph pass (us): n=%zu V=%zu upload %.0f index %.0f run %.0f results %.0f "
              "host %.0f\n",
              n, V, us(t_enter, t_up), us(t_up, t_run0), us(t_run0, t_run1), us(t_run1, t_res),
              us(t_res, t_end));
    }
  }

  // A small graph's pass (graph_small.hip): one launch, one read-back.
  uint8_t *h_small = nullptr;      // the pass's results: mapped pinned host memory
  uint8_t *h_small_dev = nullptr;  // its device address (k_graph_small writes it)
  size_t h_small_cap = 0;
  void small_pass(size_t n, const uint64_t *dot, const uint32_t *dep_off, const uint64_t *dep_dot,
                  const uint64_t *cmd_shards, const uint64_t *dep_shards, size_t V, size_t KB,
                  size_t DB, const uint64_t *ddot_v, const uint32_t *dko, const uint32_t *dk,
                  const uint32_t *ddo, const uint64_t *dd, const uint64_t *dexc, uint32_t nexc,
                  const Upload &up, const AppendDst &adst) {
    DSet &W = ds[cur];
    DSet &N = ds[1 - cur];
    // the next set holds at most every current vertex, key and dependency
    const size_t KT = size_t(W.KP) + KB, DT = size_t(W.DP) + DB;
    uint64_t *ndot = grow_keep(N.dot, V + 1, 0, stream);
    uint32_t *nkoff = grow_keep(N.koff, V + 2, 0, stream);
    uint32_t *nkey = grow_keep(N.key32, KT + 1, 0, stream);
    uint32_t *ndoff = grow_keep(N.doff, V + 2, 0, stream);
    uint64_t *nddot = grow_keep(N.ddot, DT + 1, 0, stream);
    // read-back block: header, executed dots, labels, missing dots, pending
    // flags, carried flags of the executed
    const size_t hdr = 128, bytes = hdr + V * 16 + DT * 8 + 2 * V;  // header: 32 words

    if (h_small_cap < bytes) {
      if (h_small) FH_HIP(hipHostFree(h_small));
      h_small = nullptr;
      h_small_cap = 0;
      FH_HIP(hipHostMalloc(reinterpret_cast<void **>(&h_small), bytes * 2, hipHostMallocMapped));
      FH_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&h_small_dev), h_small, 0));
      h_small_cap = bytes * 2;
    }
    SmallPass sp;
    sp.up = up;
    sp.dst = adst;
    sp.V = uint32_t(V);
    sp.P = uint32_t(V - n);
    sp.dot = ddot_v;
    sp.koff = dko;
    sp.key32 = dk;
    sp.doff = ddo;
    sp.ddot = dd;
    sp.frontier = d_frontier.get();
    sp.exc = dexc;
    sp.nexc = nexc;
    uint8_t *blk = h_small_dev;
    sp.header = reinterpret_cast<uint32_t *>(blk);
    sp.xdot = reinterpret_cast<uint64_t *>(blk + hdr);
    sp.xlab = sp.xdot + V;
    sp.miss = sp.xlab + V;
    sp.miss_cap = uint32_t(DT);
    sp.blocked = reinterpret_cast<uint8_t *>(sp.miss + DT);
    sp.xcar = sp.blocked + V;
    sp.ndot = ndot;
    sp.nkoff = nkoff;
    sp.nkey32 = nkey;
    sp.ndoff = ndoff;
    sp.nddot = nddot;
    static const bool debug = getenv("FH_GRAPH_DEBUG") != nullptr;
    sp.stamps = debug ? 1 : 0;
    // 0 is the value the host stores before the launch: never a sequence
    if (++small_seq == 0) small_seq = 1;
    sp.seq = small_seq;
    sp.delay_us = small_delay_us;
    volatile uint32_t *done = reinterpret_cast<volatile uint32_t *>(h_small) + 31;
    *done = 0;
    const auto t_launch = std::chrono::steady_clock::now();
    launch_graph_small(sp, stream);  // writes the mapped block: no read-back copy
    // the kernel's last store is the completion word (polled: ~4 us sooner
    // than a stream synchronize at a batch of one); the stream is queried now
    // and then so that a failed launch cannot spin forever, and a pass that
    // has not finished by the deadline fails the call instead of hanging it
    try {
      poll_completion(done, sp.seq, [&] { return hipStreamQuery(stream); }, small_deadline_ms);
    } catch (...) {
      broken = true;
      throw;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    const auto t_sync = std::chrono::steady_clock::now();
    const uint32_t *hh = reinterpret_cast<const uint32_t *>(h_small);
    const uint32_t nexec = hh[0], nmiss = std::min<uint32_t>(hh[1], uint32_t(DT));
    if (debug) {
      auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      fprintf(stderr, "fh graph_small host (us): upload %.1f launch+wait %.1f\n",
              us(t_enter, t_launch), us(t_launch, t_sync));
      auto at = [&](int i) { return (uint64_t(hh[9 + 2 * i]) << 32) | hh[8 + 2 * i]; };
      fprintf(stderr, "fh graph_small V=%zu phases (us): append %.1f index %.1f resolve %.1f blocked %.1f "
              "H %.1f rounds %.1f depth %.1f order %.1f survivors %.1f\n", V,
              (at(9) - at(0)) * 0.01, (at(1) - at(9)) * 0.01, (at(2) - at(1)) * 0.01, (at(3) - at(2)) * 0.01,
              (at(4) - at(3)) * 0.01, (at(5) - at(4)) * 0.01, (at(6) - at(5)) * 0.01,
              (at(7) - at(6)) * 0.01, (at(8) - at(7)) * 0.01);
    }
    // mod.rs:235-240 (state unchanged: the next set is not taken, the
    // appended rows are ignored)
    FH_CHECK(hh[2] == 0, FH_EINVARIANT, "Graph::handle_add tried to index already indexed dot");
    batch_seq0 = next_seq;
    index_requests(n, dot, dep_off, dep_dot, dep_shards);
    batch_seq0 = ~uint64_t(0);
    const uint64_t *hx = reinterpret_cast<const uint64_t *>(h_small + hdr);
    std::vector<uint64_t> xdot(hx, hx + nexec), xlab(hx + V, hx + V + nexec);
    std::vector<uint64_t> mlist(hx + 2 * V, hx + 2 * V + nmiss);
    const uint8_t *hb = reinterpret_cast<const uint8_t *>(hx + 2 * V + DT);
    std::vector<uint8_t> bflag(hb + (V - n), hb + V);
    const uint32_t P2 = hh[3];
    FH_CHECK(P2 == V - nexec, FH_EINVARIANT, "graph: small pass counts");
    N.P = P2;
    N.KP = hh[4];
    N.DP = hh[5];
    W.P = W.KP = W.DP = 0;
    cur = 1 - cur;
    passes_small++;
    finish_pass(n, dot, dep_off, dep_dot, cmd_shards, dep_shards, xdot, xlab, bflag, mlist, P2,
                hb + V);
    if (debug)
      fprintf(stderr, "fh graph_small host (us): results %.1f\n",
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_sync)
                  .count());
  }
  std::chrono::steady_clock::time_point t_enter;  // add_batch entry (FH_GRAPH_DEBUG timings)
  uint32_t small_seq = 0;
  uint64_t passes_small = 0;
  // a small pass missed its deadline: its kernel may still be writing the
  // vertex sets, so every later call fails (FH_EHIP) until the handle is
  // destroyed (fh_graph_inject_small_delay sets both knobs in tests)
  bool broken = false;
  double small_deadline_ms = 30000.0;
  uint32_t small_delay_us = 0;

  // The host side of a pass: the drained vertices, executed clock, metrics,
  // the survivors' pending metadata and the missing dependencies.
  void finish_pass(size_t n, const uint64_t *dot, const uint32_t *dep_off, const uint64_t *dep_dot,
                   const uint64_t *cmd_shards, const uint64_t *dep_shards,
                   const std::vector<uint64_t> &xdot, const std::vector<uint64_t> &xlab,
                   const std::vector<uint8_t> &bflag, std::vector<uint64_t> &mlist, uint32_t P2,
                   const uint8_t *xcar = nullptr) {
    // xcar: per executed vertex, carried or not -- only the carried ones have
    // host metadata to look up (a hash lookup per executed vertex cost ~60
    // ns: most of a 1M-command batch's host time)
    const size_t nexec = xdot.size();
    // every drained dot is a carried vertex or one of this batch's executed
    // vertices (the reference panics otherwise): the batch part is checked by
    // count and by a sum of mixed dots over both sides (O(n), no set)
    auto mix = [](uint64_t x) {
      x ^= x >> 33;
      x *= 0xff51afd7ed558ccdull;
      x ^= x >> 33;
      x *= 0xc4ceb9fe1a85ec53ull;
      return x ^ (x >> 33);
    };
    uint64_t want_n = 0, want_h = 0, got_n = 0, got_h = 0;
    for (size_t i = 0; i < n; i++)
      if (!bflag[i]) {
        want_n++;
        want_h += mix(dot[i]);
      }
    for (uint32_t j = 0; j < nexec; j++) {
      const uint64_t d = xdot[j];
      ready.emplace_back(d, xlab[j]);
      // metrics: one ChainSize per SCC (members are contiguous in the
      // execution order), one ExecutionDelay per command
      if (j == 0 || xlab[j - 1] != xlab[j]) m_chain.push_back(0);
      m_chain.back()++;
      auto it = (!xcar || xcar[j]) ? pend.find(d) : pend.end();
      if (it != pend.end()) {  // a carried vertex
        m_delay.push_back(now_ms >= it->second.time ? now_ms - it->second.time : 0);
        porder.erase(it->second.seq);
        pend.erase(it);
      } else {  // a vertex of this batch (stamped now)
        m_delay.push_back(0);
        got_n++;
        got_h += mix(d);
      }
    }
    FH_CHECK(got_n == want_n && got_h == want_h, FH_EINVARIANT,
             "graph: an executed dot was neither a pending vertex nor one of the batch");
    clock.add_all(xdot.data(), nexec);  // executed clock update (tarjan.rs:296)
    // the batch's survivors join the host's pending metadata, in arrival
    // order (after the pass: a failed pass leaves host and device sets equal)
    for (size_t i = 0; i < n; i++) {
      if (!bflag[i]) continue;
      PInfo pi;
      pi.seq = next_seq++;
      pi.cshard = cmd_shards ? cmd_shards[i] : 0;
      pi.time = now_ms;
      pi.deps.assign(dep_dot + dep_off[i], dep_dot + dep_off[i + 1]);
      pi.dshards.resize(pi.deps.size(), 0);
      if (dep_shards)
        std::copy(dep_shards + dep_off[i], dep_shards + dep_off[i + 1], pi.dshards.begin());
      porder.emplace(pi.seq, dot[i]);
      pend.emplace(dot[i], std::move(pi));
    }
    FH_CHECK(pend.size() == P2, FH_EINVARIANT, "graph: host pending set disagrees with the pass");
    std::sort(mlist.begin(), mlist.end());
    mlist.erase(std::unique(mlist.begin(), mlist.end()), mlist.end());
    missing_now.swap(mlist);
    // PendingIndex entries go once their parent dot is indexed or executed
    // (index.rs remove, called from check_pending)
    for (auto it = requested.begin(); it != requested.end();) {
      if (clock.contains(*it) || pend.count(*it))
        it = requested.erase(it);
      else
        ++it;
    }
  }

  // VertexIndex::monitor_pending (index.rs:53-103): pending vertices older
  // than threshold_ms, longest pending first, with each one's missing
  // dependencies found through other pending vertices
  // (missing_dependencies, index.rs:105-142); a pending vertex without any
  // is a liveness bug: FH_EINVARIANT, where the reference panics.
  void monitor_pending(uint64_t threshold_ms, std::vector<std::pair<uint64_t, uint64_t>> &old_out,
                       std::vector<uint64_t> &nmissing) {
    std::vector<std::pair<uint64_t, uint64_t>> idx;  // (time, dot), arrival order
    for (const auto &so : porder) {
      const PInfo &pi = pend.at(so.second);
      if (now_ms >= pi.time && now_ms - pi.time >= threshold_ms) idx.emplace_back(pi.time, so.second);
    }
    std::stable_sort(idx.begin(), idx.end(),
                     [](const auto &a, const auto &b) { return a.first < b.first; });
    std::vector<uint64_t> stuck;
    for (const auto &tv : idx) {
      const uint64_t v = tv.second;
      std::unordered_set<uint64_t> visited, missing;
      std::vector<uint64_t> stack{v};
      visited.insert(v);
      while (!stack.empty()) {
        const uint64_t x = stack.back();
        stack.pop_back();
        for (uint64_t d : pend.at(x).deps) {
          if (d == x || clock.contains(d)) continue;
          if (!pend.count(d))
            missing.insert(d);
          else if (visited.insert(d).second)
            stack.push_back(d);
        }
      }
      if (missing.empty()) stuck.push_back(v);
      old_out.emplace_back(v, now_ms - tv.first);
      nmissing.push_back(missing.size());
    }
    if (!stuck.empty()) {
      std::string m = "monitor_pending: commands pending without missing dependencies:";
      for (uint64_t d : stuck) m += " (" + std::to_string(d >> 56) + "," +
                                   std::to_string(d & 0x00FFFFFFFFFFFFFFull) + ")";
      throw Error(FH_EINVARIANT, m);
    }
  }

  size_t drain(uint64_t *dots, uint64_t *labels, size_t cap) {
    size_t c = 0;
    while (!ready.empty() && c < cap) {
      if (dots) dots[c] = ready.front().first;
      if (labels) labels[c] = ready.front().second;
      ready.pop_front();
      c++;
    }
    return c;
  }
};

}  // namespace fh

struct fh_graph {
  fh::GraphDevice dev;
  fh_graph(uint32_t p, uint64_t s, const fh_config &c) : dev(p, s, c) {}
};

extern "C" {

fh_status fh_graph_create(uint32_t process_id, uint64_t shard_id, const fh_config *cfg,
                          fh_graph **out) {
  FH_API_BEGIN
  FH_CHECK(cfg && out, FH_EINVAL, "null argument");
  *out = new fh_graph(process_id, shard_id, *cfg);
  FH_API_END
}

fh_status fh_graph_destroy(fh_graph *h) {
  FH_API_BEGIN
  delete h;
  FH_API_END
}

fh_status fh_graph_add_batch(fh_graph *h, size_t n, const uint64_t *dot, const uint32_t *key_off,
                             const uint64_t *key_id, const uint32_t *dep_off,
                             const uint64_t *dep_dot) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  h->dev.add_batch(n, dot, key_off, key_id, dep_off, dep_dot);
  FH_API_END
}

fh_status fh_graph_add_batch_sharded(fh_graph *h, size_t n, const uint64_t *dot,
                                     const uint32_t *key_off, const uint64_t *key_id,
                                     const uint32_t *dep_off, const uint64_t *dep_dot,
                                     const uint64_t *cmd_shards, const uint64_t *dep_shards) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  FH_CHECK(h->dev.shard_id < 64, FH_EINVAL, "shard sets are 64-bit masks: shard_id must be < 64");
  h->dev.add_batch(n, dot, key_off, key_id, dep_off, dep_dot, cmd_shards, dep_shards);
  FH_API_END
}

fh_status fh_graph_requests(fh_graph *h, uint64_t *dot, uint64_t *shard, size_t cap,
                            size_t *len) {
  FH_API_BEGIN
  FH_CHECK(h && len, FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  auto &r = h->dev.out_requests;
  *len = r.size();
  if (r.empty()) return FH_OK;
  FH_CHECK(dot && shard && cap >= r.size(), FH_ECAP, "request output capacity too small");
  size_t i = 0;
  for (const auto &p : r) {
    shard[i] = p.first;
    dot[i] = p.second;
    i++;
  }
  r.clear();
  FH_API_END
}

fh_status fh_graph_handle_requests(fh_graph *h, uint64_t from_shard, size_t n,
                                   const uint64_t *dots) {
  FH_API_BEGIN
  FH_CHECK(h && (n == 0 || dots), FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  h->dev.process_requests(from_shard, dots, n);
  FH_API_END
}

fh_status fh_graph_cleanup(fh_graph *h) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  h->dev.retry_buffered();
  FH_API_END
}

fh_status fh_graph_request_replies(fh_graph *h, size_t cap, uint64_t *to_shard, uint8_t *kind,
                                   uint64_t *dot, uint64_t *cmd_shards, uint32_t *dep_off,
                                   size_t dep_cap, uint64_t *dep_dot, uint64_t *dep_shards,
                                   size_t *n_replies, size_t *n_deps) {
  FH_API_BEGIN
  FH_CHECK(h && n_replies && n_deps, FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  auto &rs = h->dev.replies;
  size_t nd = 0;
  for (const auto &r : rs) nd += r.deps.size();
  *n_replies = rs.size();
  *n_deps = nd;
  if (rs.empty()) return FH_OK;
  FH_CHECK(cap >= rs.size() && dep_cap >= nd && to_shard && kind && dot && cmd_shards && dep_off &&
               (nd == 0 || (dep_dot && dep_shards)),
           FH_ECAP, "reply output capacity too small");
  size_t e = 0;
  dep_off[0] = 0;
  for (size_t i = 0; i < rs.size(); i++) {
    const auto &r = rs[i];
    to_shard[i] = r.to;
    kind[i] = r.kind;
    dot[i] = r.dot;
    cmd_shards[i] = r.cshard;
    for (size_t j = 0; j < r.deps.size(); j++, e++) {
      dep_dot[e] = r.deps[j];
      dep_shards[e] = r.dshards[j];
    }
    dep_off[i + 1] = uint32_t(e);
  }
  rs.clear();
  FH_API_END
}

fh_status fh_graph_drain(fh_graph *h, uint64_t *exec_dot, uint64_t *scc_label, size_t cap,
                         size_t *len) {
  FH_API_BEGIN
  FH_CHECK(h && len, FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  *len = h->dev.drain(exec_dot, scc_label, exec_dot || scc_label ? cap : 0);
  FH_API_END
}

fh_status fh_graph_mark_executed(fh_graph *h, size_t n, const uint64_t *dot) {
  FH_API_BEGIN
  FH_CHECK(h && (n == 0 || dot), FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  for (size_t i = 0; i < n; i++) h->dev.clock_changed |= h->dev.clock.add(dot[i]);
  FH_API_END
}

// Raise source's contiguous frontier to seq (never lowers it): exceptions at
// or below it go, and exceptions right above it fold in, as AEClock::add does.
fh_status fh_graph_set_executed_frontier(fh_graph *h, uint32_t source, uint64_t seq) {
  FH_API_BEGIN
  FH_CHECK(h && source < 256, FH_EINVAL, "bad argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  auto &c = h->dev.clock;
  FH_CHECK(seq >= c.frontier[source], FH_EINVAL,
           "set_executed_frontier: the executed frontier cannot move backwards");
  if (seq == c.frontier[source]) return FH_OK;
  c.raise_frontier(source, seq);
  h->dev.clock_changed = true;
  FH_API_END
}

fh_status fh_graph_set_time(fh_graph *h, uint64_t now_ms) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  h->dev.now_ms = now_ms;
  FH_API_END
}

fh_status fh_graph_monitor_pending(fh_graph *h, uint64_t threshold_ms, uint64_t *dots,
                                   uint64_t *pending_ms, uint64_t *missing, size_t cap,
                                   size_t *len) {
  FH_API_BEGIN
  FH_CHECK(h && len, FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  std::vector<std::pair<uint64_t, uint64_t>> old;
  std::vector<uint64_t> nm;
  h->dev.monitor_pending(threshold_ms, old, nm);
  *len = old.size();
  for (size_t i = 0; i < old.size() && i < cap; i++) {
    if (dots) dots[i] = old[i].first;
    if (pending_ms) pending_ms[i] = old[i].second;
    if (missing) missing[i] = nm[i];
  }
  FH_API_END
}

fh_status fh_graph_take_metrics(fh_graph *h, uint64_t *chain_size, size_t chain_cap,
                                uint64_t *exec_delay, size_t delay_cap, size_t *n_chain,
                                size_t *n_delay) {
  FH_API_BEGIN
  FH_CHECK(h && n_chain && n_delay, FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  auto &d = h->dev;
  *n_chain = d.m_chain.size();
  *n_delay = d.m_delay.size();
  FH_CHECK((d.m_chain.empty() || (chain_size && chain_cap >= d.m_chain.size())) &&
               (d.m_delay.empty() || (exec_delay && delay_cap >= d.m_delay.size())),
           FH_ECAP, "metrics output capacity too small");
  std::copy(d.m_chain.begin(), d.m_chain.end(), chain_size);
  std::copy(d.m_delay.begin(), d.m_delay.end(), exec_delay);
  d.m_chain.clear();
  d.m_delay.clear();
  FH_API_END
}

fh_status fh_graph_passes(fh_graph *h, uint64_t *passes, uint64_t *skipped) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  if (passes) *passes = h->dev.passes;
  if (skipped) *skipped = h->dev.skipped;
  FH_API_END
}

fh_status fh_graph_inject_small_delay(fh_graph *h, uint32_t delay_us, uint32_t deadline_ms) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_CHECK(delay_us <= 10u * 1000 * 1000, FH_EINVAL, "delay_us <= 10 s");
  h->dev.small_delay_us = delay_us;
  if (deadline_ms) h->dev.small_deadline_ms = double(deadline_ms);
  FH_API_END
}

fh_status fh_selftest_poll_deadline(uint32_t deadline_ms) {
  FH_API_BEGIN
  FH_CHECK(deadline_ms >= 1 && deadline_ms <= 60000, FH_EINVAL, "deadline_ms in [1, 60000]");
  volatile uint32_t word = 0;
  fh::poll_completion(&word, 1u, [] { return hipErrorNotReady; }, double(deadline_ms));
  FH_API_END
}

fh_status fh_graph_pending(fh_graph *h, size_t *count) {
  FH_API_BEGIN
  FH_CHECK(h && count, FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  *count = h->dev.pend.size();
  FH_API_END
}

fh_status fh_graph_missing(fh_graph *h, uint64_t *dots, size_t cap, size_t *len) {
  FH_API_BEGIN
  FH_CHECK(h && len, FH_EINVAL, "null argument");
  FH_CHECK(!h->dev.broken, FH_EHIP, "graph: an earlier small pass missed its deadline");
  const auto &m = h->dev.missing_now;
  *len = m.size();
  for (size_t i = 0; i < m.size() && i < cap && dots; i++) dots[i] = m[i];
  FH_API_END
}

}  // extern "C"

extern "C" {

fh_status fh_execlog_replay(const fh_execlog *h, fh_graph *g, size_t batch, size_t *executed) {
  FH_API_BEGIN
  FH_CHECK(h && g, FH_EINVAL, "null argument");
  FH_CHECK(g->dev.shard_id < 64, FH_EINVAL, "shard sets are 64-bit masks: shard_id must be < 64");
  const fh::ExecLog &L = fh::execlog_of(h);
  auto &dev = g->dev;
  const size_t ready0 = dev.ready.size();
  const size_t E = L.kind.size();
  const size_t cap = batch ? batch : E + 1;
  std::vector<uint32_t> koff, doff;
  size_t i = 0;
  while (i < E) {
    const uint8_t k = L.kind[i];
    if (k == FH_LOG_ADD || k == FH_LOG_REPLY_INFO) {
      // a run of adds: event arrays are already CSR; rebase the offsets
      size_t j = i;
      while (j < E && j - i < cap && (L.kind[j] == FH_LOG_ADD || L.kind[j] == FH_LOG_REPLY_INFO))
        j++;
      koff.assign(L.key_off.begin() + i, L.key_off.begin() + j + 1);
      doff.assign(L.dep_off.begin() + i, L.dep_off.begin() + j + 1);
      for (auto &o : koff) o -= L.key_off[i];
      for (auto &o : doff) o -= L.dep_off[i];
      dev.add_batch(j - i, L.dot.data() + i, koff.data(), L.key_id.data() + L.key_off[i],
                    doff.data(), L.dep_dot.data() + L.dep_off[i], L.shards.data() + i,
                    L.dep_shards.data() + L.dep_off[i]);
      i = j;
    } else if (k == FH_LOG_REQUEST) {
      dev.process_requests(L.shards[i], L.dep_dot.data() + L.dep_off[i],
                           L.dep_off[i + 1] - L.dep_off[i]);
      i++;
    } else if (k == FH_LOG_REPLY_EXECUTED) {
      size_t j = i;
      while (j < E && L.kind[j] == FH_LOG_REPLY_EXECUTED) dev.clock_changed |= dev.clock.add(L.dot[j++]);
      dev.add_batch(0, nullptr, nullptr, nullptr, nullptr, nullptr);  // pending retry
      i = j;
    } else {
      i++;  // Executed: handle_executed on the shared clock is a no-op here
    }
  }
  if (executed) *executed = dev.ready.size() - ready0;
  FH_API_END
}

}  // extern "C"
