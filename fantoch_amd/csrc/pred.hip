// pred.hip -- Caesar's PredecessorsExecutor drop-in (fh_pred_*).
//
// PredecessorsGraph semantics (fantoch_ps/src/executor/pred/mod.rs:26-352)
// for batches of PredecessorsExecutionInfo (executor.rs): a command executes
// once (phase one, :132-182) every dependency is committed and (phase two,
// :186-253) every dependency with a lower clock has executed; a command never
// depends on itself (:106-109).  Batch restatement: vertices = carried
// pending commands (earlier arrivals) + the batch.  A dependency is
//   executed                          -> ignored,
//   a vertex with a lower clock       -> an edge (phase-two wait),
//   a vertex with a higher clock      -> nothing (committed is enough),
//   neither (not committed yet)       -> the command is blocked (phase one).
// A command stays pending iff it reaches a blocked command through
// lower-clock edges (a fixpoint on the device); the others execute, drained
// in clock order -- a linearisation of every phase-two wait.  Caesar reports
// every conflicting command with a lower clock as a dependency
// (KeyClocks::predecessors, protocol/common/pred/clocks/keys/sequential.rs:
// 74-119), so every key's execution sequence is its commands in clock order,
// the order the reference's cascade produces.
//
// Clocks are packed (seq << 8) | process_id (Clock's derived Ord,
// protocol/common/pred/clocks/mod.rs:15-30).
#include <algorithm>
#include <deque>
#include <vector>

#include "dotindex.h"
#include "scan.h"
#include "sort.h"

namespace fh {
namespace {

constexpr unsigned kB = 256;
#define PRED_STRIDE(i, n) \
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += gridDim.x * blockDim.x)

// per vertex: lower-clock edges, and whether a dependency is uncommitted
__global__ void k_pred_count(uint32_t V, const uint64_t *__restrict__ dot,
                             const uint64_t *__restrict__ clk, const uint32_t *__restrict__ doff,
                             const uint64_t *__restrict__ ddot, const uint64_t *__restrict__ sd,
                             const uint32_t *__restrict__ sv, const uint64_t *__restrict__ frontier,
                             const uint64_t *__restrict__ exc, uint32_t nexc,
                             uint32_t *__restrict__ cnt, uint8_t *__restrict__ blocked0) {
  PRED_STRIDE(v, V) {
    uint32_t c = 0;
    bool uncommitted = false;
    const uint64_t self = dot[v], cv = clk[v];
    for (uint32_t e = doff[v]; e < doff[v + 1]; e++) {
      const uint64_t d = ddot[e];
      if (d == self || executed_dev(d, frontier, exc, nexc)) continue;
      const int64_t u = find_vid(d, sd, sv, V);
      if (u < 0)
        uncommitted = true;
      else if (clk[u] < cv)
        c++;
    }
    cnt[v] = c;
    blocked0[v] = uncommitted;
  }
}

__global__ void k_pred_fill(uint32_t V, const uint64_t *__restrict__ dot,
                            const uint64_t *__restrict__ clk, const uint32_t *__restrict__ doff,
                            const uint64_t *__restrict__ ddot, const uint64_t *__restrict__ sd,
                            const uint32_t *__restrict__ sv, const uint64_t *__restrict__ frontier,
                            const uint64_t *__restrict__ exc, uint32_t nexc,
                            const uint32_t *__restrict__ off, uint32_t *__restrict__ dst) {
  PRED_STRIDE(v, V) {
    uint32_t o = off[v];
    const uint64_t self = dot[v], cv = clk[v];
    for (uint32_t e = doff[v]; e < doff[v + 1]; e++) {
      const uint64_t d = ddot[e];
      if (d == self || executed_dev(d, frontier, exc, nexc)) continue;
      const int64_t u = find_vid(d, sd, sv, V);
      if (u >= 0 && clk[u] < cv) dst[o++] = uint32_t(u);
    }
  }
}

// one round of "blocked if a lower-clock dependency is blocked"
__global__ void k_pred_blocked_iter(uint32_t V, const uint32_t *__restrict__ off,
                                    const uint32_t *__restrict__ dst, uint8_t *blocked,
                                    uint32_t *changed) {
  PRED_STRIDE(v, V) {
    if (blocked[v]) continue;
    for (uint32_t e = off[v]; e < off[v + 1]; e++) {
      if (__hip_atomic_load(&blocked[dst[e]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        blocked[v] = 1;
        *changed = 1;
        break;
      }
    }
  }
}

__global__ void k_pred_ready_flags(uint32_t V, const uint8_t *__restrict__ blocked,
                                   uint32_t *__restrict__ f) {
  PRED_STRIDE(v, V) f[v] = blocked[v] ? 0u : 1u;
}

// executable vertices (clock, vid), compacted in vid order
__global__ void k_pred_compact(uint32_t V, const uint8_t *__restrict__ blocked,
                               const uint32_t *__restrict__ pos, const uint64_t *__restrict__ clk,
                               uint64_t *__restrict__ kc, uint32_t *__restrict__ kv) {
  PRED_STRIDE(v, V) {
    if (blocked[v]) continue;
    kc[pos[v]] = clk[v];
    kv[pos[v]] = v;
  }
}

}  // namespace

struct PredDevice {
  uint32_t process_id;
  fh_config cfg;
  int device = 0;
  hipStream_t stream = nullptr;
  AEClock committed, executed;  // mod.rs:29-30
  // carried pending commands (arrival order)
  std::vector<uint64_t> p_dot, p_clk, p_deps;
  std::vector<uint32_t> p_doff{0};
  std::deque<uint64_t> ready;  // to_execute (mod.rs:37)
  DBuf<uint64_t> d_dot, d_clk, d_ddot, d_sd, d_sd2, d_frontier, d_exc, d_kc, d_kc2, d_kco;
  DBuf<uint32_t> d_doff, d_cnt, d_off, d_dst, d_sv, d_sv2, d_err, d_chg, d_f, d_pos, d_kv, d_kv2,
      d_kv3;
  DBuf<uint8_t> d_blocked;
  SortWorkspace sort_ws;
  ScanWorkspace scan_ws;

  PredDevice(uint32_t pid, uint64_t sid, const fh_config &c) : process_id(pid), cfg(c) {
    device = pick_device(&c, sid);
    FH_HIP(hipSetDevice(device));
    FH_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    d_err.ensure(4);
    d_chg.ensure(4);
    d_frontier.ensure(256);
  }
  ~PredDevice() {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
  }

  uint32_t read_u32(const uint32_t *p) { return fetch_u32(p, stream); }

  void add_batch(size_t n, const uint64_t *dot, const uint64_t *clock, const uint32_t *dep_off,
                 const uint64_t *dep_dot) {
    FH_CHECK(n == 0 || (dot && clock && dep_off), FH_EINVAL, "null argument");
    FH_HIP(hipSetDevice(device));
    // index_committed_command (mod.rs:263-273): a dot is committed once
    for (size_t i = 0; i < n; i++)
      FH_CHECK(!committed.contains(dot[i]), FH_EINVARIANT,
               "Predecessors::index tried to index already indexed dot");
    const size_t P = p_dot.size(), V = P + n;
    FH_CHECK(V < (size_t(1) << 30), FH_EINVAL, "too many vertices");
    if (V == 0) return;
    std::vector<uint64_t> vdot(p_dot), vclk(p_clk), deps(p_deps);
    std::vector<uint32_t> doff(p_doff);
    vdot.insert(vdot.end(), dot, dot + n);
    vclk.insert(vclk.end(), clock, clock + n);
    for (size_t i = 0; i < n; i++) {
      deps.insert(deps.end(), dep_dot + dep_off[i], dep_dot + dep_off[i + 1]);
      doff.push_back(uint32_t(deps.size()));
    }
    // executed set mirror
    std::vector<uint64_t> exc;
    executed.exceptions(exc);
    FH_HIP(hipMemcpyAsync(d_frontier.get(), executed.frontier, sizeof(executed.frontier),
                          hipMemcpyHostToDevice, stream));
    uint64_t *dexc = d_exc.ensure(exc.size() + 1);
    if (!exc.empty())
      FH_HIP(hipMemcpyAsync(dexc, exc.data(), exc.size() * sizeof(uint64_t),
                            hipMemcpyHostToDevice, stream));
    uint64_t *ddot_v = d_dot.ensure(V), *dclk = d_clk.ensure(V);
    FH_HIP(hipMemcpyAsync(ddot_v, vdot.data(), V * 8, hipMemcpyHostToDevice, stream));
    FH_HIP(hipMemcpyAsync(dclk, vclk.data(), V * 8, hipMemcpyHostToDevice, stream));
    uint32_t *ddo = d_doff.ensure(V + 1);
    FH_HIP(hipMemcpyAsync(ddo, doff.data(), (V + 1) * 4, hipMemcpyHostToDevice, stream));
    uint64_t *dd = d_ddot.ensure(deps.size() + 1);
    if (!deps.empty())
      FH_HIP(hipMemcpyAsync(dd, deps.data(), deps.size() * 8, hipMemcpyHostToDevice, stream));
    // dot -> vid
    uint64_t *sd = nullptr;
    uint32_t *sv = nullptr;
    sort_pairs<uint64_t, uint32_t>(ddot_v, nullptr, d_sd.ensure(V), d_sv.ensure(V), d_sd2.ensure(V),
                         d_sv2.ensure(V), V, 64, sort_ws, stream, &sd, &sv);
    FH_HIP(hipMemsetAsync(d_err.get(), 0, sizeof(uint32_t), stream));
    k_dup_check<<<grid_for(V, kB), kB, 0, stream>>>(uint32_t(V), sd, d_err.get());
    FH_CHECK(read_u32(d_err.get()) == 0, FH_EINVARIANT,
             "Predecessors::index tried to index already indexed dot");
    for (size_t i = 0; i < n; i++) committed.add(dot[i]);
    // lower-clock edges, phase-one blocks
    uint32_t *cnt = d_cnt.ensure(V + 1);
    uint8_t *blocked = d_blocked.ensure(V + 1);
    k_pred_count<<<grid_for(V, kB), kB, 0, stream>>>(uint32_t(V), ddot_v, dclk, ddo, dd, sd, sv,
                                                      d_frontier.get(), dexc,
                                                      uint32_t(exc.size()), cnt, blocked);
    uint32_t *off = d_off.ensure(V + 1);
    exclusive_scan_u32(cnt, off, V, scan_ws, stream);
    const uint32_t E = read_u32(off + V);
    uint32_t *dst = d_dst.ensure(E + 1);
    k_pred_fill<<<grid_for(V, kB), kB, 0, stream>>>(uint32_t(V), ddot_v, dclk, ddo, dd, sd, sv,
                                                     d_frontier.get(), dexc, uint32_t(exc.size()),
                                                     off, dst);
    // phase two: blocked through lower-clock edges (a DAG: clocks decrease)
    for (;;) {
      FH_HIP(hipMemsetAsync(d_chg.get(), 0, sizeof(uint32_t), stream));
      k_pred_blocked_iter<<<grid_for(V, kB), kB, 0, stream>>>(uint32_t(V), off, dst, blocked,
                                                               d_chg.get());
      if (!read_u32(d_chg.get())) break;
    }
    // executable commands in clock order
    uint32_t *f = d_f.ensure(V + 1), *pos = d_pos.ensure(V + 1);
    k_pred_ready_flags<<<grid_for(V, kB), kB, 0, stream>>>(uint32_t(V), blocked, f);
    exclusive_scan_u32(f, pos, V, scan_ws, stream);
    const uint32_t X = read_u32(pos + V);
    std::vector<uint32_t> order(X);
    std::vector<uint8_t> hblocked(V);
    if (X) {
      uint64_t *kc = d_kc.ensure(X), *kco = nullptr;
      uint32_t *kv = d_kv.ensure(X), *kvo = nullptr;
      k_pred_compact<<<grid_for(V, kB), kB, 0, stream>>>(uint32_t(V), blocked, pos, dclk, kc, kv);
      sort_pairs<uint64_t, uint32_t>(kc, kv, d_kco.ensure(X), d_kv2.ensure(X), d_kc2.ensure(X),
                           d_kv3.ensure(X), X, 64, sort_ws, stream, &kco, &kvo);
      FH_HIP(hipMemcpyAsync(order.data(), kvo, X * 4, hipMemcpyDeviceToHost, stream));
    }
    FH_HIP(hipMemcpyAsync(hblocked.data(), blocked, V, hipMemcpyDeviceToHost, stream));
    FH_HIP(hipStreamSynchronize(stream));
    for (uint32_t v : order) {
      ready.push_back(vdot[v]);
      executed.add(vdot[v]);  // save_to_execute (mod.rs:330-331)
    }
    p_dot.clear();
    p_clk.clear();
    p_deps.clear();
    p_doff.assign(1, 0);
    for (size_t v = 0; v < V; v++) {
      if (!hblocked[v]) continue;
      p_dot.push_back(vdot[v]);
      p_clk.push_back(vclk[v]);
      p_deps.insert(p_deps.end(), deps.begin() + doff[v], deps.begin() + doff[v + 1]);
      p_doff.push_back(uint32_t(p_deps.size()));
    }
  }

  size_t drain(uint64_t *dots, size_t cap) {
    size_t c = 0;
    while (!ready.empty() && c < cap) {
      if (dots) dots[c] = ready.front();
      ready.pop_front();
      c++;
    }
    return c;
  }
};

}  // namespace fh

struct fh_pred {
  fh::PredDevice dev;
  fh_pred(uint32_t p, uint64_t s, const fh_config &c) : dev(p, s, c) {}
};

extern "C" {

fh_status fh_pred_create(uint32_t process_id, uint64_t shard_id, const fh_config *cfg,
                         fh_pred **out) {
  FH_API_BEGIN
  FH_CHECK(cfg && out, FH_EINVAL, "null argument");
  *out = new fh_pred(process_id, shard_id, *cfg);
  FH_API_END
}

fh_status fh_pred_destroy(fh_pred *h) {
  FH_API_BEGIN
  delete h;
  FH_API_END
}

fh_status fh_pred_add_batch(fh_pred *h, size_t n, const uint64_t *dot, const uint64_t *clock,
                            const uint32_t *dep_off, const uint64_t *dep_dot) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.add_batch(n, dot, clock, dep_off, dep_dot);
  FH_API_END
}

fh_status fh_pred_drain(fh_pred *h, uint64_t *exec_dot, size_t cap, size_t *len) {
  FH_API_BEGIN
  FH_CHECK(h && len, FH_EINVAL, "null argument");
  *len = h->dev.drain(exec_dot, exec_dot ? cap : 0);
  FH_API_END
}

fh_status fh_pred_pending(fh_pred *h, size_t *count) {
  FH_API_BEGIN
  FH_CHECK(h && count, FH_EINVAL, "null argument");
  *count = h->dev.p_dot.size();
  FH_API_END
}

}  // extern "C"
