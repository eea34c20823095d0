// graph_core.h -- batch SCC + execution order on the device.
//
// Input: V vertices in arrival order (vid = arrival position), dependency
// edges as vids (CSR), an optional "blocked" flag per vertex (it has a
// dependency that is neither executed nor in the batch), the vertex dots and
// keys.  Output: the SCC partition, the execution order and the per-key
// execution sequence the reference's incremental DependencyGraph
// (fantoch_ps/src/executor/graph/mod.rs:215-644) + TarjanSCCFinder
// (tarjan.rs:98-319) produce for the same arrival order, and the set of
// vertices that stay pending (PendingIndex, index.rs:145-211).
//
// Batch equivalence: a vertex executes iff nothing it
// reaches is missing; the SCCs found are the SCCs of the final graph; the
// reference executes SCC S at arrival time H(S) = max arrival position
// reachable from S ("ready time"), deps first.  The device computes
//   kappa(S) = max(kappa0(S), max_{S->S'} kappa(S') + 1),
//   kappa0(S) = (maxpos(S), 0)  packed as (H << 32 | depth)
// whose fixpoint is a strict topological order of the condensation that
// orders SCCs by ready time; members of an SCC run in dot order
// (tarjan.rs:14-15).
//
// SCC discovery: every cycle contains a forward edge (dep arrived later).
// Windows of 128 arrival positions (stride 64) compute their local transitive
// closure with a bit-matrix Warshall held in one wave's registers; mutually
// reachable vertices are united with a lock-free union-find.  Overlapping
// local SCCs chain into large ones (e.g. one stream-wide SCC under 100%
// conflict).  Convergence of kappa certifies the partition (a missed cycle
// would make kappa grow forever); if it does not converge within a bound the
// exact coloring fallback (Orzan-style, over the condensation) completes it.
#pragma once

#include <utility>
#include <vector>

#include "fh_common.h"
#include "scan.h"
#include "sort.h"

namespace fh {

struct GraphInput {
  uint32_t V = 0;
  const uint32_t *off = nullptr;     // [V+1]; null = fixed stride
  uint32_t stride = 0;               // edges of v at dst[v*stride ..) when off == null
  const uint32_t *dst = nullptr;     // [E] dependency vids (v itself = padding)
  const uint8_t *blocked0 = nullptr; // [V] or null: has a missing dependency
  const uint64_t *dot = nullptr;     // [V]
  // [V] or null: an initial partition, each vertex's class root (the class's
  // minimum vid); the global path treats its classes as strongly connected
  // (dgraph's split hub vertices)
  const uint32_t *rep0 = nullptr;
  // keys: fixed k per vertex (key_off == null) or CSR
  uint32_t k = 0;
  const uint32_t *key_off = nullptr; // [V+1] or null
  const uint32_t *key32 = nullptr;   // [elements]
  int key_bits = 1;
  // fast path hint: elements already sorted by (key, arrival) -- reused as
  // the per-key order when the graph turns out to be trivially ordered
  const uint32_t *sorted_keys = nullptr;  // [M]
  const uint32_t *sorted_vid = nullptr;   // [M] vid of each sorted element
  bool no_forward_hint = false;           // edges all point backwards
  // [64] or null: the forward edges, counted by the producer of the edges
  // (the sum is count_forward's result, without its pass)
  const unsigned long long *fwd_counts = nullptr;
  bool want_per_key = true;               // build the per-key sequence
  bool global_only = false;               // skip the tile path (fh_dgraph: rep + kap wanted)
  bool want_orders = true;                // false: SCCs, kappa and labels only (out.kap)
  bool per_key_dots = false;              // ... of dots (pk_dot) instead of vids
  // dots packable as src << dot_sb | seq in dot_pbits <= 32 bits (0: not
  // known / not packable): the per-key sort then moves 4-byte values
  int dot_sb = 0, dot_pbits = 0;
  // optional: per-source (max seq, count) of the executed dots, accumulated
  // by a pass that reads every dot anyway (GraphOutput::src_stats_done)
  unsigned long long *src_mx = nullptr;   // [256]
  unsigned int *src_cnt = nullptr;        // [256]
  // the engine's key-order graph (engine.hip, cmd_views_keyorder): edge
  // slots are 8-bit distances (dst_codes), the
  // dots packed 32-bit (dot32, src << dot32_sb | seq; `dot` unused), and
  // only the tile path runs: on a certificate failure run() returns with
  // out.nexec == 0 and the caller takes another route.  On success the
  // tiles' outputs are read through tile_h / tile_rank / tile_count /
  // tile_start and out.scc_label.
  bool dst_codes = false;  // dst = one u32 per vertex of signed 8-bit
                           // distances (byte s: v - target, 0 none, -128:
                           // target + 1 in dst_esc[v·stride + s])
  const uint32_t *dst_esc = nullptr;
  bool tile_prio = false;  // tile kernel waves at raised issue priority
  const uint32_t *dot32 = nullptr;
  int dot32_sb = 0;
  bool tiles_only = false;
  // tiles_only with the key-order outputs written by the tiles themselves
  // (TileOut::ko_*, graph_tile.hip): per-key sequence, command-order
  // records and straddle differences of multi-member groups
  uint64_t *ko_seq = nullptr;
  uint4 *ko_hl = nullptr;
  uint32_t *ko_diff = nullptr;
  const uint32_t *ko_cmd = nullptr;
  uint32_t ko_cstride = 0, ko_cmask = 0;
};

struct GraphOutput {
  // device pointers owned by GraphCore, valid until the next run
  uint32_t nexec = 0;          // executed vertices
  uint32_t npending = 0;
  bool trivial = false;        // no forward edges, no pending: arrival order
  bool fallback_used = false;
  uint32_t kappa_iters = 0;
  uint32_t *rep = nullptr;        // [V] representative (min vid) of the SCC
  uint64_t *scc_label = nullptr;  // [V] min dot of the SCC
  uint8_t *blocked = nullptr;     // [V] pending
  uint32_t *exec_order = nullptr; // [nexec] vids in execution order (null if trivial)
  uint32_t *exec_rank = nullptr;  // [V] position in exec order, ~0u if pending
  uint32_t nelem = 0;             // per-key sequence length
  uint32_t *pk_key = nullptr;     // [nelem] keys, ascending
  uint32_t *pk_vid = nullptr;     // [nelem] vids in per-key execution order
  uint64_t *pk_dot = nullptr;     // [nelem] their dots (per_key_dots: pk_vid null)
  bool src_stats_done = false;    // src_mx / src_cnt accumulated
  uint64_t *kap = nullptr;        // [V] by representative: (ready time << 32) | depth
                                  // (global path only)
};

struct TileOut;  // graph_tile.hip

struct GraphCore {
  hipStream_t stream = nullptr;
  SortWorkspace sort_ws;
  ScanWorkspace scan_ws;
  DBuf<uint32_t> rep, cnt, pos, order, rank, tmp32a, tmp32b, tmp32c, tmp32d, flags;
  DBuf<uint32_t> kraise;  // [V] last kappa iteration that raised kap[rep]
  DBuf<uint32_t> erep;    // [E] rep[dst[e]] (refresh_edge_rep)
  uint64_t nedges = 0;
  DBuf<uint64_t> kap, label, tmp64a, tmp64b, tmp64c, pk_da, pk_db;
  DBuf<uint8_t> blocked;
  DBuf<uint32_t> t_h, t_rank, t_cnt, t_start;
  DBuf<uint8_t> t_fail;     // graph_tile mixed bounds: pass-1 failed tiles
  DBuf<uint32_t> t_cores;   // graph_tile mixed bounds: pass-2 cores (start, length)
  uint32_t dbg_mixed_redo = 0;
  // run_tiles left the execution order as (ready time, rank in group, group
  // starts): build_per_key's fill computes each rank itself (no order array)
  bool fill_from_groups = false;
  DBuf<uint64_t> t_prof;  // tile path: ready time, group rank/count/start
  uint32_t dbg_tile_fail = 0, dbg_tile_ok = 0;
  DBuf<uint8_t> fb_pushed;    // coloring reach: vertices that pushed this round
  DBuf<uint32_t> fb_bits;     // coloring H propagation: three class bitmaps (frontier)
  bool prefer_full = false;   // the last global-path run needed the full coloring
  bool kap_seed_ok = true;    // kap holds a bounded run's ready times (k_fb_seed)
  DBuf<uint32_t> conv;        // device-side convergence flags (converge())
  template <class L>
  void converge(uint32_t words, uint32_t &launches, L launch);
  DBuf<uint32_t> hseed;       // [V] exact ready time per vertex from the full coloring
  bool hseed_ok = false;
  uint32_t dbg_kap_list = 0;  // vertices the seeded kappa run relaxed after its first launch      // hseed holds this run's first full coloring round
  uint32_t tile_r0 = 1536;  // graph_tile: first reach bound to try (set from
                            // the last run's maximum excess)
  DBuf<uint32_t> scalars;  // device scalars (changed flags, counters)
  bool profile = false;
  uint32_t dbg_rounds = 0, dbg_hprop = 0, dbg_reach = 0;  // FH_GRAPH_DEBUG counters
  uint32_t dbg_cand = 0, dbg_restricted = 0, dbg_sync_n = 0, dbg_left = 0;
  double dbg_sync_us = 0;
  // per-kernel timing (engine profiling)
  std::vector<std::pair<const char *, hipEvent_t>> *marks = nullptr;

  void run(const GraphInput &in, GraphOutput &out);
  // tile outputs of the last run (valid after a tiles_only run succeeded):
  // ready time H, rank in the ready group, group size at the root (0
  // elsewhere), first execution position of each group
  const uint32_t *tile_h() const { return t_h.get(); }
  const uint32_t *tile_rank() const { return t_rank.get(); }
  const uint32_t *tile_count() const { return t_cnt.get(); }
  const uint32_t *tile_start() const { return t_start.get(); }

  // back to a fresh engine's first guesses (fh_engine_forget_tuning)
  void forget_tuning() {
    prefer_full = false;
    tile_r0 = 1536;
  }
 private:
  void mark(const char *name);
  void take_sorted(const uint32_t *vs, DBuf<uint32_t> &out);
  uint32_t read_scalar(int i);
  void pending_closure(const GraphInput &in, GraphOutput &out);
  uint64_t count_forward(const GraphInput &in);
  void init_rep(const GraphInput &in);
  void find_sccs(const GraphInput &in);
  void refresh_edge_rep(const GraphInput &in);
  bool order_kappa(const GraphInput &in, uint32_t max_iters, uint32_t &iters,
                   bool give_up_early = false);
  // false: restricted candidates too many, nothing done
  bool coloring_fallback(const GraphInput &in, uint32_t recent_iter);
  void build_orders(const GraphInput &in, GraphOutput &out);
  void build_labels(const GraphInput &in, GraphOutput &out);
  void build_per_key(const GraphInput &in, GraphOutput &out);
  // tile-local path (graph_tile.hip): false = certificate failed, nothing set
  bool tiles_eligible(const GraphInput &in) const;
  bool run_tiles(const GraphInput &in, GraphOutput &out);
  bool tiles_mixed(const GraphInput &in, TileOut &to, uint32_t r2, uint32_t *st);
};

}  // namespace fh
