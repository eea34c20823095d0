// keybucket.h -- single-view, one-key-per-command KeyDeps + per-key order in
// two launches (the C2 hot path).
//
// SequentialKeyDeps::do_add_cmd
// (fantoch_ps/src/protocol/common/graph/deps/keys/sequential.rs:72-104) over a
// whole batch: the dependency of command i is the previous command (arrival
// order) on its key, or latest[key] from an earlier batch at the key's first
// occurrence; the key's last command becomes latest[key] (:88-95).  The
// per-key execution sequence (ExecutionOrderMonitor, fantoch/src/executor/
// monitor.rs:20-28) of a single view is the key's commands in arrival order.
//
// Keys are mapped through a bijection of the 2^kb key space (Fibonacci
// multiplier) so Zipf-hot ids spread over buckets; the latest table of the
// single view is indexed by the mapped key, so one bucket's entries are one
// contiguous slice of the table.
//   k_kb_partition  per 4096-command tile: stable partition of the tile by
//                   bucket (high bits of the mapped key), tile-local bucket
//                   offsets (u16), executed-clock partials
//   k_kb_order      per bucket: gather its runs from every tile in tile
//                   (= arrival) order, per-slot rank and predecessor with
//                   wave64 ballot matching, write the key-grouped sequence and
//                   each command's dependency; tails update latest
#pragma once

#include "fh_common.h"

namespace fh {

struct KeyBucketPlan {
  bool ok = false;
  int kb = 0;  // key bits (mapped key space = 2^kb)
  int bb = 0;  // bucket bits
  int hb = 0;  // slot bits inside a bucket (kb - bb)
  int vb = 0;  // command-index bits
  uint32_t tiles = 0;
  uint32_t kmul = 1, kinv = 1, kmask = 0;  // mapped key = (key * kmul) & kmask
};

// Plan for n commands over ids < 2^kb; ok == false if the batch does not fit
// the two-launch path (kb > 22, more than 1024 tiles, or packed width > 32).
KeyBucketPlan keybucket_plan(size_t n, int kb);

// The key bijection alone (same multiplier as the plan), for paths that share
// the single-view latest table.
void keybucket_map(int kb, uint32_t *kmul, uint32_t *kinv, uint32_t *kmask);

struct KeyBucketWorkspace {
  DBuf<uint32_t> part;  // [n] tile-partitioned (slot << vb | command index)
  DBuf<uint16_t> toff;  // [tiles][B + 1] tile-local bucket offsets
};

// Runs both launches on stream s.  Outputs, in key-grouped order (buckets
// ascending, slots ascending, arrival order inside a key): sk = key ids,
// sv = command indices, dep_sorted = dependency of that command (0 none,
// index + 1 in-batch, otherwise the dot from latest).  latest is indexed by
// the mapped key; frontier / excount receive the per-source executed-clock
// max / count of the batch.
void keybucket_run(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32, const uint64_t *dot,
                   uint64_t *latest, unsigned long long *frontier, unsigned long long *excount,
                   KeyBucketWorkspace &ws, uint32_t *sk, uint32_t *sv, uint64_t *dep_sorted,
                   hipStream_t s);

}  // namespace fh
