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
//                   (= arrival) order, stable LDS sort by slot (wave64 ballot
//                   ranks), write the key-grouped sequence of dots, each
//                   command's dependency dot and each key's run bounds;
//                   tails update latest
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
// the two-launch path (kb > 22, more than 4M commands, or packed width > 32).
KeyBucketPlan keybucket_plan(size_t n, int kb);

// The key bijection alone (same multiplier as the plan), for paths that share
// the single-view latest table.
void keybucket_map(int kb, uint32_t *kmul, uint32_t *kinv, uint32_t *kmask);

struct KeyBucketWorkspace {
  DBuf<uint32_t> part;  // [n] tile-partitioned (slot << vb | command index)
  DBuf<uint32_t> hot;   // [16] hot mapped keys the batch was partitioned with
  DBuf<uint32_t> toff;  // [BT][tiles] tile-local bucket offset | count << 16
  DBuf<uint32_t> mc;    // [B][4][4096] slot tables of multi-chunk buckets
};

// The executed clock the path maintains (AEClock::add for every executed
// dot, tarjan.rs:296): a partition launch adds its batch's per-source max
// sequence / count to 8 shards of [max[256], count[256]] (u64) in `fold`;
// the launch that orders the batch folds them into frontier (max) and
// excount (sum) and clears them.  Batch parity selects one of two shard sets.
struct KeyBucketClock {
  unsigned long long *fold = nullptr;
  unsigned long long *frontier = nullptr;
  unsigned long long *excount = nullptr;
};
constexpr size_t kKeyBucketClockWords = 8 * 512;

// Workgroup schedule of the order role (a performance hint; any permutation
// orders correctly): order launches record each bucket's size, and
// keybucket_sched turns the last recorded sizes into a largest-first
// permutation used by the following launches, so the few Zipf-hot buckets
// start in the first round of workgroups instead of finishing last.
//
// Hot keys: a key with at least hot_min commands in one batch (a Zipf head)
// is routed by the partition to one of 16 hot-key buckets after the B
// regular ones; such a bucket holds one key, so it needs no sort, and the
// regular buckets stay near n / B.  Order launches offer candidates (key
// runs >= hot_min); keybucket_sched rebuilds the table.
struct KeyBucketSched {
  DBuf<uint32_t> sizes;  // [BT] commands per bucket (B regular + 16 hot), last order launch
  DBuf<uint32_t> perm;   // [BT] workgroup -> bucket
  DBuf<uint32_t> hot;    // [16] hot mapped keys (~0 empty), [1] candidates, [64][2] (count, key)
  uint32_t B = 0;        // BT of the plan the buffers were prepared for
  int bb = -1;
  uint32_t hot_min = 0;
  bool valid = false;    // perm computed for this width
};
void keybucket_sched(KeyBucketSched &sc, hipStream_t s);

// What the order launch writes.  In key-grouped order (buckets ascending,
// slots ascending, arrival order inside a key): sk = key ids, seq = the
// commands' dots.  By command index: rows = the command's dependency as a
// dot (~0 for none; the previous command on its key, or latest[key] from an
// earlier batch, resolved through dlog).  Per key id: runs[2 key] = the
// first position of the key's run, runs[2 key + 1] = its end | run_tag <<
// kRunEndBits.  A key the batch does not hold keeps an entry of another tag,
// so runs is cleared only when the tags wrap (zero is no tag).  latest is
// indexed by the mapped key; the batch's commands sit at log positions
// log_base + index.
constexpr int kRunEndBits = 23;  // run ends <= 2^22 (the plan's batch bound)
constexpr uint32_t kRunTags = 1u << (32 - kRunEndBits);
struct KeyBucketOut {
  uint32_t *sk = nullptr;
  uint64_t *seq = nullptr;
  uint64_t *rows = nullptr;
  uint32_t *runs = nullptr;
  uint32_t run_tag = 1;  // 1 .. kRunTags - 1
  const uint64_t *bdot = nullptr;  // the batch's dots
  const uint64_t *dlog = nullptr;  // the dot log
};

// Both launches on stream s.
void keybucket_run(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32, const uint64_t *dot,
                   uint64_t log_base, uint64_t *latest, const KeyBucketClock &clock,
                   KeyBucketWorkspace &ws, const KeyBucketOut &out, hipStream_t s,
                   KeyBucketSched *sc = nullptr);

// The two launches separately: keybucket_order reads the workspace
// keybucket_partition filled; clk = the shard set of that batch.
void keybucket_partition(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32,
                         const uint64_t *dot, unsigned long long *clk, KeyBucketWorkspace &ws,
                         hipStream_t s, KeyBucketSched *sc = nullptr);
void keybucket_order(const KeyBucketPlan &p, uint32_t n, uint64_t log_base, uint64_t *latest,
                     KeyBucketWorkspace &ws, const KeyBucketOut &out, const KeyBucketClock &clock,
                     hipStream_t s, KeyBucketSched *sc = nullptr);

// One launch that orders batch b (partitioned earlier into ws, clock shards
// clock.fold) and partitions batch b+1 (p2 / n2 / key32_2 / dot_2) into ws2
// with its clock shards in clk.
void keybucket_step(const KeyBucketPlan &p, uint32_t n, uint64_t log_base, uint64_t *latest,
                    KeyBucketWorkspace &ws, const KeyBucketOut &out, const KeyBucketClock &clock, const KeyBucketPlan &p2, uint32_t n2,
                    const uint32_t *key32_2, const uint64_t *dot_2, unsigned long long *clk,
                    KeyBucketWorkspace &ws2, hipStream_t s, KeyBucketSched *sc = nullptr);

}  // namespace fh
