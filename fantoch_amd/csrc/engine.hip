// engine.hip -- fused, device-resident dependency engine (fh_engine_*).
//
// One batch of committed commands goes through, without leaving HBM:
//   KeyDeps    per replica view: stable radix sort of (replica, key, arrival)
//              elements, previous element of each (replica, key) segment is the
//              dependency (SequentialKeyDeps::do_add_cmd,
//              fantoch_ps/src/protocol/common/graph/deps/keys/sequential.rs:72-104);
//              the persistent latest table answers segment heads
//   union      the committed deps of a command are the union of its fast-quorum
//              members' reports (QuorumDeps, deps/quorum.rs:28-98, called at
//              atlas.rs:356-366 / epaxos.rs:333-342); each member's report is
//              the coordinator's deps plus its own (atlas.rs:303-309)
//   graph      SCC + execution order + per-key sequence (graph_core.hip)
//   clock      the executed clock advances (AEClock::add, tarjan.rs:296)
// With a single view every dependency points to an earlier arrival, so the
// arrival order is already topological and the per-key order is the key-sorted
// element order: the graph stage certifies that and reuses it.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "engine_internal.h"
#include "hoststage.h"
#include "graph_core.h"
#include "keybucket.h"
#include "sort_impl.h"
#include "srcstats.h"

namespace fh {
namespace {

constexpr unsigned B = 256;
#define GRID_STRIDE(i, n) \
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += gridDim.x * blockDim.x)
// wave-uniform trip count (lanes past n see i >= n): shuffles inside are safe
#define WAVE_STRIDE(i, n)                                                      \
  for (uint32_t i##_b = blockIdx.x * blockDim.x; i##_b < (n);                  \
       i##_b += gridDim.x * blockDim.x)                                        \
    for (uint32_t i = i##_b + threadIdx.x, i##_once = 1; i##_once; i##_once = 0)

// Replica views as per-replica arrival logs: replica r's SequentialKeyDeps
// sees the commands of log r in log order (its add_cmd calls, atlas.rs:236,
// :303-309).  Command logs: element x = q·k + s is key slot s of log entry q
// (entry e = c·fq + j: command c as fast-quorum member j).  Element logs
// (partial replication, FH_STREAM_ELEMENT_LOGS): entry q is one element,
// position (c·fq + j)·k + s, as each shard's replicas process only the
// command's keys on their shard (Command::keys(shard), command.rs:95-100).
// Entries are concatenated replica by replica, so element order is (replica,
// arrival, slot) and a stable sort by the segment id (r + 1)·K + key yields
// every (replica, key) segment in arrival order.  The value is the element's
// command-major position (c·fq + j)·k + s, where the union reads it.
// One chunk of the logs: replica r contributes its entries
// [first[r], first[r] + count[r]) (chunk-local element order = replica, then
// arrival, then slot); cum[r] = elements of the replicas before r.
constexpr int kMaxLogs = 64;
struct LogChunk {
  uint32_t first[kMaxLogs];
  uint32_t cum[kMaxLogs + 1];
  // the replica holding chunk element x: the last r with cum[r] <= x
  __device__ __forceinline__ uint32_t replica(uint32_t x, uint32_t nlog) const {
    uint32_t lo = 0, hi = nlog - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (cum[mid] <= x)
        lo = mid;
      else
        hi = mid - 1;
    }
    return lo;
  }
};

// Dependency-code placement (replica views).  Writing each element's code
// straight to its command-major position is a 4-byte write to a random
// address of the chunk's ~50 MB window, ~32 B of fabric traffic each.
// Instead, one bucketing pass groups (position - base, code) pairs by the
// position's bits [15, 24) -- an LDS-staged scatter with contiguous runs per
// tile and bucket, as in the sort -- and k_place assembles each bucket's 32K
// positions in LDS and writes them out whole.  An element below the base or
// past the 2^24-position span wraps into some bucket; k_place writes such
// strays directly (correct, slower).
constexpr int kPlaceShift = 15;
constexpr int kPlaceDB = 9;  // 512 buckets
constexpr uint32_t kPlaceBuckets = 1u << kPlaceDB;
constexpr uint32_t kPlaceSpan = 1u << kPlaceShift;
constexpr uint32_t kPlaceSlack = 1u << 16;  // default (FH_PLACE_SLACK): arrivals ahead of earlier commands
constexpr uint32_t kPlaceNone = ~0u;        // never a code (log references < 2^31 - 1)

// emin (may be null): the placement base of the chunk.  One workgroup per
// sort tile (kTile consecutive elements): it also writes the tile's digit
// counts at shift 0 (digits of dmask + 1 values, sort_digit_bits) for the
// sort's first pass (sort_pairs_counted: no separate counting pass over the
// keys it just wrote).
// elem != 0: element logs (each entry a position (c·fq + j)·k + s).
__global__ void __launch_bounds__(kThreads)
    k_log_keys(uint32_t M, uint32_t k, uint32_t fq, uint32_t nlog, uint32_t elem, LogChunk ch,
               const uint32_t *__restrict__ ent, const uint32_t *__restrict__ key32,
               uint32_t K, uint32_t *__restrict__ keys, uint32_t *__restrict__ vals,
               uint32_t *__restrict__ emin, uint32_t slack, uint32_t *__restrict__ counts,
               uint32_t dmask) {
  __shared__ uint32_t s_h[256];
  __shared__ uint32_t s_r0;
  // the chunk's log table in LDS: indexed per lane, the kernel argument was a
  // vector load from the argument segment per element and lookup
  __shared__ uint32_t s_cum[kMaxLogs + 1], s_first[kMaxLogs];
  s_h[threadIdx.x] = 0;
  if (threadIdx.x <= nlog) s_cum[threadIdx.x] = ch.cum[threadIdx.x];
  if (threadIdx.x < nlog) s_first[threadIdx.x] = ch.first[threadIdx.x];
  const uint32_t base = blockIdx.x * uint32_t(kTile), end = min(M, base + uint32_t(kTile));
  // the tile's first log, searched once: a tile spans a log or two, so each
  // element advances from there (element logs: 40 logs, a search per element
  // was half the kernel)
  if (threadIdx.x == 0) s_r0 = base < M ? ch.replica(base, nlog) : 0u;
  __syncthreads();
  uint32_t r = s_r0;
  const uint32_t per = fq * k;
  for (uint32_t x = base + threadIdx.x; x < end; x += kThreads) {
    while (r + 1 < nlog && s_cum[r + 1] <= x) r++;
    const uint32_t y = x - s_cum[r];
    uint32_t key, val;
    if (elem) {
      val = ent[s_first[r] + y];
      key = (r + 1) * K + key32[(val / per) * k + val % k];
    } else {
      const uint32_t q = s_first[r] + y / k, s = y % k;
      const uint32_t e = ent[q];
      key = (r + 1) * K + key32[(e / fq) * k + s];
      val = e * k + s;
    }
    keys[x] = key;
    vals[x] = val;
    atomicAdd(&s_h[key & dmask], 1u);
  }
  __syncthreads();
  if (threadIdx.x <= dmask) counts[size_t(blockIdx.x) * (dmask + 1) + threadIdx.x] = s_h[threadIdx.x];
  // placement base: the smallest first entry of the replicas' slices, less a
  // slack for entries that arrive before earlier commands.  Only a hint (see
  // above).  An exact minimum by atomics serialised the kernel on one word:
  // 1.37 ms instead of 0.04 per chunk.
  if (emin && blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t m = ~0u;
    for (uint32_t r = 0; r < nlog; r++)
      if (ch.cum[r + 1] > ch.cum[r]) m = min(m, elem ? ent[ch.first[r]] : ent[ch.first[r]] * k);
    *emin = m > slack ? m - slack : 0u;
  }
}

// bucketing source: element j of the chunk's (key, arrival) order yields
// (its position - base, its dependency code): the previous element's
// command, or the latest entry at a segment head
struct PrevSrc {
  const uint32_t *ks, *vs, *ebase;
  const uint64_t *latest;
  uint32_t per_cmd;
  __device__ __forceinline__ uint32_t key(uint32_t j) const { return vs[j] - *ebase; }
  __device__ __forceinline__ uint32_t code(uint32_t j) const {
    const uint32_t seg = ks[j];
    if (j == 0 || ks[j - 1] != seg) {
      const uint64_t x = latest[seg];
      return x ? (0x80000000u | uint32_t(x - kLogFlag)) : 0u;
    }
    return vs[j - 1] / per_cmd + 1;
  }
  // as a sort source (k_up's tile counts read the key only)
  __device__ __forceinline__ void get(uint32_t j, uint32_t &k, uint32_t &v) const {
    k = key(j);
    v = 0;
  }
};

// The bucketing pass: k_down's tile staging, but the order within a bucket
// is free, so ranks come from LDS atomics (no ballot matching).  One
// 512-thread workgroup takes two count tiles (8192 elements): the runs of
// consecutive tiles in one bucket are adjacent in the output, so a bucket's
// run per workgroup averages 16 elements (64 B per array) instead of 8 --
// 4096-element workgroups wrote 32 B runs, half-line writes.
// With `defer` set the pass also makes the segment tails the latest entries
// (k_tail_engine's job): every head of the workgroup has read its latest
// entry before the barrier, so the tail of a segment that starts in the
// workgroup is written in place; the tail of the first segment, if it began
// in an earlier workgroup (whose head may not have read yet), goes to
// defer[2·b] = (segment, command) for k_place to apply.
constexpr int kBucketThreads = 512;
constexpr int kBucketWaves = kBucketThreads / 64;
constexpr int kBucketTile = 2 * kTile;  // 8192
__global__ void __launch_bounds__(kBucketThreads)
    k_bucket_codes(PrevSrc src, uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                   uint32_t n, const uint32_t *__restrict__ counts,
                   const uint32_t *__restrict__ gsum, uint32_t gsize,
                   const uint32_t *__restrict__ dbase, uint64_t *latest_w,  // aliases src.latest
                   uint64_t log_base, uint32_t *__restrict__ defer) {
  constexpr uint32_t R = kPlaceBuckets;
  __shared__ uint32_t s_def[2];
  static_assert(R == kBucketThreads, "one bucket per thread in the scan");
  __shared__ uint32_t s_k[kBucketTile], s_v[kBucketTile];
  __shared__ uint32_t s_cnt[R], s_dex[R], s_gb[R];
  __shared__ uint32_t s_tmp[kBucketWaves];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t tile0 = blockIdx.x * 2, base = blockIdx.x * kBucketTile;
  // this workgroup's run of bucket d starts where count tile tile0's does
  s_cnt[tid] = 0;
  s_gb[tid] = dbase[tid] + gsum[size_t(tile0 / gsize) * R + tid] + counts[size_t(tile0) * R + tid];
  // all loads first: the element's key and position, its predecessor's,
  // then the latest entries of the segment heads
  const uint32_t eb = *src.ebase;
  uint32_t key[kItems], val[kItems], seg[kItems], pseg[kItems], pv[kItems], nseg[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + uint32_t(lane);
    const bool ok = idx < n;
    key[i] = ok ? src.vs[idx] - eb : 0u;
    seg[i] = ok ? src.ks[idx] : 0u;
    pseg[i] = ok && idx > 0 ? src.ks[idx - 1] : ~0u;
    pv[i] = ok && idx > 0 ? src.vs[idx - 1] : 0u;
  }
  if (defer) {
    // the next element's segment: lane + 1 of the same item, lane 0 of the
    // next item for lane 63, a load for the wave's last element only
#pragma unroll
    for (int i = 0; i < kItems; i++) {
      const uint32_t up = __shfl_down(seg[i], 1, 64);
      const uint32_t nx = i + 1 < kItems ? __shfl(seg[i + 1 < kItems ? i + 1 : i], 0, 64) : 0u;
      const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + uint32_t(lane);
      nseg[i] = lane < 63 ? up : nx;
      if (idx + 1 >= n) nseg[i] = ~0u;
      else if (lane == 63 && i + 1 == kItems) nseg[i] = src.ks[idx + 1];
    }
  }
  const uint32_t first_seg = defer && base > 0 ? src.ks[base - 1] : ~0u;
  if (defer && tid == 0) s_def[0] = ~0u;
  uint64_t lat[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) lat[i] = pseg[i] != seg[i] ? src.latest[seg[i]] : 0ull;
#pragma unroll
  for (int i = 0; i < kItems; i++)
    val[i] = pseg[i] != seg[i] ? (lat[i] ? (0x80000000u | uint32_t(lat[i] - kLogFlag)) : 0u)
                               : pv[i] / src.per_cmd + 1;
  __syncthreads();
  if (defer) {
#pragma unroll
    for (int i = 0; i < kItems; i++) {
      const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + uint32_t(lane);
      if (idx < n && nseg[i] != seg[i]) {
        const uint32_t cmd = (key[i] + eb) / src.per_cmd;
        if (seg[i] == first_seg) {
          s_def[0] = seg[i];
          s_def[1] = cmd;
        } else {
          latest_w[seg[i]] = kLogFlag | (log_base + cmd);
        }
      }
    }
  }
  uint32_t rank[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + uint32_t(lane);
    rank[i] = idx < n ? atomicAdd(&s_cnt[(key[i] >> kPlaceShift) & (R - 1)], 1u) : 0u;
  }
  __syncthreads();
  {
    // exclusive scan of the bucket counts, one bucket per thread
    const uint32_t c = s_cnt[tid];
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(x, o, 64);
      if (lane >= o) x += t;
    }
    if (lane == 63) s_tmp[w] = x;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int i = 0; i < kBucketWaves; i++)
      if (i < w) pre += s_tmp[i];
    s_dex[tid] = pre + x - c;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + uint32_t(lane);
    if (idx < n) {
      const uint32_t p = s_dex[(key[i] >> kPlaceShift) & (R - 1)] + rank[i];
      s_k[p] = key[i];
      s_v[p] = val[i];
    }
  }
  __syncthreads();
  if (defer && tid == 0) {
    defer[2 * blockIdx.x] = s_def[0];
    defer[2 * blockIdx.x + 1] = s_def[1];
  }
  const uint32_t tile_n = min(uint32_t(kBucketTile), n - base);
#pragma unroll 4
  for (uint32_t j = tid; j < tile_n; j += kBucketThreads) {
    const uint32_t kk = s_k[j];
    const uint32_t d = (kk >> kPlaceShift) & (R - 1);
    const uint32_t o = s_gb[d] + (j - s_dex[d]);
    kout[o] = kk;
    vout[o] = s_v[j];
  }
}

// one workgroup per bucket d: positions base + [d·2^15, (d+1)·2^15)
// It also applies k_bucket_codes' deferred tails (defer: nb slots).
__global__ void __launch_bounds__(1024)
    k_place(uint32_t Mc, const uint32_t *__restrict__ dbase, const uint32_t *__restrict__ rel,
            const uint32_t *__restrict__ code, const uint32_t *__restrict__ ebase,
            uint32_t *__restrict__ out, const uint32_t *__restrict__ defer, uint32_t nb,
            uint64_t *__restrict__ latest, uint64_t log_base) {
  __shared__ uint32_t s_c[kPlaceSpan];  // 128 KB
  const uint32_t d = blockIdx.x;
  if (defer) {
    const uint32_t b = d * 1024 + threadIdx.x;
    if (b < nb && defer[2 * b] != ~0u) latest[defer[2 * b]] = kLogFlag | (log_base + defer[2 * b + 1]);
  }
  for (uint32_t i = threadIdx.x; i < kPlaceSpan; i += 1024) s_c[i] = kPlaceNone;
  __syncthreads();
  const uint32_t s = dbase[d], t = d + 1 < kPlaceBuckets ? dbase[d + 1] : Mc;
  const uint32_t eb = *ebase;
  for (uint32_t j = s + threadIdx.x; j < t; j += 1024) {
    const uint32_t r = rel[j], c = code[j];
    if ((r >> kPlaceShift) == d)
      s_c[r & (kPlaceSpan - 1)] = c;
    else
      out[eb + r] = c;  // a stray (below the base or past the span)
  }
  __syncthreads();
  uint32_t *o = out + eb + (d << kPlaceShift);
  for (uint32_t i = threadIdx.x; i < kPlaceSpan; i += 1024) {
    const uint32_t c = s_c[i];
    if (c != kPlaceNone) o[i] = c;
  }
}

// ---------------------------------------------------------------------------
// Command-level KeyDeps over replica views (one key per command).
//
// The chunked path sorts every replica's elements: fq elements per command.
// Here the commands are sorted once by key (stable, so each key's commands
// stay in stream order) and every element finds its replica-local
// predecessor among its key's neighbours in that order.  The search is
// bounded by the logs' inversion span W: for each replica log,
// W_r = max over positions of (largest command index seen so far - this
// command), computed at staging, W = max_r W_r.  Then for two commands c, c'
// that replica r both processes:
//   c' <  c - W  =>  c' arrives at r before c;
//   c' arrives at r before c  =>  c' <= c + W.
// So the predecessor of (c, r) -- the latest arrival at r before c among the
// key's commands (SequentialKeyDeps::add_cmd, sequential.rs:72-104) -- is
// found scanning back until past (first r-command below c - W) - W, and
// forward up to c + W; (c, r) is the key's last arrival at r (its tail:
// latest_deps becomes c, :88-95) iff no r-command of the key arrives later,
// which the same scans decide (any r-command beyond c + W arrives later).
// Batches whose logs exceed kCmdMaxW take the chunked path.
constexpr uint32_t kCmdMaxW = 4096;
constexpr int kSrchThreads = 1024;
constexpr int kKoSrchThreads = 512;  // the key-order path (cmd_views_keyorder)
constexpr uint32_t kRecT = 27;  // rec = replica << 27 | arrival position
constexpr uint32_t kNoCmd = ~0u;

struct LogOffs {
  uint32_t off[kMaxLogs + 1];
  // the replica id log r's records carry (identity, or for element logs the
  // pair-level search's local ids: EngineDevice::unit_meta)
  uint32_t rid[kMaxLogs];
};

// rec[e] for every element e = c·fq + j: which replica (log) holds it and at
// which position of that log.  Element e sits at e / fq of the stream, so a
// direct scatter from each log writes every line in fq pieces, far apart in
// time (3.4 ms at C4).  Workgroup w instead takes the w-th slice of every
// log -- commands ~[w·n/G, (w+1)·n/G) -- assembles their records in an LDS
// window of kRecWin positions and writes the window out whole; an element
// outside its window (a late arrival) is written directly.
// 64 KB of LDS: two workgroups per CU (FH_REC_WIN=32768, one: 1072 against
// 935 us per C4 launch; 8192: 1391)
constexpr uint32_t kRecWin = 16384;
constexpr uint32_t kRecNone = ~0u;    // never a record (replica < 16)
// window positions below the slice's first command
constexpr uint32_t rec_slack(uint32_t win) { return win / 16; }
template <uint32_t WIN>
__global__ void __launch_bounds__(1024)
    k_view_records(uint32_t n, uint32_t fq, uint32_t np, uint32_t G, LogOffs lo,
                   const uint32_t *__restrict__ ent, uint32_t *__restrict__ rec,
                   const uint32_t *__restrict__ bounds) {
  __shared__ uint32_t s_v[WIN];
  __shared__ uint32_t s_pre[kMaxLogs + 1], s_q0[kMaxLogs], s_ql[kMaxLogs];
  const uint32_t w = blockIdx.x;
  for (uint32_t p = threadIdx.x; p < WIN; p += 1024) s_v[p] = kRecNone;
  const uint64_t c0 = uint64_t(n) * w / G;
  const uint64_t e0 = c0 * fq > rec_slack(WIN) ? c0 * fq - rec_slack(WIN) : 0;
  // the slice's entries of all logs as one run (log r's part from s_pre[r]:
  // entry f is ent[s_q0[r] + f], position s_ql[r] + f of log r), sixteen per
  // thread with their loads issued together (tried: log by log, four loads
  // per trip: 836 us per C4 launch)
  // bounds (element logs, staged): slice w of log r is its entries from the
  // first one of command >= c0 -- a log's share of the commands drifts
  // along the stream when which processes hold a command depends on its
  // keys, so proportional slices would leave most records outside the window
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t r = 0; r < np; r++) {
      const uint64_t len = lo.off[r + 1] - lo.off[r];
      const uint32_t q0 = lo.off[r] + (bounds ? bounds[size_t(w) * np + r] : uint32_t(len * w / G));
      const uint32_t q1 = lo.off[r] + (bounds ? bounds[size_t(w + 1) * np + r]
                                             : uint32_t(len * (w + 1) / G));
      s_pre[r] = t;
      s_q0[r] = q0 - t;
      // the replica id rides in the record base: lo.rid[r] indexed per lane
      // in the loop below was a waterfall of scalar kernel-argument loads
      // (C4 view records 0.61 -> 0.90 ms when the ids arrived, round 6)
      s_ql[r] = (lo.rid[r] << kRecT) + (q0 - lo.off[r] - t);
      t += q1 - q0;
    }
    s_pre[np] = t;
  }
  __syncthreads();
  const uint32_t tot = s_pre[np];
  constexpr int kU = 16;
  for (uint32_t fb = 0; fb < tot; fb += kU * 1024) {
    uint32_t ev[kU], vv[kU];
    uint32_t r = 0;
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint32_t f = fb + u * 1024 + threadIdx.x;
      ev[u] = kRecNone;
      if (f < tot) {
        while (f >= s_pre[r + 1]) r++;
        ev[u] = ent[s_q0[r] + f];
        vv[u] = s_ql[r] + f;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint32_t e = ev[u];
      if (e == kRecNone) continue;
      const uint64_t rel = uint64_t(e) - e0;
      if (e >= e0 && rel < WIN)
        s_v[rel] = vv[u];
      else
        rec[e] = vv[u];
    }
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < WIN; p += 1024) {
    const uint32_t v = s_v[p];
    if (v != kRecNone) rec[e0 + p] = v;
  }
}

// The command-level sort input.  Each command travels through the key sort
// with everything the search needs, so the search reads only the sorted
// arrays (a gather of its view records in key order, as round 2's first
// version did, cost a random line per command: 10.4 ms at C4).  The key word
// holds the key in bits [0, kb) -- the sort's digits cover exactly those --
// and meta bits above; the u64 value holds the command in bits [0, cb) and
// the rest of the meta.  The meta is, per view j, the replica id (rb bits)
// and its arrival position in that replica's log modulo 2^qb.
//
// Arrival order from the truncated positions.  For two commands c1 != c2
// that replica r both processes, with the logs' inversion span W:
//   c1 + W < c2  =>  c1 arrives first;   c2 + W < c1  =>  c2 arrives first;
// otherwise every log entry between their arrivals is a command in
// [min - W, max + W] (one arriving later than that range would have been
// preceded by a larger command than W allows, and symmetrically), so their
// positions differ by at most 3W + 1 < 2^(qb-1): the sign of the difference
// modulo 2^qb decides.  The host checks 3W + 1 < 2^(qb-1) before taking
// this path.
struct CmdMeta {
  uint32_t fq, rb, qb, vb;  // views; bits per view: replica, arrival, both
  uint32_t kb, cb;          // key word: meta from bit kb; value: command in [0, cb)
  uint32_t kmask, W;
  uint64_t cmask, qmask;
  // the pair-level search (element logs, k keys per command): the units are
  // (command, key slot) pairs u = c << us | s, so a unit's command is u >> us
  // (us = 0: units are commands); region records cover 2^rsh units each
  uint32_t us, rsh;
  __device__ __forceinline__ uint64_t meta(uint32_t kw, uint64_t v) const {
    return (v >> cb) | ((uint64_t(kw) >> kb) << (64 - cb));
  }
  __device__ __forceinline__ uint32_t rep(uint64_t m, uint32_t j) const {
    return uint32_t(m >> (j * vb + qb)) & ((1u << rb) - 1);
  }
  __device__ __forceinline__ uint32_t arr(uint64_t m, uint32_t j) const {
    return uint32_t((m >> (j * vb)) & qmask);
  }
  // the arrival of the command whose meta is m at replica r, if it has one
  __device__ __forceinline__ bool find(uint64_t m, uint32_t r, uint32_t *t) const {
    bool f = false;
    for (uint32_t j = 0; j < fq; j++) {
      const bool h = rep(m, j) == r;
      *t = h ? arr(m, j) : *t;
      f |= h;
    }
    return f;
  }
  // (c1, arrival q1) reaches the replica before (c2, q2)
  __device__ __forceinline__ bool before(uint32_t c1, uint32_t q1, uint32_t c2, uint32_t q2) const {
    const bool lo = uint64_t(c1) + W < c2, hi = uint64_t(c2) + W < c1;
    const uint32_t d = (q2 - q1) & uint32_t(qmask);
    return lo || (!hi && d != 0 && d <= uint32_t(qmask >> 1));
  }
};

// Sorted command values: the u64 (command | meta) alone, or (key-order
// path) with the command's packed 32-bit dot beside it (V3, 12 B), so the
// search and the graph read each command's dot in key order without a
// gather.
struct V3 {
  uint32_t x, y, z;  // u64 value (lo, hi), packed dot
  V3() = default;
  __host__ __device__ V3(int) : x(0), y(0), z(0) {}
};
__device__ __forceinline__ uint64_t vload(const uint64_t *v, uint32_t i) { return v[i]; }
__device__ __forceinline__ uint64_t vload(const V3 *v, uint32_t i) {
  const V3 t = v[i];
  return uint64_t(t.x) | (uint64_t(t.y) << 32);
}
__device__ __forceinline__ uint32_t vdot32(const uint64_t *, uint32_t) { return 0u; }
__device__ __forceinline__ uint32_t vdot32(const V3 *v, uint32_t i) { return v[i].z; }

// One workgroup per sort tile: packs each command's key, index and view
// records (k_view_records) into the sort input, and writes the tile's digit
// counts for the sort's first pass (sort_pairs_counted).
__global__ void __launch_bounds__(kThreads)
    k_cmd_pack(uint32_t n, CmdMeta cm, const uint32_t *__restrict__ key32,
               const uint32_t *__restrict__ rec, uint32_t *__restrict__ kw,
               uint64_t *__restrict__ val, uint32_t *__restrict__ counts, uint32_t dmask) {
  // unit x = c << us | s (us = 0: a command): view j's record is element
  // (c·fq + j)·k + s of the element logs' layout
  const uint32_t kmask1 = (1u << cm.us) - 1u;
  __shared__ uint32_t s_h[256];
  s_h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * uint32_t(kTile), end = min(n, base + uint32_t(kTile));
  for (uint32_t x = base + threadIdx.x; x < end; x += kThreads) {
    const uint32_t key = key32[x];
    uint64_t m = 0;
    for (uint32_t j = 0; j < cm.fq; j++) {
      const uint32_t r =
          rec[((size_t(x >> cm.us) * cm.fq + j) << cm.us) | (x & kmask1)];
      m |= ((uint64_t(r >> kRecT) << cm.qb) | (r & cm.qmask)) << (j * cm.vb);
    }
    val[x] = uint64_t(x) | (m << cm.cb);
    kw[x] = key | uint32_t((m >> (64 - cm.cb)) << cm.kb);
    atomicAdd(&s_h[key & dmask], 1u);
  }
  __syncthreads();
  if (threadIdx.x <= dmask) counts[size_t(blockIdx.x) * (dmask + 1) + threadIdx.x] = s_h[threadIdx.x];
}

// The key-order path's sort input, produced inside the sort's first scatter
// (sort_pairs_counted_src): element x's key word (as k_cmd_pack packs it)
// and V3 value (k_cmd_pack's u64 and the command's packed dot), computed from
// the command's key, view records and packed dot as the scatter loads the
// element (the packed arrays are never written: 2 x 16 B per command less
// traffic).  k_key_counts writes the tile digit
// counts of that first pass.
struct PackSrc {
  CmdMeta cm;
  const uint32_t *key32, *rec, *dot32;
  __device__ __forceinline__ void get(uint32_t x, uint32_t &kw, V3 &o) const {
    const uint32_t key = key32[x];
    uint64_t m = 0;
    uint32_t rr[3];
    if (cm.fq == 3) {  // the command's three records in one 12-B load
      const auto t = *reinterpret_cast<const HIP_vector_type<uint32_t, 3> *>(rec + size_t(x) * 3);
      rr[0] = t.x;
      rr[1] = t.y;
      rr[2] = t.z;
    } else {
      for (uint32_t j = 0; j < cm.fq; j++) rr[j] = rec[size_t(x) * cm.fq + j];
    }
    for (uint32_t j = 0; j < cm.fq; j++) {
      const uint32_t r = rr[j];
      m |= ((uint64_t(r >> kRecT) << cm.qb) | (r & cm.qmask)) << (j * cm.vb);
    }
    const uint64_t v = uint64_t(x) | (m << cm.cb);
    o.x = uint32_t(v);
    o.y = uint32_t(v >> 32);
    o.z = dot32[x];
    kw = key | uint32_t((m >> (64 - cm.cb)) << cm.kb);
  }
};
__global__ void __launch_bounds__(kThreads)
    k_key_counts(uint32_t n, const uint32_t *__restrict__ key32, uint32_t *__restrict__ counts,
                 uint32_t dmask) {
  __shared__ uint32_t s_h[256];
  s_h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * uint32_t(kTile), end = min(n, base + uint32_t(kTile));
  for (uint32_t x = base + threadIdx.x; x < end; x += kThreads) atomicAdd(&s_h[key32[x] & dmask], 1u);
  __syncthreads();
  if (threadIdx.x <= dmask) counts[size_t(blockIdx.x) * (dmask + 1) + threadIdx.x] = s_h[threadIdx.x];
}

// One thread per command in (key, command) order, a 1024-command tile staged
// in LDS with kSrchHalo neighbours on either side, unpacked: key, command and
// the arrival position at each replica (kNoArr if the replica does not
// process it), stored shifted to the top of the word so that arrival
// differences wrap modulo 2^qb by themselves.  A scan that leaves the staged
// span continues on the packed global arrays.  Per view j the predecessor is
// the key's latest arrival at replica r_j before the command
// (SequentialKeyDeps::add_cmd, sequential.rs:72-104).  Backward, every
// r_j-command arriving earlier is a candidate; one c' with c' + W below the
// best candidate so far arrives before it and cannot win, nor can anything
// further back, so the scan stops once that holds for every view.  Forward,
// commands up to c + W may still arrive earlier; nothing beyond c + W does.
//
// Tails (latest_deps becomes the key's last arrival, :88-95) need no forward
// search: in the arrival order of one (key, replica) every element but the
// last is the predecessor of the next one, so an element is the tail iff no
// element names it.  Each command marks its views' predecessors: in LDS when
// the predecessor is a core command of the tile, else in `mrem` (one byte of
// replica bits per sorted position, atomic OR); k_cmd_tails combines both.
//
// Codes: with `rec` set (fq <= 3), each command's (command, codes) record is
// written into its command region's slice of `rec` (c >> kRegShift; the
// tile's run of each region claimed from the region's cursor `rcur`), and
// k_code_scatter moves the records region by region, so the scattered code stores of a moment stay in
// a cache-sized slice of the code array (a random 12-B store per command over
// the whole array ran at 4.6 ms per 100M commands, confined to 4M-command
// regions at 1.7 ms: tools/scatter_bench.hip, profiles/r05_scatter_bench.jsonl).
constexpr int kSrchHalo = 128;
constexpr int kSrchMaxRep = 8;  // replicas (logs) of the command-level path
constexpr uint32_t kNoArr = ~0u;
constexpr uint32_t kRegShift = 22;   // code regions of 4M commands (48 MB of codes)
constexpr uint32_t kMaxRegions = 128;  // units < 2^29 at 4M per region (C4: 24 regions)

// Per-view scan state; `bc` is the best candidate's command + 1 (0: none),
// `bp` its sorted position.  Arrivals are shifted left by 32 - qb, so `close`
// -- the candidate reaches the replica first, when the two commands are
// within W of each other -- is one wrapping subtraction and one compare
// (CmdMeta::before).
struct ViewScan {
  uint32_t c, tq, H;
  uint32_t bc = 0, bt = 0, bp = 0;
  __device__ __forceinline__ static bool close(uint32_t d, uint32_t H) { return d - 1u < H; }
  // backward neighbour: command cc (ccW1 = cc + W + 1, far = cc + W < c),
  // arrival t at the view's replica, sorted position p
  __device__ __forceinline__ void back(bool sk, uint32_t cc, uint32_t ccW1, bool far, uint32_t t, uint32_t p) {
    const bool earlier = sk & (t != kNoArr) & (far | close(tq - t, H));
    const bool better = earlier & ((bc == 0u) | (!(ccW1 < bc) & close(t - bt, H)));
    bt = better ? t : bt;
    bc = better ? cc + 1u : bc;
    bp = better ? p : bp;
  }
  // forward neighbour (c < cc <= c + W)
  __device__ __forceinline__ void fwd(bool sk, uint32_t cc, uint32_t W, uint32_t t, uint32_t p) {
    const bool earlier = sk & (t != kNoArr) & close(tq - t, H);
    const bool better = earlier & ((bc == 0u) | (bc + W <= cc) | close(t - bt, H));
    bt = better ? t : bt;
    bc = better ? cc + 1u : bc;
    bp = better ? p : bp;
  }
};

// KO (key-order path, VS = V3): the key-order graph's edges are each
// command's in-batch predecessors as signed 8-bit distances in sorted
// position (pe8[i], byte j: i - position, 0 = none; key-order edges span a
// handful of positions, C4 <= 20), with -128 escaping to the full position +
// 1 in pcode[i·FQ + j]; the region records carry the predecessors' packed
// dots instead of their commands (the union then needs no gather), and the
// command's own packed dot goes to pd32[i].
template <uint32_t FQ, int TH, class VS, bool KO>
__global__ void __launch_bounds__(TH)
    k_cmd_search(uint32_t n, CmdMeta cm, uint32_t K, uint32_t np, const uint32_t *__restrict__ kws,
                 const VS *__restrict__ vals, const uint64_t *__restrict__ latest,
                 uint32_t *__restrict__ code, uint4 *__restrict__ rec,
                 uint32_t *__restrict__ rcur, uint8_t *__restrict__ tailm,
                 uint32_t *__restrict__ mrem, uint32_t *__restrict__ pcode,
                 uint32_t *__restrict__ pd32, uint32_t *__restrict__ pe8) {
  constexpr int kSpan = TH + 2 * kSrchHalo;
  __shared__ uint32_t s_key[kSpan], s_c[kSpan];
  __shared__ uint32_t s_q[kSpan * kSrchMaxRep];
  __shared__ uint32_t s_d[KO ? kSpan : 1];
  __shared__ uint8_t s_mark[TH * kSrchMaxRep];
  __shared__ uint32_t s_reg[kMaxRegions], s_rb[kMaxRegions];
  const uint32_t tid = threadIdx.x, core = blockIdx.x * TH, i = core + tid;
  const uint32_t lo = core > uint32_t(kSrchHalo) ? core - kSrchHalo : 0u;
  const uint32_t hi = min(n, core + TH + kSrchHalo);
  const uint32_t span = hi - lo;
  const uint32_t qs = 32u - cm.qb;  // arrival shift
  for (uint32_t x = tid; x < span * np; x += TH) s_q[x] = kNoArr;
  for (uint32_t x = tid; x < TH * np; x += TH) s_mark[x] = 0;
  if (tid < kMaxRegions) s_reg[tid] = 0;
  __syncthreads();
  for (uint32_t x = tid; x < span; x += TH) {
    const uint32_t kw = kws[lo + x];
    const uint64_t v = vload(vals, lo + x);
    const uint64_t m = cm.meta(kw, v);
    s_key[x] = kw & cm.kmask;
    s_c[x] = uint32_t(v & cm.cmask);
    if constexpr (KO) s_d[x] = vdot32(vals, lo + x);
#pragma unroll
    for (uint32_t j = 0; j < FQ; j++) s_q[x * np + cm.rep(m, j)] = cm.arr(m, j) << qs;
  }
  // the command's slot among the tile's records of its region (rec mode)
  uint32_t reg = 0, rank = 0;
  if (rec && i < n) {
    reg = uint32_t(vload(vals, i) & cm.cmask) >> cm.rsh;
    rank = atomicAdd(&s_reg[reg], 1u);
  }
  __syncthreads();
  // Region r's records fill rec[r << kRegShift, ...) exactly (a region holds
  // 2^kRegShift commands), in any order: the tile claims its run of each
  // region from the region's cursor, one atomic per (tile, region), issued
  // now and read after the scans' barrier
  if (rec && tid < uint32_t(kMaxRegions) && s_reg[tid])
    s_rb[tid] = (tid << cm.rsh) + atomicAdd(&rcur[tid], s_reg[tid]);
  const bool act = i < n;
  const uint32_t me = i - lo;
  const uint32_t W = cm.W, H = uint32_t(cm.qmask >> 1) << qs;
  uint32_t key = 0, c = 0;
  ViewScan vs[FQ];
  uint32_t rr[FQ];
  if (act) {
    key = s_key[me];
    c = s_c[me];
    const uint64_t m0 = cm.meta(kws[i], vload(vals, i));
#pragma unroll
    for (uint32_t j = 0; j < FQ; j++) {
      rr[j] = cm.rep(m0, j);
      vs[j].c = c;
      vs[j].H = H;
      vs[j].tq = cm.arr(m0, j) << qs;
    }
    // backward: the staged span, then global memory (a neighbour outside the
    // span is unpacked from the packed arrays); every view's state moves on
    // each neighbour, and the scan ends when no view can still improve
    // (tried: batches of 4 neighbours with the batch's LDS loads issued
    // together: 4.15 against 3.2 ms at C4, the extra steps cost more VALU
    // than the waits they hid)
    bool go = true;
    for (uint32_t x = me; go && x > 0;) {
      x--;
      const bool sk = s_key[x] == key;
      const uint32_t cc = s_c[x], ccW1 = cc + W + 1u;
      const bool far = cc + W < c;
      uint32_t lim = ~0u;
#pragma unroll
      for (uint32_t j = 0; j < FQ; j++) {
        vs[j].back(sk, cc, ccW1, far, s_q[x * np + rr[j]], lo + x);
        lim = min(lim, vs[j].bc);
      }
      go = sk & !(ccW1 < lim);
    }
    for (uint32_t ip = lo; go && ip-- > 0;) {
      const uint32_t kw = kws[ip];
      const uint64_t v = vload(vals, ip);
      const uint64_t m = cm.meta(kw, v);
      const bool sk = (kw & cm.kmask) == key;
      const uint32_t cc = uint32_t(v & cm.cmask), ccW1 = cc + W + 1u;
      const bool far = cc + W < c;
      uint32_t lim = ~0u;
#pragma unroll
      for (uint32_t j = 0; j < FQ; j++) {
        uint32_t t = kNoArr;
        if (cm.find(m, rr[j], &t)) t <<= qs;
        vs[j].back(sk, cc, ccW1, far, t, ip);
        lim = min(lim, vs[j].bc);
      }
      go = sk & !(ccW1 < lim);
    }
    // forward, up to c + W
    go = true;
    for (uint32_t x = me + 1; go && x < span; x++) {
      const uint32_t cc = s_c[x];
      const bool sk = (s_key[x] == key) & (cc <= c + W);
#pragma unroll
      for (uint32_t j = 0; j < FQ; j++) vs[j].fwd(sk, cc, W, s_q[x * np + rr[j]], lo + x);
      go = sk;
    }
    for (uint32_t ip = hi; go && ip < n; ip++) {
      const uint32_t kw = kws[ip];
      const uint64_t v = vload(vals, ip);
      const uint64_t m = cm.meta(kw, v);
      const uint32_t cc = uint32_t(v & cm.cmask);
      const bool sk = ((kw & cm.kmask) == key) & (cc <= c + W);
#pragma unroll
      for (uint32_t j = 0; j < FQ; j++) {
        uint32_t t = kNoArr;
        if (cm.find(m, rr[j], &t)) t <<= qs;
        vs[j].fwd(sk, cc, W, t, ip);
      }
      go = sk;
    }
    // mark each view's predecessor: it is not the tail of that replica
#pragma unroll
    for (uint32_t j = 0; j < FQ; j++) {
      if (vs[j].bc == 0u) continue;
      const uint32_t p = vs[j].bp;
      if (p >= core && p < core + uint32_t(TH)) {
        s_mark[(p - core) * np + rr[j]] = 1;
      } else {
        atomicOr(&mrem[p >> 2], (1u << rr[j]) << ((p & 3u) * 8u));
      }
    }
  }
  __syncthreads();
  uint32_t cds[FQ];
  if (act) {
    uint32_t msk = 0, e8 = 0;
#pragma unroll
    for (uint32_t j = 0; j < FQ; j++) {
      if (vs[j].bc != 0u) {
        if constexpr (KO) {
          // the predecessor's packed dot (staged, or beyond the span)
          const uint32_t p = vs[j].bp;
          cds[j] = p >= lo && p < hi ? s_d[p - lo] : vdot32(vals, p);
          const int d = int(i) - int(p);
          if (d >= -127 && d <= 127) {
            e8 |= (uint32_t(d) & 0xFFu) << (8 * j);
          } else {
            e8 |= 0x80u << (8 * j);
            pcode[size_t(i) * FQ + j] = p + 1u;
          }
        } else {
          cds[j] = ((vs[j].bc - 1u) >> cm.us) + 1u;  // in-batch: the command's vid + 1
        }
      } else {
        const uint64_t xl = latest[uint64_t(rr[j] + 1) * K + key];
        cds[j] = xl ? (0x80000000u | uint32_t(xl - kLogFlag)) : 0u;
      }
      msk |= s_mark[tid * np + rr[j]] ? 0u : 1u << j;
    }
    tailm[i] = uint8_t(msk);
    if constexpr (KO) {
      pd32[i] = s_d[me];
      pe8[i] = e8;
    }
    if (!rec) {
      uint32_t *o = code + size_t(c) * FQ;
      if constexpr (FQ == 4) {
        *reinterpret_cast<uint4 *>(o) = make_uint4(cds[0], cds[1], cds[2], cds[3]);
      } else {
#pragma unroll
        for (uint32_t j = 0; j < FQ; j++) o[j] = cds[j];
      }
    }
  }
  if (!rec) return;  // uniform over the grid
  if (act) {
    uint4 o = make_uint4(c, 0u, 0u, 0u);
    if constexpr (FQ >= 1) o.y = cds[0];
    if constexpr (FQ >= 2) o.z = cds[1];
    if constexpr (FQ >= 3) o.w = cds[2];
    rec[s_rb[reg] + rank] = o;
  }
}

// The (command, codes) records, region-major -> their command slots of the
// code array (fq <= 3).  Blocks run in order, so the stores of a moment land
// in one or two regions' slices of `code` (a few tens of MB: cache-resident).
template <uint32_t FQ>
__global__ void __launch_bounds__(256)
    k_code_scatter(uint32_t n, const uint4 *__restrict__ rec, uint32_t *__restrict__ code) {
  GRID_STRIDE(i, n) {
    const uint4 o = rec[i];
    uint32_t *d = code + size_t(o.x) * FQ;
    if constexpr (FQ == 3) {
      *reinterpret_cast<HIP_vector_type<uint32_t, 3> *>(d) = HIP_vector_type<uint32_t, 3>(o.y, o.z, o.w);
    } else {
      d[0] = o.y;
      if constexpr (FQ >= 2) d[1] = o.z;
    }
  }
}

// the tails become the replicas' latest entries (after every head's read):
// view j of a sorted command is its replica's tail iff neither the tile
// (tailm) nor another tile (mrem) marked it as some element's predecessor
template <class VS>
__global__ void k_cmd_tails(uint32_t n, CmdMeta cm, uint32_t K, const uint32_t *__restrict__ kws,
                            const VS *__restrict__ vals, const uint8_t *__restrict__ tailm,
                            const uint8_t *__restrict__ mrem, uint64_t *__restrict__ latest,
                            uint64_t log_base) {
  // sixteen commands' tail masks per load (the buffer is padded to 16
  // bytes): most are zero, and the side stream runs this with few waves per
  // CU, so each thread's loop is bound by its loads' latency
  const uint32_t nw = (n + 15) / 16;
  GRID_STRIDE(w, nw) {
    const uint4 m16 = reinterpret_cast<const uint4 *>(tailm)[w];
    const uint32_t mw[4] = {m16.x, m16.y, m16.z, m16.w};
#pragma unroll
    for (int h = 0; h < 4; h++) {
      uint32_t msk4 = mw[h];
      while (msk4) {
        const uint32_t b = uint32_t(__builtin_ctz(msk4)) >> 3;
        const uint32_t i = 16 * w + 4 * h + b;
        const uint32_t msk = (msk4 >> (8 * b)) & 0xFFu;
        msk4 &= ~(0xFFu << (8 * b));
        if (i >= n) break;
        const uint32_t rm = mrem[i];
        const uint32_t kw = kws[i];
        const uint64_t v = vload(vals, i);
        const uint64_t m = cm.meta(kw, v);
        const uint32_t key = kw & cm.kmask, c = uint32_t(v & cm.cmask);
        for (uint32_t j = 0; j < cm.fq; j++) {
          const uint32_t r = cm.rep(m, j);
          if ((msk & (1u << j)) && !(rm & (1u << r)))
            latest[uint64_t(r + 1) * K + key] = kLogFlag | (log_base + (c >> cm.us));
        }
      }
    }
  }
}

// ---- the key-order path (one key per command, fast quorums of 2-3, dots
// packable in 31 bits; EngineDevice::cmd_views_keyorder).  Every dependency
// joins two commands of one key, so the graph is a disjoint union of per-key
// graphs and the (key, command) sort order is as good a vertex order as the
// arrival order: ready times, SCCs, depths and ties map monotonically
// between the two inside a key.  Ordered by key, every edge spans a handful
// of positions (C4: <= 20, maximum excess H(v) - v 65 against 728 in
// arrival order at 5M commands, tools/keyorder_stats.py), so the tile
// kernel runs with no certificate failures, its per-key execution order is
// the per-key sequence itself (groups never straddle keys), and only the
// per-command outputs travel back to command order.

// The key-order path's committed deps (QuorumDeps union, quorum.rs:28-98)
// straight from the search's region records: each record's fq entries (0
// none, 0x80000000 | x an earlier batch's log reference, else an in-batch
// packed dot) as dots, sorted and deduplicated into the command's row of fq
// slots, empty slots holding the reserved all-ones dot (stage_logs rejects
// it as a dot).  One pass: no command-order entry array, count pass or scan
// (pack_dep_rows builds the ABI's CSR from the rows when results() asks).
// Records are region-major, so the row stores of a moment stay in one or
// two regions' slices of `rows`.  An external dot equal to an in-batch one
// (a dot of the batch repeating an earlier batch's) sets *err, as the
// general union reports it.
// 16 bytes at 8-byte alignment (one global_store_dwordx4)
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(8)));
// Rows of u64 dots, or of the batch's 32-bit packed dots (src << sb | seq,
// order-preserving; ~0u, never a packed dot of <= 31 bits, for an empty
// slot) when every dot of the log packs that way (EngineDevice::rows32_ok):
// half the scattered bytes beside the tile kernel, unpacked by results().
template <class RT>
__device__ __forceinline__ RT row_dot(uint32_t e, const uint64_t *__restrict__ dlog, int sb,
                                      uint32_t *__restrict__ err) {
  if constexpr (sizeof(RT) == 8) {
    return e == 0u ? ~0ull
           : (e & 0x80000000u) ? dlog[e & 0x7FFFFFFFu]
                               : (uint64_t(e >> sb) << 56) | (e & ((1u << sb) - 1));
  } else {
    if (e == 0u) return ~0u;
    if (!(e & 0x80000000u)) return e;  // an in-batch dot, packed already
    const uint64_t d = dlog[e & 0x7FFFFFFFu];
    const uint64_t src = d >> 56, seq = d & 0x00FFFFFFFFFFFFFFull;
    if (seq >> sb || (src << sb) >> 31) atomicOr(err, 2u);  // (the host checked the log)
    return uint32_t((src << sb) | seq);
  }
}
template <uint32_t FQ, class RT = uint64_t>
__device__ __forceinline__ void row_place_one(const uint4 o, const uint64_t *__restrict__ dlog,
                                              int sb, RT *__restrict__ rows,
                                              uint32_t *__restrict__ err) {
  constexpr RT kNone = RT(~RT(0));
  const uint32_t e[3] = {o.y, o.z, o.w};
  RT r[FQ];
  uint32_t codes = 0;
#pragma unroll
  for (uint32_t j = 0; j < FQ; j++) {
    bool dup = e[j] == 0u;
#pragma unroll
    for (uint32_t q = 0; q < j; q++) dup |= e[q] == e[j];
    codes += dup ? 0u : 1u;
    r[j] = row_dot<RT>(e[j], dlog, sb, err);
  }
#pragma unroll
  for (uint32_t a = 0; a < FQ; a++)
#pragma unroll
    for (uint32_t b2 = a + 1; b2 < FQ; b2++) {
      const RT x = r[a], y = r[b2];
      r[a] = x < y ? x : y;
      r[b2] = x < y ? y : x;
    }
  // the unique dots first, then the sentinel
  RT w[FQ];
  uint32_t m = 0;
#pragma unroll
  for (uint32_t j = 0; j < FQ; j++) w[j] = kNone;
#pragma unroll
  for (uint32_t j = 0; j < FQ; j++)
    if (r[j] != kNone && (j == 0 || r[j] != r[j - 1])) {
#pragma unroll
      for (uint32_t q = 0; q < FQ; q++)
        if (q == m) w[q] = r[j];
      m++;
    }
  if (m != codes) atomicOr(err, 1u);
  // the row in as few store instructions as it takes (a scattered store
  // costs the address unit a line per lane whatever its width, and the
  // tile kernel beside this one waits on the same unit)
  RT *d = rows + size_t(o.x) * FQ;
  if constexpr (FQ == 3 && sizeof(RT) == 4) {
    *reinterpret_cast<HIP_vector_type<uint32_t, 3> *>(d) =
        HIP_vector_type<uint32_t, 3>(w[0], w[1], w[2]);
  } else if constexpr (FQ == 3) {
    const u32x4u lo4{uint32_t(w[0]), uint32_t(w[0] >> 32), uint32_t(w[1]), uint32_t(w[1] >> 32)};
    *reinterpret_cast<u32x4u *>(d) = lo4;
    d[2] = w[2];
  } else {
#pragma unroll
    for (uint32_t j = 0; j < FQ; j++) d[j] = w[j];
  }
}
// One record per thread per trip: eight per trip (loads issued together)
// doubled it beside the tile kernel, 3.1 -> 7.0 ms, and slowed the tile
// kernel 5.3 -> 7.5 ms -- more random row stores in flight congest the
// write path the tile kernel's own stores wait on.  (Nontemporal row stores,
// here or for the tile kernel's outputs, measured no different: 12.28 ms per
// C4 step against 12.26-12.32.)
template <uint32_t FQ, class RT = uint64_t>
__global__ void __launch_bounds__(256)
    k_row_place(uint32_t n, const uint4 *__restrict__ rec, const uint64_t *__restrict__ dlog,
                int sb, RT *__restrict__ rows, uint32_t *__restrict__ err) {
  GRID_STRIDE(i, n) row_place_one<FQ, RT>(rec[i], dlog, sb, rows, err);
}

// Rows -> CSR (results(), outside the run): the length of every row, then
// (after a scan) each row's dots at its offset.
__global__ void k_rows_count(uint32_t n, uint32_t fq, const uint64_t *__restrict__ rows,
                             uint32_t *__restrict__ cnt) {
  GRID_STRIDE(i, n) {
    uint32_t c = 0;
    for (uint32_t j = 0; j < fq; j++) c += rows[size_t(i) * fq + j] != ~0ull;
    cnt[i] = c;
  }
}
__global__ void k_rows32_count(uint32_t n, uint32_t fq, const uint32_t *__restrict__ rows,
                               uint32_t *__restrict__ cnt) {
  GRID_STRIDE(i, n) {
    uint32_t c = 0;
    for (uint32_t j = 0; j < fq; j++) c += rows[size_t(i) * fq + j] != ~0u;
    cnt[i] = c;
  }
}
__global__ void k_rows32_compact(uint32_t n, uint32_t fq, const uint32_t *__restrict__ rows, int sb,
                                 const uint32_t *__restrict__ off, uint64_t *__restrict__ dep) {
  GRID_STRIDE(i, n) {
    const uint32_t o = off[i], c = off[i + 1] - o;
    for (uint32_t j = 0; j < c; j++) {
      const uint32_t x = rows[size_t(i) * fq + j];
      dep[o + j] = (uint64_t(x >> sb) << 56) | (x & ((1u << sb) - 1));
    }
  }
}
__global__ void k_rows_compact(uint32_t n, uint32_t fq, const uint64_t *__restrict__ rows,
                               const uint32_t *__restrict__ off, uint64_t *__restrict__ dep) {
  GRID_STRIDE(i, n) {
    const uint32_t o = off[i], c = off[i + 1] - o;
    for (uint32_t j = 0; j < c; j++) dep[o + j] = rows[size_t(i) * fq + j];
  }
}

// Command order: exec_rank[c] = start(t) + rank with t the group's ready
// time in command order and start(t) = t - straddle(t) (ss = exclusive scan
// of the difference array: straddle(t) = ss[t + 1]); a vertex outside a
// multi-member group (d[c + 1] == 0) is its group's root with rank 0 and
// its own label.
// The straddle difference array (graph_tile.hip, key-order outputs): +1 at
// c(u) + 1 from each raised member u of a ready group (H(u) > u), -(size -
// 1) at c(t) + 1 from each multi-member root t -- no slot written twice,
// d[c + 1] != 0 exactly for the vertices of multi-member groups -- so that
// straddle(t) = vertices before t whose group runs at or after t.  Also the
// executed clock over the batch's dots (per source: max sequence, count).
__global__ void __launch_bounds__(256)
    k_ko_final(uint32_t n, const uint32_t *__restrict__ diff, const uint4 *__restrict__ hl,
               const uint32_t *__restrict__ ss, const uint64_t *__restrict__ dot,
               uint64_t *__restrict__ label, uint32_t *__restrict__ rank,
               unsigned long long *__restrict__ smx, unsigned int *__restrict__ scnt) {
  __shared__ unsigned long long s_mx[256];
  __shared__ unsigned int s_cnt[256];
  SrcAcc acc;
  acc.init(s_mx, s_cnt);
  __syncthreads();
  // four commands per thread per trip, each dependent level's loads issued
  // together (diff / dot / ss, then hl, then the root's ss; two per trip,
  // 8 waves per SIMD instead of 5: 832-887 against 821-831 us, r05ku)
  constexpr int kU = 4;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t c0 = blockIdx.x * blockDim.x + threadIdx.x; c0 < n; c0 += kU * stride) {
    uint64_t dc[kU];
    uint32_t df[kU], sc[kU], sr[kU];
    uint4 r[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint32_t c = c0 + u * stride;
      df[u] = 0u;
      if (c < n) {
        dc[u] = dot[c];
        df[u] = diff[c + 1];
        sc[u] = ss[c + 1];
      }
    }
#pragma unroll
    for (int u = 0; u < kU; u++)
      if (df[u]) r[u] = hl[c0 + u * stride];
#pragma unroll
    for (int u = 0; u < kU; u++)
      if (df[u]) sr[u] = ss[r[u].x + 1];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint32_t c = c0 + u * stride;
      if (c >= n) break;
      acc.add(dc[u]);
      if (df[u]) {
        rank[c] = r[u].x - sr[u] + r[u].y;
        label[c] = uint64_t(r[u].z) | (uint64_t(r[u].w) << 32);
      } else {
        rank[c] = c - sc[u];
        label[c] = dc[u];
      }
    }
  }
  acc.commit(smx, scnt);
}

// Certificate failure on the key-order graph: its in-batch edges back to
// command order as command-index references (the general path's encoding)
// over the command-order entries (which hold packed dots there; external
// and empty entries stay), then the general union + graph run as for any
// batch.
template <uint32_t FQ>
__global__ void k_pcode_to_vid(uint32_t n, const V3 *__restrict__ vals, uint64_t cmask,
                               const uint32_t *__restrict__ pe8, const uint32_t *__restrict__ pcode,
                               uint32_t *__restrict__ code) {
  GRID_STRIDE(p, n) {
    const uint32_t c = uint32_t(vload(vals, p) & cmask);
    const uint32_t e8 = pe8[p];
#pragma unroll
    for (uint32_t j = 0; j < FQ; j++) {
      const int d = int(int8_t(uint8_t(e8 >> (8 * j))));
      if (d == 0) continue;
      const uint32_t q = d == -128 ? pcode[size_t(p) * FQ + j] - 1u : uint32_t(int(p) - d);
      code[size_t(c) * FQ + j] = uint32_t(vload(vals, q) & cmask) + 1u;
    }
  }
}

// Element dependency code (one u64 per element, command-major position e):
// 0 = none, in-batch vid + 1 (< 2^48) for the previous element of its
// segment, else the persistent latest entry of the segment at the head (a
// dot, >= 2^56, or a command-log reference, [2^48, 2^56)).
template <class KT>
__global__ void k_prev_engine(uint32_t M, const KT *__restrict__ ks, const uint32_t *__restrict__ vs,
                              int tb, uint32_t per_cmd, const uint64_t *__restrict__ latest,
                              uint64_t lmul, uint64_t lmask, uint64_t *__restrict__ dep_code,
                              uint32_t *__restrict__ sorted_vid) {
  GRID_STRIDE(j, M) {
    const uint32_t e = vs[j];
    const KT seg = ks[j] >> tb;
    const bool head = j == 0 || (ks[j - 1] >> tb) != seg;
    // the segment id is the latest-table slot: key, or replica * K + key
    dep_code[e] = head ? latest[(uint64_t(seg) * lmul) & lmask] : uint64_t(vs[j - 1] / per_cmd) + 1;
    if (sorted_vid) sorted_vid[j] = e / per_cmd;
  }
}

// Segment tails become the latest entries (sequential.rs:88-95), in a launch
// of their own so that every head of k_prev_engine has read the old value:
// the command's dot (replica views) or its command-log reference.
template <class KT>
__global__ void k_tail_engine(uint32_t M, const KT *__restrict__ ks, const uint32_t *__restrict__ vs,
                              int tb, uint32_t per_cmd, uint64_t *__restrict__ latest,
                              uint64_t lmul, uint64_t lmask, const uint64_t *__restrict__ bdot,
                              uint64_t log_base) {
  GRID_STRIDE(j, M) {
    const KT seg = ks[j] >> tb;
    if (j + 1 == M || (ks[j + 1] >> tb) != seg) {
      const uint32_t cmd = vs[j] / per_cmd;
      latest[(uint64_t(seg) * lmul) & lmask] = bdot ? bdot[cmd] : (kLogFlag | (log_base + cmd));
    }
  }
}

// decode an element's dependency code: in-batch vid (true) or external value
// Element dependency codes, decoded by the union:
//  u64 (single view, k > 1): 0 none, in-batch vid + 1 (< 2^48), else the
//      segment head's latest entry: a dot (>= 2^56) or a command-log
//      reference (kLogFlag | position, [2^48, 2^56));
//  u32 (replica views): 0 none, vid + 1 (< 2^31), else 0x80000000 | the log
//      position of the head's latest entry (views' latest tables hold log
//      references only).
// A log reference into the batch itself (written by an earlier chunk of the
// batch's replica logs) is an in-batch dependency.  Returns 1 = in batch
// (*v), 2 = external dot (*x), 0 = none.
__device__ __forceinline__ int decode_dep(uint64_t c, uint32_t *v, uint64_t *x,
                                          const uint64_t *__restrict__ dlog, uint64_t bbase,
                                          uint32_t n) {
  if (c == 0) return 0;
  if (c < kLogFlag) {
    *v = uint32_t(c - 1);
    return 1;
  }
  if (is_log_ref(c)) {
    const uint64_t pos = c - kLogFlag;
    if (pos >= bbase && pos < bbase + n) {
      *v = uint32_t(pos - bbase);
      return 1;
    }
    *x = dlog[pos];
    return 2;
  }
  *x = c;
  return 2;
}
__device__ __forceinline__ int decode_dep(uint32_t c, uint32_t *v, uint64_t *x,
                                          const uint64_t *__restrict__ dlog, uint64_t bbase,
                                          uint32_t n) {
  if (c == 0) return 0;
  if (!(c & 0x80000000u)) {
    *v = c - 1;
    return 1;
  }
  const uint64_t pos = c & 0x7FFFFFFFu;
  if (pos >= bbase && pos < bbase + n) {
    *v = uint32_t(pos - bbase);
    return 1;
  }
  *x = dlog[pos];
  return 2;
}

__device__ __forceinline__ uint32_t sort_unique_u64(uint64_t *a, uint32_t n) {
  for (uint32_t i = 1; i < n; i++) {
    const uint64_t x = a[i];
    uint32_t j = i;
    while (j > 0 && a[j - 1] > x) {
      a[j] = a[j - 1];
      j--;
    }
    a[j] = x;
  }
  uint32_t w = n ? 1 : 0;
  for (uint32_t i = 1; i < n; i++)
    if (a[i] != a[w - 1]) a[w++] = a[i];
  return w;
}

// k_cmd_engine for rows of at most kRegSlots slots, in registers: every slot
// is read into a fixed register position (absent = all ones), a bitonic
// network sorts the 16 dots, and the unique ones stream out.  (The general
// path's insertion sort runs on the global row: a dependent load/store chain
// per step; C5's 12-slot rows spent 15 ms there.)  A dot is never all ones
// (ProcessId 255 with sequence 2^56 - 1), so the sentinel cannot collide.
constexpr uint32_t kRegSlots = 16;
template <uint32_t kRegSlots, class CT>
__device__ __forceinline__ void cmd_union_regs(
    uint32_t i, uint32_t S, const uint64_t *__restrict__ dot,
    const CT *__restrict__ dep_code, const uint64_t *__restrict__ dlog,
    const uint64_t *__restrict__ frontier, uint64_t *__restrict__ dep_dot,
    uint32_t *__restrict__ dep_cnt, uint32_t *__restrict__ dst, uint8_t *__restrict__ blocked0,
    uint32_t *nblocked, uint32_t *__restrict__ nv_out, uint64_t bbase, uint32_t n,
    const uint32_t *__restrict__ out_off, uint32_t *__restrict__ err, uint32_t vbase,
    bool edges_at_deps, uint32_t &fwd, const uint32_t *__restrict__ dot32, int sb32) {
  uint64_t r[kRegSlots];
  uint32_t vv[kRegSlots];
  bool missing = false;
#pragma unroll
  for (uint32_t t = 0; t < kRegSlots; t++) {
    r[t] = ~0ull;
    vv[t] = ~0u;
    if (t < S) {
      uint64_t x = 0;
      uint32_t v = 0;
      const int kind =
          decode_dep(dep_code[size_t(i) * S + t], &v, &x, dlog, bbase, n);
      if (kind == 1) {
        vv[t] = v;
      } else if (kind == 2) {
        r[t] = x;
        if ((x & 0x00FFFFFFFFFFFFFFull) > frontier[x >> 56]) missing = true;
      }
    }
  }
  if (blocked0) blocked0[i] = missing;
  if (missing) atomicAdd(nblocked, 1u);
  {
  // in-batch deps: one dot gather per distinct vid (the fast-quorum
  // members' reports often name the same previous command)
#pragma unroll
  for (uint32_t t = 0; t < kRegSlots; t++) {
    bool dup = vv[t] == ~0u;
#pragma unroll
    for (uint32_t q = 0; q < t; q++) dup |= vv[q] == vv[t];
    if (!dup) {
      if (dot32) {  // the packed copy: half the bytes per gathered line
        const uint32_t pd = dot32[vv[t]];
        r[t] = (uint64_t(pd >> sb32) << 56) | (pd & ((1u << sb32) - 1));
      } else {
        r[t] = dot[vv[t]];
      }
    }
  }
  // bitonic sort of the 16 register slots, ascending
#pragma unroll
  for (uint32_t kk = 2; kk <= kRegSlots; kk <<= 1) {
#pragma unroll
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (uint32_t a = 0; a < kRegSlots; a++) {
        const uint32_t b = a ^ j;
        if (b > a) {
          const uint64_t x = r[a], y = r[b];
          const bool sw = (a & kk) == 0 ? x > y : x < y;
          r[a] = sw ? y : x;
          r[b] = sw ? x : y;
        }
      }
    }
  }
  // out_off: the committed deps go straight to their CSR row (sized by
  // k_cmd_count); otherwise to a fixed-stride row, zero padded
  uint64_t *dd = out_off ? dep_dot + out_off[i] : dep_dot + size_t(i) * S;
  const uint32_t cap = out_off ? out_off[i + 1] - out_off[i] : S;
  uint32_t m = 0;
  uint64_t prev = 0;  // dots are never 0
#pragma unroll
  for (uint32_t t = 0; t < kRegSlots; t++) {
    if (r[t] != ~0ull && r[t] != prev) {
      if (m < cap) dd[m] = r[t];
      m++;
      prev = r[t];
    }
  }
  if (out_off) {
    if (m != cap) atomicOr(err, 1u);  // an in-batch dot repeated outside the batch
  } else {
    for (uint32_t q = m; q < S; q++) dd[q] = 0;
  }
  dep_cnt[i] = m;
  }
  // graph edges: a fixed-stride row of S, or (edges_at_deps) the command's
  // committed-deps row of the CSR (its in-batch deps are a subset), both
  // padded with the vertex itself (self loops are ignored); forward edges
  // (a dependency that arrived later) are counted for the graph stage
  uint32_t *ds = edges_at_deps ? dst + out_off[i] : dst + size_t(i) * S;
  const uint32_t ecap = edges_at_deps ? out_off[i + 1] - out_off[i] : S;
  uint32_t nv = 0;
#pragma unroll
  for (uint32_t t = 0; t < kRegSlots; t++) {
    if (vv[t] != ~0u) {
      bool dup = false;
#pragma unroll
      for (uint32_t q = 0; q < t; q++) dup |= vv[q] == vv[t];
      if (!dup) {
        if (nv < ecap) ds[nv] = vv[t];
        nv++;
        fwd += vv[t] > vbase + i;
      }
    }
  }
  for (uint32_t q = nv; q < ecap; q++) ds[q] = vbase + i;
  if (nv_out) nv_out[i] = nv;
}

// Per command: union of its fast-quorum members' element deps (vids and
// external dots), committed dep dots (sorted, fixed stride S), graph edges
// (vids, padded with the vertex itself), latest-table update at tails and the
// missing-dependency flag for external deps that are not executed.
template <class CT>
__global__ void k_cmd_engine(uint32_t n, uint32_t S, const uint64_t *__restrict__ dot,
                             const CT *__restrict__ dep_code,
                             const uint64_t *__restrict__ dlog,
                             const uint64_t *__restrict__ frontier,
                             uint64_t *__restrict__ dep_dot, uint32_t *__restrict__ dep_cnt,
                             uint32_t *__restrict__ dst, uint8_t *__restrict__ blocked0,
                             uint32_t *nblocked, uint32_t *__restrict__ nv_out,
                             uint64_t bbase, const uint32_t *__restrict__ out_off,
                             uint32_t *__restrict__ err, uint32_t vbase, uint32_t edges_at_deps,
                             unsigned long long *__restrict__ nfwd,
                             const uint32_t *__restrict__ dot32, int sb32) {
  // dot32 (or null): the batch's dots packed src << sb32 | seq, gathered
  // instead of the u64 dots
  // uniform: the register path, with a sorting network sized to the row
  const uint32_t cn = n;
  const bool ead = edges_at_deps != 0 && out_off != nullptr;
  uint32_t fwd = 0;
  if (S <= 4) {
    // XCD-contiguous blocks (grid a multiple of 8): workgroup b runs on XCD
    // b mod 8, which takes the b/8-th block of its own eighth of the
    // commands, so the recent dependencies' dot lines are gathered into the
    // L2 of the XCD that gathers them again
    const uint32_t nb = gridDim.x;
    const uint32_t lb = nb % 8 == 0 ? (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : blockIdx.x;
    for (size_t j = size_t(lb) * blockDim.x + threadIdx.x; j < cn; j += size_t(nb) * blockDim.x)
      cmd_union_regs<4>(uint32_t(j), S, dot, dep_code, dlog, frontier, dep_dot, dep_cnt, dst,
                        blocked0, nblocked, nv_out, bbase, n, out_off, err, vbase, ead, fwd, dot32,
                        sb32);
  } else if (S <= 8) {
    GRID_STRIDE(j, cn) {
      cmd_union_regs<8>(j, S, dot, dep_code, dlog, frontier, dep_dot, dep_cnt, dst, blocked0,
                        nblocked, nv_out, bbase, n, out_off, err, vbase, ead, fwd, dot32, sb32);
    }
  } else if (S <= kRegSlots) {
    GRID_STRIDE(j, cn) {
      cmd_union_regs<kRegSlots>(j, S, dot, dep_code, dlog, frontier, dep_dot, dep_cnt, dst,
                                blocked0, nblocked, nv_out, bbase, n, out_off, err, vbase, ead,
                                fwd, dot32, sb32);
    }
  } else {
    GRID_STRIDE(i, cn) {
      uint64_t *dd = dep_dot + size_t(i) * S;
      uint32_t *ds = dst + size_t(i) * S;
      uint32_t nv = 0, nd = 0;
      bool missing = false;
      for (uint32_t t = 0; t < S; t++) {
        uint64_t x = 0;
        uint32_t v = 0;
        const int kind = decode_dep(dep_code[size_t(i) * S + t], &v, &x, dlog, bbase, n);
        if (kind == 1) {
          bool dup = false;
          for (uint32_t q = 0; q < nv; q++) dup |= ds[q] == v;
          if (!dup) {
            ds[nv++] = v;
            fwd += v > vbase + i;
          }
          dd[nd++] = dot[v];
        } else if (kind == 2) {
          {
            dd[nd++] = x;
            // executed? (AEClock frontier; exceptions are not carried by the
            // fused engine: every earlier batch executed completely)
            if ((x & 0x00FFFFFFFFFFFFFFull) > frontier[x >> 56]) missing = true;
          }
        }
      }
      for (uint32_t q = nv; q < S; q++) ds[q] = vbase + i;  // padding: self loops are ignored
      if (nv_out) nv_out[i] = nv;
      const uint32_t m = S == 1 ? nd : sort_unique_u64(dd, nd);
      for (uint32_t q = m; q < S; q++) dd[q] = 0;
      dep_cnt[i] = m;
      if (blocked0) blocked0[i] = missing;
      if (missing) atomicAdd(nblocked, 1u);
    }
  }
  // forward-edge count: a block sum, one atomic per block over 64 counters
  // (per-wave atomics into them cost C4 1.2 ms of union time; the count is
  // asked for only where the tile path does not apply, wide rows)
  if (nfwd) {
    __shared__ uint32_t s_f[8];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) fwd += __shfl_xor(fwd, o, 64);
    if ((threadIdx.x & 63) == 0) s_f[threadIdx.x >> 6] = fwd;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (uint32_t w = 0; w < (blockDim.x >> 6); w++) t += s_f[w];
      if (t) atomicAdd(&nfwd[blockIdx.x & 63], (unsigned long long)t);
    }
  }
}

// Committed-dep count per command (rows of at most kRegSlots slots), from
// the codes alone: in-batch deps dedup by vid, external ones by dot (dots are
// unique, so this is the union's count).  Its scan places k_cmd_engine's
// output straight into the CSR: no fixed-stride rows, no compaction pass.
template <uint32_t kSlots, class CT>
__device__ __forceinline__ uint32_t cmd_count_regs(uint32_t i, uint32_t S,
                                                   const CT *__restrict__ dep_code,
                                                   const uint64_t *__restrict__ dlog,
                                                   uint64_t bbase, uint32_t n) {
  uint64_t r[kSlots];
#pragma unroll
  for (uint32_t t = 0; t < kSlots; t++) {
    r[t] = ~0ull;
    if (t < S) {
      uint64_t x = 0;
      uint32_t v = 0;
      const int kind = decode_dep(dep_code[size_t(i) * S + t], &v, &x, dlog, bbase, n);
      r[t] = kind == 1 ? uint64_t(v) : kind == 2 ? x : ~0ull;  // dots >= 2^56 > vids
    }
  }
  uint32_t c = 0;
#pragma unroll
  for (uint32_t t = 0; t < kSlots; t++) {
    bool dup = r[t] == ~0ull;
#pragma unroll
    for (uint32_t q = 0; q < t; q++) dup |= r[q] == r[t];
    c += dup ? 0u : 1u;
  }
  return c;
}

template <class CT>
__global__ void k_cmd_count(uint32_t n, uint32_t S, const CT *__restrict__ dep_code,
                            const uint64_t *__restrict__ dlog, uint64_t bbase,
                            uint32_t *__restrict__ cnt) {
  if (S <= 4) {
    GRID_STRIDE(i, n) cnt[i] = cmd_count_regs<4>(i, S, dep_code, dlog, bbase, n);
  } else if (S <= 8) {
    GRID_STRIDE(i, n) cnt[i] = cmd_count_regs<8>(i, S, dep_code, dlog, bbase, n);
  } else {
    GRID_STRIDE(i, n) cnt[i] = cmd_count_regs<kRegSlots>(i, S, dep_code, dlog, bbase, n);
  }
}

// ---- single view, one key per command: two fused passes over the sorted
// (key, vid) elements.  Deps and the per-key sequence in one pass; the
// latest-table update (segment tails) and the executed-clock advance in the
// next, so no head reads a latest entry a tail of the same batch rewrote.
// dep encoding in the single-view path: 0 = none, (vid + 1) for an in-batch
// dependency (the top byte of a dot is its ProcessId, never 0), otherwise the
// external dot from the latest table
__device__ __forceinline__ uint64_t enc_vid(uint32_t v) { return uint64_t(v) + 1; }

__global__ void __launch_bounds__(256)
    k_sv_deps(uint32_t M, const uint32_t *__restrict__ ks, const uint32_t *__restrict__ vs,
              const uint64_t *__restrict__ latest, uint32_t lmul, uint32_t lmask,
              uint64_t *__restrict__ dep_sorted) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool ok = j < M;
  const uint32_t key = ok ? ks[j] : 0u;
  const uint32_t vid = ok ? vs[j] : 0u;
  uint32_t pkey = __shfl_up(key, 1, 64);
  uint32_t pvid = __shfl_up(vid, 1, 64);
  if (lane == 0 && ok && j > 0) {
    pkey = ks[j - 1];
    pvid = vs[j - 1];
  }
  if (!ok) return;
  const bool head = j == 0 || pkey != key;
  // sequential.rs:83-96: the previous command on the key, or the latest
  // command on it from an earlier batch
  dep_sorted[j] = head ? latest[(key * lmul) & lmask] : enc_vid(pvid);
}

// Per-source {min, max, count} of a wave's dots: the lanes holding one source
// are grouped by ballot (a batch has few sources), reduced with shuffles, and
// the group leader folds the result into LDS.
__device__ __forceinline__ void src_stats_wave(bool ok, uint64_t d, unsigned long long *s_mn,
                                               unsigned long long *s_mx, unsigned int *s_cnt) {
  const int lane = threadIdx.x & 63;
  const uint32_t src = uint32_t(d >> 56);
  const unsigned long long q = d & 0x00FFFFFFFFFFFFFFull;
  uint64_t rem = __ballot(ok);
  while (rem) {
    const int leader = __builtin_ctzll(rem);
    const uint32_t s0 = __shfl(src, leader, 64);
    const bool mine = ok && src == s0;
    const uint64_t m = __ballot(mine);
    unsigned long long vmn = mine ? q : ~0ull, vmx = mine ? q : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long a = __shfl_xor(vmn, o, 64), b = __shfl_xor(vmx, o, 64);
      vmn = a < vmn ? a : vmn;
      vmx = b > vmx ? b : vmx;
    }
    if (lane == leader) {
      atomicMin(&s_mn[s0], vmn);
      atomicMax(&s_mx[s0], vmx);
      atomicAdd(&s_cnt[s0], unsigned(__popcll(m)));
    }
    rem &= ~m;
  }
}

// Segment tails update the latest table; every batch dot is executed, which
// advances the executed clock: per source the frontier becomes the max
// sequence and the executed count grows by the batch's count (the executed
// set is contiguous from 1 iff count == frontier, checked when results are
// read).  4096 elements per workgroup (16 per thread, loads issued up front),
// per-source partials in LDS, one global atomic per source per workgroup.
constexpr int kTailItems = 16;
constexpr int kTailTile = 256 * kTailItems;

__global__ void __launch_bounds__(256)
    k_sv_tails(uint32_t M, const uint32_t *__restrict__ ks, const uint32_t *__restrict__ vs,
               const uint64_t *__restrict__ dot, uint64_t log_base, uint64_t *__restrict__ latest,
               uint32_t lmul, uint32_t lmask, unsigned long long *__restrict__ frontier,
               unsigned long long *__restrict__ excount) {
  __shared__ unsigned long long s_mx[256];
  __shared__ unsigned int s_cnt[256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  s_mx[tid] = 0;
  s_cnt[tid] = 0;
  const uint32_t base = blockIdx.x * kTailTile + uint32_t(w) * 64 * kTailItems;
  uint32_t key[kTailItems + 1];
  uint64_t d[kTailItems];
#pragma unroll
  for (int i = 0; i < kTailItems; i++) {
    const uint32_t j = base + i * 64 + lane;
    key[i] = j < M ? ks[j] : ~0u;
    d[i] = j < M ? dot[j] : 0ull;  // batch dots in arrival order
  }
  {
    const uint32_t j = base + kTailItems * 64;  // first element after this wave's run
    key[kTailItems] = j < M ? ks[j] : ~0u;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kTailItems; i++) {
    const uint32_t j = base + i * 64 + lane;
    uint32_t nk = __shfl_down(key[i], 1, 64);
    const uint32_t nxt = __shfl(key[i + 1], 0, 64);
    if (lane == 63) nk = nxt;
    if (j < M) {
      if (j + 1 == M || nk != key[i])  // sequential.rs:88-95
        latest[(key[i] * lmul) & lmask] = kLogFlag | (log_base + vs[j]);
      const uint32_t src = uint32_t(d[i] >> 56);
      atomicMax(&s_mx[src], d[i] & 0x00FFFFFFFFFFFFFFull);
      atomicAdd(&s_cnt[src], 1u);
    }
  }
  __syncthreads();
  if (s_cnt[tid]) {
    atomicMax(&frontier[tid], s_mx[tid]);
    atomicAdd(&excount[tid], (unsigned long long)s_cnt[tid]);
  }
}

// results: single-view sorted deps -> per-command dep dots
// Single view: each command's one dependency slot, from sorted order to its
// command's row (rows of one slot, the reserved all-ones dot for none:
// results() packs the rows into the ABI's CSR, so no count, scan or
// compaction runs in the step).
__global__ void k_sv_rows(uint32_t M, const uint32_t *__restrict__ vs,
                          const uint64_t *__restrict__ dep_sorted,
                          const uint64_t *__restrict__ dot, const uint64_t *__restrict__ dlog,
                          uint64_t *__restrict__ rows, uint64_t *__restrict__ lab,
                          uint32_t *__restrict__ rank) {
  GRID_STRIDE(j, M) {
    const uint64_t x = dep_sorted[j];
    rows[vs[j]] = x == 0 ? ~0ull
                  : is_log_ref(x) ? dlog[x - kLogFlag]  // an earlier batch
                  : (x >> 56) == 0 ? dot[x - 1]         // in-batch index + 1
                                   : x;
    // the trivial order (every SCC a singleton, arrival order topological):
    // label = own dot, rank = position, in command order j
    if (lab) {
      lab[j] = dot[j];
      rank[j] = j;
    }
  }
}
__global__ void k_seq_dots(uint32_t m, const uint32_t *__restrict__ pk_vid,
                           const uint64_t *__restrict__ dot, uint64_t *__restrict__ seq) {
  GRID_STRIDE(j, m) seq[j] = dot[pk_vid[j]];
}

// executed-clock frontier advance for a fully executed batch (srcstats.h)
__global__ void __launch_bounds__(256)
    k_src_stats(uint32_t n, const uint64_t *__restrict__ dot, unsigned long long *__restrict__ mx,
                unsigned int *__restrict__ cnt) {
  __shared__ unsigned long long s_mx[256];
  __shared__ unsigned int s_cnt[256];
  SrcAcc acc;
  acc.init(s_mx, s_cnt);
  __syncthreads();
  GRID_STRIDE(i, n) acc.add(dot[i]);
  acc.commit(mx, cnt);
}

// The fused engine's executed clock: per source the highest executed
// sequence and the number of executed dots.  Every batch executes completely
// (no pending vertex is carried), and a dependency from an earlier batch can
// only come from the latest tables, which hold executed dots; so the
// `seq <= frontier[source]` test k_cmd_engine applies to external
// dependencies is exact for the engine's own streams, including key shards
// of a global stream whose executed sets are not contiguous per source.
__global__ void k_frontier_update(const unsigned long long *__restrict__ mx,
                                  const unsigned int *__restrict__ cnt, uint64_t *frontier,
                                  unsigned long long *excount) {
  const uint32_t s = threadIdx.x;
  if (s >= 256 || cnt[s] == 0) return;
  if (mx[s] > frontier[s]) frontier[s] = mx[s];
  excount[s] += cnt[s];
}

// The bucket path's per-key sequence: element j of the key-grouped order
// moves by its run's shift (run_offsets) to its ascending-key place; the
// trivial order's labels (own dot) and ranks (position) in the same pass
// (one element per command: single view, one key).
__global__ void k_run_place(uint32_t m, const uint32_t *__restrict__ keys,
                            const uint32_t *__restrict__ delta, const uint64_t *__restrict__ seqg,
                            uint64_t *__restrict__ out, const uint64_t *__restrict__ dot,
                            uint64_t *__restrict__ lab, uint32_t *__restrict__ rank) {
  GRID_STRIDE(j, m) {
    out[j + delta[keys[j]]] = seqg[j];
    lab[j] = dot[j];
    rank[j] = j;
  }
}

__global__ void k_bcast_u32(uint32_t n, uint32_t *p, uint32_t v) { GRID_STRIDE(i, n) p[i] = v; }

__global__ void k_identity_labels(uint32_t n, const uint64_t *__restrict__ dot,
                                  uint64_t *__restrict__ lab, uint32_t *__restrict__ rank) {
  GRID_STRIDE(i, n) {
    lab[i] = dot[i];
    rank[i] = i;
  }
}

// 32-bit packed dots: src << sb | seq.  Order-preserving (dots order by
// (src, seq), id.rs) when every sequence is below 2^sb and src fits the
// 32 - sb bits above it; the host picks sb (pb = src bits + sb <= 32) before
// taking this form, else the dots stay u64.
__global__ void k_pack_dots(uint32_t n, const uint64_t *__restrict__ dot, int sb,
                            uint32_t *__restrict__ out) {
  GRID_STRIDE(i, n) {
    const uint64_t d = dot[i];
    out[i] = uint32_t(((d >> 56) << sb) | (d & 0x00FFFFFFFFFFFFFFull));
  }
}

// per-key offsets straight from the sorted keys: o[k] = the number of
// elements whose key is below k (lower bound), for k in [0, K] -- one launch
// instead of a histogram (run starts, run counts) and its scan
__global__ void k_key_offsets(uint32_t m, const uint32_t *__restrict__ keys, uint32_t K,
                              uint32_t *__restrict__ o, uint32_t kmask = ~0u) {
  GRID_STRIDE(k, K + 1) {
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo) >> 1);
      if ((keys[mid] & kmask) < k)
        lo = mid + 1;
      else
        hi = mid;
    }
    o[k] = lo;
  }
}

__global__ void k_edges_csr(uint32_t n, uint32_t S, const uint32_t *__restrict__ ds,
                            const uint32_t *__restrict__ off, uint32_t *__restrict__ out) {
  GRID_STRIDE(i, n) {
    const uint32_t o = off[i], c = off[i + 1] - o;
    for (uint32_t q = 0; q < c; q++) out[o + q] = ds[size_t(i) * S + q];
  }
}

__global__ void k_compact_deps(uint32_t n, uint32_t S, const uint64_t *__restrict__ dd,
                               const uint32_t *__restrict__ off, uint64_t *__restrict__ out) {
  GRID_STRIDE(i, n) {
    const uint32_t c = off[i + 1] - off[i];
    for (uint32_t q = 0; q < c; q++) out[off[i] + q] = dd[size_t(i) * S + q];
  }
}

}  // namespace

struct EngineDevice {
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t key_space = 0;
  int key_bits = 1;
  uint32_t n_config = 0;
  // single-view latest table: indexed by the mapped key (keybucket.h) over a
  // region of kp = 2^key_bits entries; replica slots follow it
  bool lat_mapped = false;
  uint64_t kp = 0;
  uint32_t lmul = 1, lmask = 0xFFFFFFFFu;
  KeyBucketWorkspace kb_ws[2];      // double-buffered by batch parity
  size_t kb_next_part = ~size_t(0); // staged batch already partitioned by the last step
  DBuf<unsigned long long> kb_clk;  // executed-clock shard sets (2) of the bucket path
  KeyBucketSched kb_sched;          // largest-first order-workgroup schedule
  uint64_t kb_launches = 0;         // order launches (schedule refresh cadence)
  bool bucket_order = false;  // single-view per-key runs are key-grouped, not ascending
  DBuf<uint32_t> key_offs;
  // bucket path outputs: per-key run bounds in key-grouped order (zeroed per
  // batch), their shifts to ascending-key order, the key-grouped dots
  DBuf<uint32_t> kb_runs, kb_delta;
  uint32_t kb_run_tag = 0;  // the last batch's run tag
  DBuf<uint64_t> kb_seq;
  // persistent state
  DBuf<uint64_t> latest;     // [(nproc+1) * K]
  DBuf<uint64_t> frontier;   // [256] executed-clock frontier per source
  uint32_t latest_slots = 1; // replica slots allocated in `latest`
  DBuf<uint32_t> err;
  // staged batches
  fh_stream_desc desc{};
  bool staged = false;
  size_t nbatches = 0, cursor = 0, last = 0;
  DBuf<uint64_t> dot;     // the command log (every staged batch, appended)
  size_t log_len = 0;     // dots in the log
  size_t stage_base = 0;  // log position of the first staged batch
  DBuf<uint32_t> key32;
  // replica views: per batch, the replicas' arrival logs concatenated
  // (entries c·fq + j), and each batch's nproc + 1 log offsets
  DBuf<uint32_t> lent, loff;
  std::vector<uint32_t> h_loff;  // host copy of loff
  // scratch
  DBuf<uint64_t> dep_ext, dep_dot, seq_dot, lab;
  DBuf<uint32_t> dep32;  // replica views: 32-bit element dependency codes
  DBuf<uint32_t> sk32a, sk32b, sva, svb, dep_cnt, dst, sorted_vid, rank_tmp, u32tmp;
  // outputs of the last run (materialised inside run(), copied by results())
  bool deps_direct = false;  // run_general wrote o_dep_off / o_dep (no compaction)
  // the key-order path wrote each command's committed deps as a row of
  // deps_rows slots (o_rows); results() packs them into o_dep_off / o_dep
  // once (rows_packed)
  uint32_t deps_rows = 0;
  bool rows_packed = false;
  DBuf<uint64_t> o_rows;
  DBuf<uint32_t> o_rows32;  // rows of packed dots (rows32 set; unpacked with rows_sb)
  bool rows32 = false;
  int rows_sb = 0;
  // the widest source and sequence of every dot in the log (rows32_ok)
  uint64_t log_ms = 0, log_mq = 0;
  bool sv_labels_done = false;  // k_sv_compact wrote the trivial labels / ranks
  DBuf<uint32_t> o_dep_off;
  DBuf<uint64_t> o_dep;
  const uint64_t *o_label = nullptr;  // [n] min dot of each command's SCC
  const uint32_t *o_rank = nullptr;   // [n] position in the execution order
  uint32_t o_nelem = 0;               // per-key sequence length (key_offs, o_seq)
  const uint64_t *o_seq = nullptr;    // [o_nelem] per-key sequences of dots
  DBuf<uint32_t> edge_cnt, edge_off, edge_csr;  // replica views: in-batch edges as CSR
  DBuf<unsigned long long> fwd_ctr;  // [64] forward edges counted by the union
  DBuf<uint32_t> dot32;  // staged batches' dots packed to 32 bits (h_dpack)
  DBuf<uint8_t> blocked0;
  DBuf<uint32_t> scal;
  DBuf<uint32_t> place_base;  // replica views: per-chunk smallest element position
  DBuf<uint32_t> tail_defer;  // k_bucket_codes: deferred (segment, command) per workgroup
  DBuf<uint32_t> vrec;        // command-level views path: replica | arrival per element
  DBuf<uint8_t> tailm;        // command-level views path: tail views per sorted command
  DBuf<uint32_t> mrem;        // command-level views path: predecessor marks across tiles
  DBuf<uint4> crec;           // command-level views path: (command, codes) by tile and region
  DBuf<uint32_t> ctoff;       // command-level views path: region cursors
  // key-order path (cmd_views_keyorder)
  bool ko_done = false;       // this run's outputs came from the key-order path
  DBuf<V3> kv3a, kv3b;        // sort values with packed dots
  DBuf<uint32_t> kpcode;      // [n·fq] escaped edge targets (position + 1)
  DBuf<uint32_t> kpe8;        // [n] key-order edges as 8-bit distances
  DBuf<uint32_t> kpd32;       // [n] packed dot by sorted position
  DBuf<uint4> khl;            // [n] (H, rank, label) of those, by command
  DBuf<uint32_t> kdiff, kss;  // straddle counts and their scan
  // FH_KEYORDER=0 (measurement, tests): the command-order graph path
  const bool keyorder_off = [] {
    const char *e = getenv("FH_KEYORDER");
    return e && *e == '0';
  }();
  DBuf<uint64_t> cv64a, cv64b;  // command-level views path: packed sort values
  PinnedRing ring;              // staging uploads (hoststage.h)
  std::vector<uint32_t> h_win;  // per batch: the logs' inversion span W (stage_logs)
  // per batch: (seq bits, packed bits) of its dots, src << sb | seq (0: wider
  // than 32 bits), so the per-key sort can move 4-byte dots
  std::vector<std::pair<int, int>> h_dpack;
  bool deps_only = false;     // fh_engine_set_deps_only: stop after the committed deps
  bool codes_only = false;    // subset logs (fh_dgraph): stop after KeyDeps, codes in dep32
  bool last_deps_only = false;
  DBuf<unsigned long long> srcstats;
  SortWorkspace sort_ws;
  ScanWorkspace scan_ws;
  // key-order path: the command-order half of a batch (code scatter, tails,
  // union) runs on `side` beside the tile kernel on `stream`; FH_KO_SIDE=0
  // (measurement) keeps it on `stream`
  const bool side_off = [] {
    const char *e = getenv("FH_KO_SIDE");
    return e && *e == '0';
  }();
  // Workgroups of the side kernels: 256 threads, three per four CUs (below).  The
  // side kernels' random row stores are what slows the tile kernel beside
  // them (C4 with k_row_place issuing its loads but not its stores: 12.48 ->
  // 10.87 ms, r06f), so fewer side waves, finishing later, cost the tile
  // kernel less: C4, ms per step, 1 per CU 12.48-12.50, 2 per CU 12.81,
  // 3 per CU 13.99 (r06e/f).  (Round 5, with the entries scatter and the
  // union: 2 per CU 15.6, 1.5 16.9, 3 16.1, r05_side_sweep.txt.)
  unsigned side_grid = 0;
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  ScanWorkspace scan_ws2;
  GraphCore graph;
  GraphOutput gout;
  Probe probe;
  bool sv_fused = false;
  const uint32_t *sorted_keys32 = nullptr;  // single-view: keys in sorted order
  const uint32_t *sv_vs = nullptr;          // single-view: vids in sorted order
  DBuf<unsigned long long> excount;  // executed dots per source (single-view clock)
  unsigned long long *excount_ptr() {
    if (!excount.get()) {
      excount.ensure(256);
      FH_HIP(hipMemsetAsync(excount.get(), 0, 256 * sizeof(unsigned long long), stream));
    }
    return excount.get();
  }
  // timing
  bool profile = false;
  std::vector<std::pair<const char *, hipEvent_t>> marks;
  std::vector<std::pair<std::string, float>> last_times;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;

  explicit EngineDevice(const fh_config &cfg) {
    FH_CHECK(cfg.key_space >= 1 && cfg.key_space <= (uint64_t(1) << 31), FH_EINVAL,
             "key_space must be in [1, 2^31]");
    key_space = cfg.key_space;
    key_bits = bits_for(key_space);
    n_config = cfg.n;
    lat_mapped = key_bits <= 22;
    kp = key_space;
    if (lat_mapped) {
      uint32_t kinv = 0;
      keybucket_map(key_bits, &lmul, &kinv, &lmask);
      kp = uint64_t(1) << key_bits;
    }
    device = pick_device(&cfg, 0);
    FH_HIP(hipSetDevice(device));
    // (the side stream is created by the first key-order batch; queue
    // priorities -- the engine's stream highest, the side stream lowest --
    // measured no different: 14.00 / 14.16 against 14.00 / 14.32 ms, r05ba)
    FH_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    FH_HIP(hipEventCreate(&ev0));
    FH_HIP(hipEventCreate(&ev1));
    {
      int cus = 0;
      FH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
      // three workgroups per four CUs: the side stream's work (2.3 ms of
      // row placement at one per CU) has slack beside the tile kernel (4.1
      // ms), and fewer row stores in flight slow the tile kernel less (C4,
      // ms per step, 256 / 224 / 192 / 160 / 128 workgroups: 11.37-11.56 /
      // 11.30-11.43 / 11.27-11.29 / 11.30 / 12.27 on one box, r06sg)
      side_grid = unsigned(std::max(cus * 3 / 4, 1));
    }
    FH_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    FH_HIP(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));

    graph.stream = stream;
    graph.marks = &marks;
    err.ensure(4);
    scal.ensure(16);
    frontier.ensure(256);
    reset();
  }
  ~EngineDevice() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    clear_marks();
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (side) (void)hipStreamSynchronize(side);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (side) (void)hipStreamDestroy(side);
    if (stream) (void)hipStreamDestroy(stream);
  }

  void clear_marks() {
    for (auto &m : marks) (void)hipEventDestroy(m.second);
    marks.clear();
  }
  void mark(const char *name) {
    if (!profile) return;
    hipEvent_t e;
    FH_HIP(hipEventCreate(&e));
    FH_HIP(hipEventRecord(e, stream));
    marks.push_back({name, e});
  }

  // [single view: kp][replica 1: K][replica 2: K]...
  size_t latest_words(uint32_t slots) const { return size_t(kp) + size_t(slots - 1) * key_space; }
  // replica r's entry for key is views_latest()[r * K + key] (r >= 1)
  uint64_t *views_latest() { return latest.get() + (kp - key_space); }

  void ensure_latest(uint32_t slots) {
    if (latest.get() && slots <= latest_slots) return;
    latest_slots = std::max<uint32_t>(slots, 1);
    latest.ensure(latest_words(latest_slots));
    FH_HIP(hipMemsetAsync(latest.get(), 0, latest_words(latest_slots) * sizeof(uint64_t), stream));
  }

  // stream idle (staged data, the command log and the clock shards may be
  // rewritten afterwards); forgets a partition done ahead
  void sync_all() {
    if (kb_next_part != ~size_t(0) && kb_clk.get()) {
      // a batch partitioned ahead will not be ordered: drop its clock shards
      FH_HIP(hipMemsetAsync(kb_clk.get() + (kb_next_part & 1) * kKeyBucketClockWords, 0,
                            kKeyBucketClockWords * sizeof(unsigned long long), stream));
    }
    FH_HIP(hipStreamSynchronize(stream));
    // the key-order path's side stream: joined back into `stream` on every
    // normal exit, but a run that threw between its fork and its join may
    // have left side kernels running on the buffers the next stage reuses
    if (side) FH_HIP(hipStreamSynchronize(side));
    kb_next_part = ~size_t(0);
  }
  KeyBucketClock kb_clock(size_t batch) {
    KeyBucketClock c;
    c.fold = kb_clk.get() + (batch & 1) * kKeyBucketClockWords;
    c.frontier = reinterpret_cast<unsigned long long *>(frontier.get());
    c.excount = excount_ptr();
    return c;
  }

  void reset() {
    FH_HIP(hipSetDevice(device));
    sync_all();
    ensure_latest(latest_slots);
    FH_HIP(hipMemsetAsync(latest.get(), 0, latest_words(latest_slots) * sizeof(uint64_t), stream));
    FH_HIP(hipMemsetAsync(frontier.get(), 0, 256 * sizeof(uint64_t), stream));
    FH_HIP(hipMemsetAsync(excount_ptr(), 0, 256 * sizeof(unsigned long long), stream));
    FH_HIP(hipMemsetAsync(kb_clk.ensure(2 * kKeyBucketClockWords), 0,
                          2 * kKeyBucketClockWords * sizeof(unsigned long long), stream));
    FH_HIP(hipMemsetAsync(err.get(), 0, 4 * sizeof(uint32_t), stream));
    FH_HIP(hipStreamSynchronize(stream));
    log_len = 0;
    log_ms = log_mq = 0;
    staged = false;
  }

  // fq_proc / fq_time -> per-replica arrival logs: replica r processes the
  // commands it is a member for in (time, command index) order.
  static void views_to_logs(const fh_stream_desc &d, size_t nb, const uint8_t *h_proc,
                            const uint64_t *h_time, std::vector<uint64_t> &off,
                            std::vector<uint32_t> &cmd) {
    const size_t n = d.n, fq = d.views, np = d.nproc;
    off.assign(nb * np + 1, 0);
    cmd.assign(n * fq * nb, 0);
    std::vector<size_t> cnt(nb * np, 0);
    for (size_t b = 0; b < nb; b++)
      for (size_t i = 0; i < n * fq; i++) {
        const uint8_t p = h_proc[b * n * fq + i];
        FH_CHECK(p >= 1 && p <= np, FH_EINVAL, "fq_proc out of range");
        cnt[b * np + p - 1]++;
      }
    for (size_t x = 0; x < nb * np; x++) off[x + 1] = off[x] + cnt[x];
    std::vector<size_t> fill(off.begin(), off.end() - 1);
    for (size_t b = 0; b < nb; b++)
      for (size_t i = 0; i < n * fq; i++) {
        const uint8_t p = h_proc[b * n * fq + i];
        cmd[fill[b * np + p - 1]++] = uint32_t(i / fq);
      }
    const size_t logs = nb * np;
    auto work = [&](size_t lo, size_t hi) {
      std::vector<std::pair<uint64_t, uint32_t>> tmp;
      for (size_t x = lo; x < hi; x++) {
        const size_t b = x / np;
        tmp.clear();
        for (size_t q = off[x]; q < off[x + 1]; q++) {
          const uint32_t c = cmd[q];
          // this command's member on replica (x % np) + 1
          uint64_t t = 0;
          for (size_t j = 0; j < fq; j++)
            if (h_proc[(b * n + c) * fq + j] == x % np + 1) t = h_time[(b * n + c) * fq + j];
          tmp.push_back({t, c});
        }
        std::sort(tmp.begin(), tmp.end());
        for (size_t q = 0; q < tmp.size(); q++) cmd[off[x] + q] = tmp[q].second;
      }
    };
    const size_t nt = std::min<size_t>(logs, 16);
    std::vector<std::thread> ts;
    for (size_t t = 0; t < nt; t++)
      ts.emplace_back(work, logs * t / nt, logs * (t + 1) / nt);
    for (auto &t : ts) t.join();
  }

  // Replay the staged batches from a clean state: latest tables and executed
  // clock cleared on the engine stream (no host synchronisation), cursor back
  // to the first staged batch.  The command log keeps its staged dots.
  void rewind() {
    FH_CHECK(staged, FH_EINVAL, "rewind: nothing staged");
    FH_HIP(hipSetDevice(device));
    if (kb_next_part != ~size_t(0) && kb_clk.get())
      FH_HIP(hipMemsetAsync(kb_clk.get() + (kb_next_part & 1) * kKeyBucketClockWords, 0,
                            kKeyBucketClockWords * sizeof(unsigned long long), stream));
    kb_next_part = ~size_t(0);
    FH_HIP(hipMemsetAsync(latest.get(), 0, latest_words(latest_slots) * sizeof(uint64_t), stream));
    FH_HIP(hipMemsetAsync(frontier.get(), 0, 256 * sizeof(uint64_t), stream));
    FH_HIP(hipMemsetAsync(excount_ptr(), 0, 256 * sizeof(unsigned long long), stream));
    cursor = 0;
  }

  void stage(const fh_stream_desc &d, size_t nb, const uint64_t *h_dot, const uint64_t *h_key,
             const uint8_t *h_proc, const uint64_t *h_time) {
    if (!d.views) {
      stage_logs(d, nb, h_dot, h_key, nullptr, nullptr);
      return;
    }
    FH_CHECK(h_proc && h_time && d.nproc >= 1 && d.nproc <= 255, FH_EINVAL,
             "replica views need fq_proc, fq_time and nproc");
    FH_CHECK(d.views <= 16, FH_EINVAL, "views <= 16");
    std::vector<uint64_t> off;
    std::vector<uint32_t> cmd;
    views_to_logs(d, nb, h_proc, h_time, off, cmd);
    stage_logs(d, nb, h_dot, h_key, off.data(), cmd.data());
  }

  // Element logs (partial replication) through the pair-level search: the
  // units are (command, key slot) pairs u = c·k + s, each with its fq views
  // (elements (c·fq + j)·k + s).  Every process's KeyDeps handles one unit's
  // key on its own (sequential.rs:72-104 per key), so the unit's dependency at
  // view j is the latest earlier arrival of its key at that view's process,
  // exactly the command-level search over units.  Per stage:
  //  * the logs get replica ids: a greedy colouring of the logs in which two
  //    logs holding elements of one key differ (a key's processes are its
  //    shard's, so C5's 40 logs take 5 ids) -- the search indexes its
  //    per-replica arrival slots, tail marks and latest rows by these ids,
  //    and a key's table rows stay its own since no two of its logs share an
  //    id; at most kSrchMaxRep ids;
  //  * per batch: every unit's fq views lie in logs of different ids, and
  //    h_win[b] = the logs' inversion span over units (as views_entries does
  //    over commands).
  // A batch failing any of it (or k not a power of two <= 8, or a key space
  // over 2^22) keeps the chunked element path.
  std::vector<uint32_t> h_rid;      // [kMaxLogs] replica id of each log (batch-local index)
  std::vector<uint32_t> stage_rid;  // the ids the latest table's rows were last staged under
  // per batch: the view records' slice bounds of the element logs (k_view_records
  // `bounds`, (G + 1) x np entries at vbnd + h_vbnd_off[b]) and their G
  std::vector<uint32_t> h_vbnd_g;
  std::vector<size_t> h_vbnd_off;
  DBuf<uint32_t> vbnd;
  std::vector<uint8_t> h_unit_ok;   // per batch
  uint32_t unit_colors = 0;
  void unit_meta(size_t nb, size_t n, uint32_t fq, uint32_t k, size_t np, const uint64_t *h_off,
                 const uint32_t *h_cmd, const uint64_t *h_key) {
    if (k > 8 || (k & (k - 1)) || np > uint32_t(kMaxLogs) || key_space > (uint64_t(1) << 22) ||
        size_t(n) * k >= (size_t(1) << 30))
      return;
    const uint32_t us = uint32_t(__builtin_ctz(k));
    const size_t per_b = n * fq * k, T = host_threads();
    // 1. the logs holding each key (per-thread masks, OR-reduced)
    std::vector<std::vector<uint64_t>> km(T);
    const uint64_t ents = h_off[nb * np];
    par_for(ents, size_t(1) << 20, [&](size_t part, size_t l, size_t h) {
      auto &m = km[part];
      m.assign(key_space, 0);
      uint32_t x = uint32_t(std::upper_bound(h_off, h_off + nb * np + 1, uint64_t(l)) - h_off) - 1;
      for (uint64_t q = l; q < h; q++) {
        while (h_off[x + 1] <= q) x++;
        const size_t b = x / np, r = x % np;
        const uint32_t e = h_cmd[q];
        const size_t c = e / (fq * k), sl = e % k;
        m[h_key[(b * n + c) * k + sl]] |= uint64_t(1) << r;
      }
    });
    std::vector<uint64_t> adj(np, 0);
    {
      std::vector<std::vector<uint64_t>> ad(T, std::vector<uint64_t>(np, 0));
      par_for(key_space, size_t(1) << 16, [&](size_t part, size_t l, size_t h) {
        for (size_t key = l; key < h; key++) {
          uint64_t m = 0;
          for (auto &t : km) m |= t.empty() ? 0 : t[key];
          for (uint64_t b = m; b; b &= b - 1) ad[part][__builtin_ctzll(b)] |= m;
        }
      });
      for (auto &a : ad)
        for (size_t r = 0; r < np; r++) adj[r] |= a[r];
    }
    km.clear();
    // greedy colouring in log order
    std::vector<uint32_t> rid(np, 0);
    uint32_t colors = 0;
    for (size_t r = 0; r < np; r++) {
      uint32_t used = 0;
      for (size_t q = 0; q < r; q++)
        if (adj[r] >> q & 1) used |= 1u << rid[q];
      uint32_t c = 0;
      while (c < uint32_t(kSrchMaxRep) && (used >> c & 1)) c++;
      if (c >= uint32_t(kSrchMaxRep)) return;
      rid[r] = c;
      colors = std::max(colors, c + 1);
    }
    // 2. per batch: distinct ids per unit, and the inversion span over units
    std::vector<uint8_t> um(size_t(n) * k);
    struct Seg {
      uint32_t r, maxu, minu, win;
    };
    for (size_t b = 0; b < nb; b++) {
      std::fill(um.begin(), um.end(), 0);
      const uint64_t base = h_off[b * np], cnt = uint64_t(per_b);
      const uint64_t *lb = h_off + b * np;
      std::atomic<bool> bad{false};
      std::vector<std::vector<Seg>> segs(T);
      par_for(cnt, size_t(1) << 20, [&](size_t part, size_t l, size_t h) {
        auto &sg = segs[part];
        uint64_t q = base + l;
        uint32_t r = uint32_t(std::upper_bound(lb, lb + np + 1, q) - lb) - 1;
        while (q < base + h) {
          while (lb[r + 1] <= q) r++;
          const uint64_t end = std::min<uint64_t>(base + h, lb[r + 1]);
          const uint8_t bit = uint8_t(1u << rid[r]);
          Seg g{r, 0, ~0u, 0};
          uint32_t pmax = 0;
          for (; q < end; q++) {
            const uint32_t e = h_cmd[q];
            const uint32_t u = uint32_t(((e / (fq * k)) << us) | (e % k));
            if (__atomic_fetch_or(&um[u], bit, __ATOMIC_RELAXED) & bit) bad = true;  // (a view twice)
            pmax = std::max(pmax, u);
            g.win = std::max(g.win, pmax - u);
            g.minu = std::min(g.minu, u);
          }
          g.maxu = pmax;
          sg.push_back(g);
        }
      });
      if (bad) {
        h_unit_ok.assign(nb, 0);
        return;
      }
      std::vector<uint32_t> run_max(np, 0);
      std::vector<bool> started(np, false);
      uint32_t w = 0;
      for (auto &sg : segs)
        for (const Seg &g : sg) {
          w = std::max(w, g.win);
          if (started[g.r] && run_max[g.r] > g.minu) w = std::max(w, run_max[g.r] - g.minu);
          run_max[g.r] = started[g.r] ? std::max(run_max[g.r], g.maxu) : g.maxu;
          started[g.r] = true;
        }
      h_win[b] = w;
      h_unit_ok[b] = 1;
    }
    // the latest table's replica rows follow the ids: a stage that continues
    // an earlier one (log_len > 0) keeps that one's ids, or stays chunked
    std::vector<uint32_t> ids(kMaxLogs);
    for (uint32_t r = 0; r < uint32_t(kMaxLogs); r++) ids[r] = r < np ? rid[r] : r;
    if (log_len > 0 && ids != stage_rid) {
      h_unit_ok.assign(nb, 0);
      return;
    }
    h_rid = ids;
    unit_colors = colors;
    // the view records' slices (cmd_views' G): per log, the first entry of
    // each slice's first command, one monotone walk per log
    const uint32_t epc = fq * k;
    const uint32_t per = std::max<uint32_t>(1, (kRecWin - 2 * rec_slack(kRecWin)) / epc);
    const uint32_t G = std::max<uint32_t>(1, uint32_t((n + per - 1) / per));
    std::vector<uint32_t> bnd(nb * size_t(G + 1) * np);
    h_vbnd_g.assign(nb, G);
    h_vbnd_off.assign(nb, 0);
    for (size_t b = 0; b < nb; b++) {
      h_vbnd_off[b] = b * size_t(G + 1) * np;
      par_for(np, 1, [&](size_t, size_t l, size_t h) {
        for (size_t r = l; r < h; r++) {
          const uint64_t q0 = h_off[b * np + r], len = h_off[b * np + r + 1] - q0;
          uint64_t q = 0;
          for (uint32_t w = 0; w <= G; w++) {
            const uint64_t c0 = w == G ? ~uint64_t(0) : uint64_t(n) * w / G;
            while (q < len && h_cmd[q0 + q] / epc < c0) q++;
            bnd[h_vbnd_off[b] + size_t(w) * np + r] = uint32_t(q);
          }
        }
      });
    }
    FH_HIP(hipMemcpyAsync(vbnd.ensure(bnd.size() + 1), bnd.data(), bnd.size() * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    FH_HIP(hipStreamSynchronize(stream));
  }

  // Command logs of nb batches (stage_logs): validated per batch on
  // host_threads() threads and uploaded to dl.  Entry q of log r (command c)
  // is c·fq + j with j = the number of lower logs holding c: each command's
  // membership mask (bit r, set atomically; a bit set twice is a replica
  // processing c twice) gives j as a popcount, and every mask must hold
  // exactly fq bits.  h_win[b] = the logs' inversion span W, max over
  // entries of (the log's running maximum - c), combined across slices as
  // max(slice win, earlier slices' maximum - slice minimum).
  template <class M>
  void views_entries(size_t nb, size_t n, uint32_t fq, size_t np, const uint64_t *h_off,
                     const uint32_t *h_cmd, uint32_t *dl) {
    std::vector<M> mask(n);
    h_win.assign(nb, 0);
    struct Seg {
      uint32_t r, maxc, minc, win;
    };
    for (size_t b = 0; b < nb; b++) {
      if (b)
        par_for(n, size_t(1) << 22, [&](size_t, size_t l, size_t h) {
          std::memset(mask.data() + l, 0, (h - l) * sizeof(M));
        });
      const uint64_t base = h_off[b * np], cnt = uint64_t(n) * fq;
      const uint64_t *lb = h_off + b * np;  // this batch's np + 1 log bounds
      // the log holding global entry q
      auto log_of = [&](uint64_t q) {
        return uint32_t(std::upper_bound(lb, lb + np + 1, q) - lb) - 1;
      };
      std::vector<std::vector<Seg>> segs(host_threads());
      par_for(cnt, size_t(1) << 20, [&](size_t part, size_t l, size_t h) {
        auto &sg = segs[part];
        uint64_t q = base + l;
        uint32_t r = log_of(q);
        while (q < base + h) {
          while (lb[r + 1] <= q) r++;
          const uint64_t e = std::min<uint64_t>(base + h, lb[r + 1]);
          const M bit = M(M(1) << r);
          Seg g{r, 0, ~0u, 0};
          uint32_t pmax = 0;
          for (; q < e; q++) {
            const uint32_t c = h_cmd[q];
            FH_CHECK(c < n, FH_EINVAL, "logs: command index >= n");
            const M old = __atomic_fetch_or(&mask[c], bit, __ATOMIC_RELAXED);
            FH_CHECK(!(old & bit), FH_EINVAL, "logs: a replica processes a command once");
            pmax = std::max(pmax, c);
            g.win = std::max(g.win, pmax - c);
            g.minc = std::min(g.minc, c);
          }
          g.maxc = pmax;
          sg.push_back(g);
        }
      });
      std::vector<uint32_t> run_max(np, 0);
      std::vector<bool> started(np, false);
      uint32_t w = 0;
      for (auto &sg : segs)
        for (const Seg &g : sg) {
          w = std::max(w, g.win);
          if (started[g.r] && run_max[g.r] > g.minc) w = std::max(w, run_max[g.r] - g.minc);
          run_max[g.r] = started[g.r] ? std::max(run_max[g.r], g.maxc) : g.maxc;
          started[g.r] = true;
        }
      h_win[b] = w;
      par_for(n, size_t(1) << 20, [&](size_t, size_t l, size_t h) {
        for (size_t c = l; c < h; c++)
          FH_CHECK(uint32_t(__builtin_popcountll(uint64_t(mask[c]))) == fq, FH_EINVAL,
                   "logs: every command must appear in exactly `views` replica logs");
      });
      ring.upload(dl + base, cnt, [&](uint32_t *o, size_t first, size_t k) {
        uint64_t q = base + first;
        uint32_t r = log_of(q);
        for (size_t x = 0; x < k; x++, q++) {
          while (lb[r + 1] <= q) r++;
          const uint32_t c = h_cmd[q];
          o[x] = uint32_t(c * fq + uint32_t(__builtin_popcountll(uint64_t(mask[c]) & ((uint64_t(1) << r) - 1))));
        }
      }, stream);
    }
  }

  // log_off[nb·nproc + 1] (global offsets into log_cmd), log_cmd[] batch-local
  // command indices; every command appears in exactly `views` logs, at most
  // once per log
  // subset (fh_dgraph, element logs only): the logs hold a subset of the
  // batch's positions, each at most once -- one key shard's processes; runs
  // then stop after KeyDeps (codes_only)
  void stage_logs(const fh_stream_desc &d, size_t nb, const uint64_t *h_dot,
                  const uint64_t *h_key, const uint64_t *h_off, const uint32_t *h_cmd,
                  bool subset = false) {
    FH_CHECK(h_dot && h_key && nb >= 1, FH_EINVAL, "null argument");
    FH_CHECK(d.keys_per_cmd >= 1 && d.keys_per_cmd <= 8, FH_EINVAL, "keys_per_cmd in [1, 8]");
    const uint32_t fq = d.views ? d.views : 1;
    FH_CHECK(fq <= 16, FH_EINVAL, "views <= 16");
    // element positions (c·fq + j)·k + s and in-batch codes vid + 1 are u32
    // with the top bit free (C5: 100M commands x 4 keys x 3 views = 1.2G)
    FH_CHECK(size_t(d.n) * fq * d.keys_per_cmd < (size_t(1) << 31), FH_EINVAL,
             "batch too large (elements >= 2^31)");
    FH_CHECK(!d.views || (h_off && h_cmd && d.nproc >= 1 && d.nproc <= 255), FH_EINVAL,
             "replica views need per-replica logs and nproc");
    const bool elem = (d.flags & FH_STREAM_ELEMENT_LOGS) != 0;
    FH_CHECK((d.flags & ~FH_STREAM_ELEMENT_LOGS) == 0, FH_EINVAL, "stream desc: unknown flags");
    FH_CHECK(!elem || (d.views && d.nproc <= uint32_t(kMaxLogs)), FH_EINVAL,
             "element logs need replica views and nproc <= 64");
    FH_CHECK(!subset || (elem && nb == 1), FH_EINVAL, "subset logs: element logs, one batch");
    FH_CHECK(!d.views || uint64_t(d.nproc + 1) * key_space <= 0xFFFFFFFFull, FH_ENOTIMPL,
             "replica views: (nproc + 1) * key_space must fit 32 bits");
    FH_HIP(hipSetDevice(device));
    sync_all();
    const size_t n = d.n, nk = n * d.keys_per_cmd;
    // Validation first, on host_threads() threads (no device state changes
    // until the whole stream is accepted), then the uploads through pinned
    // chunks (hoststage.h); round 5 ran these loops on one thread with
    // pageable copies: 1,037 ms per 100M C4 commands.
    par_for(nk * nb, size_t(1) << 20, [&](size_t, size_t lo_, size_t hi_) {
      for (size_t e = lo_; e < hi_; e++)
        FH_CHECK(h_key[e] < key_space, FH_EINVAL, "stage: key id >= key_space");
    });
    // the all-ones dot, (255, 2^56 - 1), is the union's empty-slot sentinel;
    // per batch the widest source and sequence (the 32-bit packing)
    std::vector<std::pair<int, int>> dpack(nb, {0, 0});
    uint64_t smax_ms = 0, smax_mq = 0;  // this stage's widest
    for (size_t b = 0; b < nb; b++) {
      std::vector<std::pair<uint64_t, uint64_t>> mx(host_threads(), {0, 0});
      par_for(n, size_t(1) << 20, [&](size_t part, size_t lo_, size_t hi_) {
        uint64_t ms = 0, mq = 0;
        for (size_t i = b * n + lo_; i < b * n + hi_; i++) {
          const uint64_t x = h_dot[i];
          FH_CHECK(x != ~0ull && (x >> 56) != 0, FH_EINVAL,
                   "stage: dot (255, 2^56 - 1) is reserved and ProcessId 0 is not a process");
          ms = std::max<uint64_t>(ms, x >> 56);
          mq = std::max<uint64_t>(mq, x & 0x00FFFFFFFFFFFFFFull);
        }
        mx[part] = {ms, mq};
      });
      uint64_t ms = 0, mq = 0;
      for (auto &m : mx) {
        ms = std::max(ms, m.first);
        mq = std::max(mq, m.second);
      }
      const int sb = bits_for(mq + 1), pb = sb + bits_for(ms + 1);
      dpack[b] = pb <= 32 ? std::make_pair(sb, pb) : std::make_pair(0, 0);
      smax_ms = std::max(smax_ms, ms);
      smax_mq = std::max(smax_mq, mq);
    }
    const size_t np = d.nproc;
    std::vector<uint32_t> lo;
    const size_t per_b = n * fq * d.keys_per_cmd;  // element positions of a batch
    if (d.views) {
      FH_CHECK(elem ? (h_off[0] == 0 &&
                       (subset ? h_off[np] <= per_b : h_off[nb * np] == per_b * nb))
                    : (h_off[0] == 0 && h_off[nb * np] == n * fq * nb),
               FH_EINVAL, elem ? "element logs: every element position must appear in exactly one log"
                               : "logs: every command must appear in exactly `views` replica logs");
      FH_CHECK(elem || np <= 64, FH_ENOTIMPL, "replica views: nproc <= 64");
      lo.resize(nb * (np + 1));
      for (size_t b = 0; b < nb; b++) {
        const uint64_t base = h_off[b * np];
        if (elem)
          FH_CHECK(subset || h_off[(b + 1) * np] - base == per_b, FH_EINVAL,
                   "element logs: a batch's logs must hold n * views * keys_per_cmd entries");
        else
          FH_CHECK(h_off[(b + 1) * np] - base == n * fq, FH_EINVAL,
                   "logs: a batch's logs must hold n * views entries");
        for (size_t r = 0; r < np; r++) {
          lo[b * (np + 1) + r] = uint32_t(h_off[b * np + r] - base);
          FH_CHECK(h_off[b * np + r + 1] >= h_off[b * np + r], FH_EINVAL, "logs: offsets");
        }
        lo[b * (np + 1) + np] = uint32_t(h_off[(b + 1) * np] - base);
      }
    }
    // the device side from here: a stage that fails below leaves nothing staged
    staged = false;
    h_dpack = dpack;
    h_unit_ok.assign(nb, 0);
    h_rid.assign(kMaxLogs, 0);
    for (uint32_t r = 0; r < uint32_t(kMaxLogs); r++) h_rid[r] = r;
    unit_colors = 0;
    // append the batches' dots to the command log (grown by doubling, old
    // entries kept: earlier batches stay referenced by the latest table)
    const size_t need = log_len + n * nb + 1;
    if (need > dot.cap || !dot.get()) {
      DBuf<uint64_t> grown;
      grown.ensure(std::max(need, 2 * dot.cap));
      if (log_len)
        FH_HIP(hipMemcpyAsync(grown.get(), dot.get(), log_len * sizeof(uint64_t),
                              hipMemcpyDeviceToDevice, stream));
      FH_HIP(hipStreamSynchronize(stream));
      dot.swap(grown);
    }
    FH_CHECK(log_len + n * nb < kLogFlag, FH_ENOTIMPL, "command log exceeds 2^48 commands");
    FH_CHECK(!d.views || log_len + n * nb < (size_t(1) << 31), FH_ENOTIMPL,
             "replica views: command log exceeds 2^31 commands (32-bit dependency codes)");
    ring.upload_copy(dot.get() + log_len, h_dot, n * nb, stream);
    // the union's gathers read a packed copy of each batch's dots (input
    // layout, built here with the upload)
    {
      bool any = false;
      for (size_t b = 0; b < nb; b++) any |= h_dpack[b].second > 0;
      if (any) {
        uint32_t *d32 = dot32.ensure(n * nb + 1);
        for (size_t b = 0; b < nb; b++)
          if (h_dpack[b].second > 0)
            k_pack_dots<<<grid_for(uint32_t(n), B), B, 0, stream>>>(
                uint32_t(n), dot.get() + log_len + b * n, h_dpack[b].first, d32 + b * n);
      }
    }
    ring.upload(key32.ensure(nk * nb + 1), nk * nb, [&](uint32_t *o, size_t first, size_t cnt) {
      for (size_t e = 0; e < cnt; e++) o[e] = uint32_t(h_key[first + e]);
    }, stream);
    if (d.views) {
      uint32_t *dl = lent.ensure(size_t(h_off[subset ? np : nb * np]) + 1);
      if (elem) {
        // every position once per batch (a byte per position, set atomically
        // by the validating threads), then the entries as they are
        std::vector<uint8_t> seen(per_b);
        h_win.assign(nb, 0);
        for (size_t b = 0; b < nb; b++) {
          const uint64_t base = h_off[b * np], cnt = h_off[subset ? np : (b + 1) * np] - base;
          if (b)
            par_for(per_b, size_t(1) << 22, [&](size_t, size_t l, size_t h) {
              std::memset(seen.data() + l, 0, h - l);
            });
          par_for(cnt, size_t(1) << 20, [&](size_t, size_t l, size_t h) {
            for (uint64_t q = base + l; q < base + h; q++) {
              const uint32_t pq = h_cmd[q];
              FH_CHECK(pq < per_b && !__atomic_exchange_n(&seen[pq], uint8_t(1), __ATOMIC_RELAXED),
                       FH_EINVAL, "element logs: every element position must appear in exactly one log");
            }
          });
          ring.upload_copy(dl + base, h_cmd + base, cnt, stream);
        }
        if (!subset) unit_meta(nb, n, fq, d.keys_per_cmd, np, h_off, h_cmd, h_key);
      } else if (np <= 8) {
        views_entries<uint8_t>(nb, n, fq, np, h_off, h_cmd, dl);
      } else if (np <= 16) {
        views_entries<uint16_t>(nb, n, fq, np, h_off, h_cmd, dl);
      } else if (np <= 32) {
        views_entries<uint32_t>(nb, n, fq, np, h_off, h_cmd, dl);
      } else {
        views_entries<uint64_t>(nb, n, fq, np, h_off, h_cmd, dl);
      }
      h_loff = lo;
      FH_HIP(hipMemcpyAsync(loff.ensure(lo.size() + 1), lo.data(), lo.size() * sizeof(uint32_t),
                            hipMemcpyHostToDevice, stream));
      ensure_latest(d.nproc + 1);
    }
    stage_base = log_len;
    log_len += n * nb;
    log_ms = std::max(log_ms, smax_ms);
    log_mq = std::max(log_mq, smax_mq);
    stage_rid = h_rid;
    FH_HIP(hipStreamSynchronize(stream));
    desc = d;
    nbatches = nb;
    cursor = 0;
    staged = true;
    codes_only = subset;
  }

  // The device run of one batch: everything below is the timed hot path.
  void run(float *ms) {
    FH_CHECK(staged && cursor < nbatches, FH_EINVAL, "no staged batch left to run");
    FH_HIP(hipSetDevice(device));
    if (side) {
      // a run that threw between the side stream's fork and join left no
      // join behind: this run's kernels wait for whatever still runs there
      FH_HIP(hipEventRecord(ev_join, side));
      FH_HIP(hipStreamWaitEvent(stream, ev_join, 0));
    }
    clear_marks();
    graph.profile = profile;
    const uint32_t n = uint32_t(desc.n), k = desc.keys_per_cmd;
    const uint32_t fq = desc.views ? desc.views : 1;
    const uint32_t S = fq * k;
    const uint32_t M = n * S;
    const bool views = desc.views != 0;
    const size_t b = cursor++;
    last = b;
    last_deps_only = deps_only;
    ko_done = false;
    deps_rows = 0;
    rows32 = false;
    rows_packed = false;
    const uint64_t bbase = stage_base + b * n;  // log position of this batch
    const uint64_t *bdot = dot.get() + bbase;
    const uint32_t *bkey = key32.get() + b * size_t(n) * k;
    if (ms || profile) FH_HIP(hipEventRecord(ev0, stream));
    mark("start");
    struct ProbeGuard {
      ProbeGuard(Probe *p) { t_probe = p; }
      ~ProbeGuard() { t_probe = nullptr; }
    } probe_guard(probe.slots.empty() ? nullptr : &probe);
    uint32_t *vs = nullptr;
    uint64_t *dext = dep_ext.ensure(M + 1);  // per-element dependency codes
    uint32_t *svid = sorted_vid.ensure(M + 1);
    sorted_keys32 = nullptr;
    if (!views && k == 1) {
      uint32_t *ks = nullptr;
      uint64_t *dsorted = dep_ext.ensure(M + 1);
      const KeyBucketPlan plan = lat_mapped ? keybucket_plan(M, key_bits) : KeyBucketPlan();
      if (plan.ok) {
        // two launches: tile partition by key bucket, per-bucket order + deps
        ks = sk32a.ensure(M + 1);
        KeyBucketOut kout;
        kout.sk = ks;
        kout.seq = kb_seq.ensure(M + 1);
        kout.rows = o_rows.ensure(M + 1);
        // run bounds tagged per batch: cleared only when the tags wrap (or the
        // table is new)
        const bool fresh = kb_runs.cap < 2 * size_t(key_space) + 2;
        kout.runs = kb_runs.ensure(2 * size_t(key_space) + 2);
        if (fresh || ++kb_run_tag >= kRunTags) {
          FH_HIP(hipMemsetAsync(kout.runs, 0, 2 * size_t(key_space) * sizeof(uint32_t), stream));
          kb_run_tag = 1;
        }
        kout.run_tag = kb_run_tag;
        kout.bdot = bdot;
        kout.dlog = dot.get();
        // one launch per step: order this batch (partitioned by the previous
        // step, or now) and partition the next staged batch in the same grid
        const size_t q = b & 1;
        const KeyBucketClock clock = kb_clock(b);
        if (kb_next_part != b)
          keybucket_partition(plan, M, bkey, bdot, clock.fold, kb_ws[q], stream, &kb_sched);
        kb_next_part = ~size_t(0);
        if (b + 1 < nbatches) {
          keybucket_step(plan, M, bbase, latest.get(), kb_ws[q], kout, clock, plan, M,
                         bkey + M, bdot + M, kb_clock(b + 1).fold, kb_ws[q ^ 1], stream,
                         &kb_sched);
          kb_next_part = b + 1;
        } else {
          keybucket_order(plan, M, bbase, latest.get(), kb_ws[q], kout, clock, stream,
                          &kb_sched);
        }
        // refresh the schedule from the sizes just recorded: after the first
        // launch, then every 32 (the key distribution drifts slowly)
        if ((kb_launches++ & 31) == 0) keybucket_sched(kb_sched, stream);
        mark("keydeps_bucket");
        bucket_order = true;
      } else {
        sort_pairs<uint32_t, uint32_t>(bkey, nullptr, sk32a.ensure(M + 1), sva.ensure(M + 1),
                             sk32b.ensure(M + 1), svb.ensure(M + 1), M, key_bits, sort_ws, stream,
                             &ks, &vs);
        mark("keydeps_sort");
        const unsigned g = unsigned((M + 255) / 256);
        {
          // read key + vid (8), write the dependency (8)
          probed_launch("sv_deps", double(M) * 16.0, k_sv_deps, dim3(g), dim3(256), stream, M,
                        (const uint32_t *)ks, (const uint32_t *)vs,
                        (const uint64_t *)latest.get(), lmul, lmask, dsorted);
        }
        mark("deps");
        {
          // read key (4) and the batch dot (8)
          const unsigned gt = unsigned((M + kTailTile - 1) / kTailTile);
          probed_launch("sv_tails", double(M) * 12.0, k_sv_tails, dim3(gt), dim3(256), stream, M,
                        (const uint32_t *)ks, (const uint32_t *)vs, (const uint64_t *)bdot,
                        bbase, latest.get(), lmul, lmask,
                        reinterpret_cast<unsigned long long *>(frontier.get()), excount_ptr());
        }
        mark("tails_and_clock");
        bucket_order = false;
      }
      sv_vs = vs;
      // dependency graph: every dep is an earlier arrival (previous command
      // on the key in arrival order, or a latest entry from an executed
      // earlier batch), so SCCs are singletons and arrival order is a
      // topological order; the per-key sequence is the key-grouped order.
      gout = GraphOutput();
      gout.trivial = true;
      gout.nexec = n;
      gout.nelem = M;
      gout.pk_key = ks;
      gout.pk_vid = vs;
      sv_fused = true;
    } else if (!views) {
      sv_fused = false;
      uint32_t *ks = nullptr;
      sort_pairs<uint32_t, uint32_t>(bkey, nullptr, sk32a.ensure(M + 1), sva.ensure(M + 1),
                           sk32b.ensure(M + 1), svb.ensure(M + 1), M, key_bits, sort_ws, stream,
                           &ks, &vs);
      mark("keydeps_sort");
      k_prev_engine<uint32_t><<<grid_for(M, B), B, 0, stream>>>(
          M, ks, vs, 0, S, latest.get(), uint64_t(lmul), uint64_t(lmask), dext,
          k == 1 ? nullptr : svid);
      k_tail_engine<uint32_t><<<grid_for(M, B), B, 0, stream>>>(
          M, ks, vs, 0, S, latest.get(), uint64_t(lmul), uint64_t(lmask), nullptr, bbase);
      sorted_keys32 = ks;
    } else if (CmdMeta cm; cmd_meta(b, k, fq, n, &cm)) {
      sv_fused = false;
      if (keyorder_ok(b, fq, cm)) {
        ko_done = cmd_views_keyorder(b, n, fq, bkey, bdot, bbase, cm);
      } else {
        cmd_views(b, n, fq, M, bkey, bbase, cm);
        mark("keydeps_views");
      }
    } else {
      sv_fused = false;
      // every replica's KeyDeps over its arrival log, in chunks: chunk c
      // takes the c-th slice of each log (a replica's slices stay in arrival
      // order, so the latest table carries each (replica, key) segment across
      // chunks exactly as one sequential pass).  A chunk's commands sit in a
      // window of the stream, so its dependency scatter stays in a cache-
      // sized slice of the dependency array.
      const uint32_t np = desc.nproc;
      const bool elem = (desc.flags & FH_STREAM_ELEMENT_LOGS) != 0;
      FH_CHECK(np <= uint32_t(kMaxLogs), FH_ENOTIMPL, "replica views: nproc <= 64");
      const uint32_t *bl = h_loff.data() + b * size_t(np + 1);
      // codes placed through LDS buckets (k_place).  A chunk of Mc elements
      // spans ~Mc positions, so chunks of 15.7M keep the placement window
      // within its 2^24 positions.
      static const uint32_t place_slack = [] {
        const char *e = getenv("FH_PLACE_SLACK");  // tests: 0 makes reordered arrivals strays
        return e ? uint32_t(atol(e)) : kPlaceSlack;
      }();
      static const size_t chunk_elems = [] {
        const char *e = getenv("FH_VIEW_CHUNK");  // tests: small chunks
        return e ? size_t(std::max(1L, atol(e))) : size_t(15) << 20;
      }();
      // (chunks of chunk_elems log elements: with subset logs (fh_dgraph, one
      // rank's shards) the elements are a fraction of the M positions, and a
      // chunk's positions spread past the placement window, whose strays
      // k_place writes directly -- each bucket's strays fall in a few 128-KB
      // stripes.  Chunks of 15M positions instead made 77 chunks of 2.6M
      // elements at C5 / 8 ranks: 19.6 ms of per-chunk launches.)
      const uint32_t per_entry = elem ? 1u : k;  // elements per log entry
      const size_t tot = size_t(bl[np] - bl[0]) * per_entry;
      const uint32_t nch = uint32_t(std::max<size_t>(1, (tot + chunk_elems - 1) / chunk_elems));
      // the sentinel kPlaceNone is the code of log reference 2^31 - 1
      FH_CHECK(bbase + n < 0x7FFFFFFFull, FH_ENOTIMPL, "replica views: command log >= 2^31 - 1");
      uint32_t *pbase = place_base.ensure(nch);
      FH_HIP(hipMemsetAsync(pbase, 0xFF, size_t(nch) * sizeof(uint32_t), stream));
      // the chunk's elements are replica-major, so a stable sort by the key
      // alone already leaves every (replica, key) segment contiguous and in
      // arrival order ((key, replica, arrival) order): with K a power of two
      // the key is the composite's low bits (3 passes of 8-bit digits at
      // 2^20 keys, the last of 4 bits, instead of 3 full ones over the
      // 23-bit composite)
      const bool pow2 = (key_space & (key_space - 1)) == 0;
      const int bits = pow2 ? bits_for(key_space) : bits_for(uint64_t(np + 1) * key_space);
      const uint32_t *bent = lent.get() + (codes_only ? 0 : b * size_t(n) * fq * (elem ? k : 1));
      for (uint32_t c = 0; c < nch; c++) {
        LogChunk lc;
        lc.cum[0] = 0;
        for (uint32_t r = 0; r < np; r++) {
          const uint64_t len = bl[r + 1] - bl[r];
          const uint32_t q0 = uint32_t(len * c / nch), q1 = uint32_t(len * (c + 1) / nch);
          lc.first[r] = bl[r] + q0;
          lc.cum[r + 1] = lc.cum[r] + (q1 - q0) * per_entry;
        }
        const uint32_t Mc = lc.cum[np];
        uint32_t *lk = sk32a.ensure(Mc + 1), *lv = sva.ensure(Mc + 1);
        uint32_t *ks = nullptr;
        const uint32_t tiles = (Mc + kTile - 1) / kTile;
        sort_ws.prepare(tiles, 1, stream);
        const int db = sort_digit_bits(bits, 4);
        probed_launch("log_keys", double(Mc) * (4.0 + 4.0 + 8.0), k_log_keys, dim3(tiles),
                      dim3(kThreads), stream, Mc, k, fq, np, uint32_t(elem), lc, bent, bkey,
                      uint32_t(key_space), lk, lv, pbase + c, place_slack, sort_ws.meta.get(),
                      (1u << db) - 1);
        sort_pairs_counted<uint32_t, uint32_t>(lk, lv, sk32b.ensure(Mc + 1), svb.ensure(Mc + 1), Mc,
                                               bits, sort_ws, stream, &ks, &vs, db);
        // heads read the latest table, tails then make the chunk's last
        // commands the latest (command-log references); the sort's other
        // buffer pair takes the bucketed (position, code)
        uint32_t *bk = ks == lk ? sk32b.get() : lk, *bv = ks == lk ? svb.get() : lv;
        place_codes(Mc, ks, vs, S, pbase + c, bk, bv, dep32.ensure(M + 1), stream, bbase);
      }
      mark("keydeps_views");
    }
    if (codes_only) {
      // fh_dgraph: the codes of the staged positions are the output (dep32)
      if (ms || profile) FH_HIP(hipEventRecord(ev1, stream));
      if (ms) {
        FH_HIP(hipEventSynchronize(ev1));
        FH_HIP(hipEventElapsedTime(ms, ev0, ev1));
      }
      if (profile) collect_times();
      return;
    }
    if (!ko_done) {
      if (!sv_fused) run_general(n, k, fq, S, M, views, bkey, bdot, bbase);
      materialize(n, S, bdot);
    }
    if (ms || profile) FH_HIP(hipEventRecord(ev1, stream));
    if (ms) {
      FH_HIP(hipEventSynchronize(ev1));
      FH_HIP(hipEventElapsedTime(ms, ev0, ev1));
    }
    if (profile) collect_times();
  }

  // The command-level views path (k_cmd_search) applies to one key per
  // command, fast quorums of <= 4, and logs whose inversion span W leaves the
  // packed arrival positions enough bits (CmdMeta: 3W + 1 < 2^(qb-1)).
  // FH_VIEW_CMD=0 keeps the chunked path.
  bool cmd_meta(size_t b, uint32_t k, uint32_t fq, uint32_t n, CmdMeta *cm) const {
    static const bool on = [] {
      const char *e = getenv("FH_VIEW_CMD");
      return !(e && *e == '0');
    }();
    // element logs: the pair-level search over (command, key slot) units
    // when staging found it applicable (unit_meta)
    const bool units = (desc.flags & FH_STREAM_ELEMENT_LOGS) && !codes_only &&
                       b < h_unit_ok.size() && h_unit_ok[b];
    if (!on || fq > 4 || b >= h_win.size() || n < 2) return false;
    if (!units && (k != 1 || desc.nproc > uint32_t(kSrchMaxRep) ||
                   (desc.flags & FH_STREAM_ELEMENT_LOGS) || n >= (1u << kRecT)))
      return false;
    const uint64_t nu = uint64_t(n) * k;  // units
    if (units && nu >= (uint64_t(1) << 30)) return false;
    if (units) {  // log positions travel in kRecT bits of the view records
      const uint32_t *bl = h_loff.data() + b * size_t(desc.nproc + 1);
      for (uint32_t r = 0; r < desc.nproc; r++)
        if (bl[r + 1] - bl[r] >= (1u << kRecT)) return false;
    }
    CmdMeta m{};
    m.fq = fq;
    m.us = units ? uint32_t(__builtin_ctz(k)) : 0u;
    m.rb = uint32_t(bits_for(units ? unit_colors : desc.nproc));
    const int db = sort_digit_bits(key_bits, 4);
    const int passes = std::max(1, (key_bits + db - 1) / db);
    m.kb = uint32_t(passes * db);
    m.cb = uint32_t(bits_for(nu));
    // region records of 2^rsh units, at most kMaxRegions of them
    m.rsh = kRegShift;
    while (((nu - 1) >> m.rsh) + 1 > kMaxRegions) m.rsh++;
    if (m.kb > 32) return false;
    // the meta travels in the key word's and the value's free bits and is
    // handled as one u64
    const uint32_t spare = std::min<uint32_t>(64, (64 - m.cb) + (32 - m.kb));
    if (spare / fq <= m.rb + 2) return false;
    m.qb = std::min<uint32_t>(spare / fq - m.rb, uint32_t(kRecT));
    m.vb = m.rb + m.qb;
    m.kmask = key_bits >= 32 ? ~0u : (1u << key_bits) - 1;
    m.W = h_win[b];
    m.cmask = (uint64_t(1) << m.cb) - 1;
    m.qmask = (uint64_t(1) << m.qb) - 1;
    if (uint64_t(3) * m.W + 1 >= (uint64_t(1) << (m.qb - 1))) return false;
    *cm = m;
    return true;
  }

  // The key-order path applies to command-level batches with fast quorums of
  // 2 or 3 whose dots pack into 31 bits (the records' top bit marks a log
  // reference).
  bool keyorder_ok(size_t b, uint32_t fq, const CmdMeta &cm) const {
    return !keyorder_off && cm.us == 0 && desc.keys_per_cmd == 1 && (fq == 2 || fq == 3) &&
           b < h_dpack.size() &&
           h_dpack[b].second > 0 && h_dpack[b].second <= 31 && dot32.get() != nullptr;
  }

  // One batch through the key-order path (kernels above k_row_place): the
  // commands sorted by key once, carrying their packed dots; KeyDeps,
  // union entries, graph edges, the tile kernel and the per-key sequence in
  // key order; the committed deps, labels and execution ranks in command
  // order.  Returns false (after leaving command-order codes in dep32) if the
  // tile certificate fails, so the general path takes the batch.
  bool cmd_views_keyorder(size_t b, uint32_t n, uint32_t fq, const uint32_t *bkey,
                          const uint64_t *bdot, uint64_t bbase, const CmdMeta &cm) {
    const uint32_t np = desc.nproc;
    const int sb = h_dpack[b].first;
    LogOffs lo{};
    const uint32_t *bl = h_loff.data() + b * size_t(np + 1);
    for (uint32_t r = 0; r <= np; r++) lo.off[r] = bl[r];
    for (uint32_t r = 0; r < np; r++) lo.rid[r] = h_rid[r];
    const uint32_t *bent = lent.get() + b * size_t(n) * fq;
    const uint32_t M = n * fq;
    uint32_t *rec = vrec.ensure(M + 1);
    const uint32_t per = std::max<uint32_t>(1, (kRecWin - 2 * rec_slack(kRecWin)) / fq);
    const uint32_t G = std::max<uint32_t>(1, (n + per - 1) / per);
    const uint32_t tiles = (n + kTile - 1) / kTile;
    sort_ws.prepare(tiles, 1, stream);
    const int db = sort_digit_bits(key_bits, 4);
    if (!side_off && !side) FH_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    // the pass-0 tile counts need only the keys: on the side stream beside
    // the view records
    // (k_cmd_pack3 writing the packed arrays, then the sort: 724 + 864 against
    // 1226 us per C4 step for the first pass producing its own input, r05r)
    hipStream_t ks0 = side_off ? stream : side;
    if (!side_off) {
      FH_HIP(hipEventRecord(ev_fork, stream));
      FH_HIP(hipStreamWaitEvent(side, ev_fork, 0));
    }
    k_key_counts<<<dim3(tiles), dim3(kThreads), 0, ks0>>>(n, bkey, sort_ws.meta.get(),
                                                          (1u << db) - 1);
    probed_launch("view_records", double(M) * (4.0 + 4.0), k_view_records<kRecWin>, dim3(G),
                  dim3(1024), stream, n, fq, np, G, lo, bent, rec, (const uint32_t *)nullptr);
    if (!side_off) {
      FH_HIP(hipEventRecord(ev_join, side));
      FH_HIP(hipStreamWaitEvent(stream, ev_join, 0));
    }
    uint32_t *kwa = sk32a.ensure(n + 1);
    V3 *va = kv3a.ensure(n + 1);
    uint32_t *ks = nullptr;
    V3 *vs = nullptr;
    const PackSrc src{cm, bkey, rec, dot32.get() + b * size_t(n)};
    sort_pairs_counted_src<uint32_t, V3, PackSrc>(src, kwa, va, sk32b.ensure(n + 1),
                                                  kv3b.ensure(n + 1), n, key_bits, sort_ws,
                                                  stream, &ks, &vs, db);
    uint8_t *tm = tailm.ensure(n + 16);  // (k_cmd_tails reads it 16 bytes at a time)
    const size_t mwords = (size_t(n) + 3) / 4;
    uint32_t *mr = mrem.ensure(mwords);
    FH_HIP(hipMemsetAsync(mr, 0, mwords * sizeof(uint32_t), stream));
    // 512-command tiles: four workgroups per CU (38 KB of LDS each) against two
    // at 1024, so one tile's staging and barriers overlap three others' scans
    // (C4, ms per step: 1024 13.39 / 13.70, 512 12.41 / 12.43, 256 13.82 /
    // 14.08, r05th / r05th2; halos of 64 or 32 instead of 128: no different,
    // r05ha; tiles contiguous per XCD, so a tile's halo sits in the L2 its
    // predecessor staged it through: 13.84 against 12.94, r05xc)
    const uint32_t sth = kKoSrchThreads;
    const uint32_t stiles = (n + sth - 1) / sth;
    const uint32_t nreg = uint32_t((uint64_t(n) - 1) >> kRegShift) + 1;
    FH_CHECK(nreg <= kMaxRegions, FH_EINVARIANT, "command regions");
    uint4 *rec4 = crec.ensure(size_t(n) + 1);
    uint32_t *rcur = ctoff.ensure(kMaxRegions);
    FH_HIP(hipMemsetAsync(rcur, 0, kMaxRegions * sizeof(uint32_t), stream));
    uint32_t *pcode = kpcode.ensure(size_t(n) * fq + 1);
    uint32_t *pd32 = kpd32.ensure(n + 1);
    uint32_t *pe8 = kpe8.ensure(n + 1);
    uint32_t *codes = dep32.ensure(size_t(M) + 1);
    const uint32_t K = uint32_t(key_space);
    const uint64_t *lat = views_latest();
    // the straddle differences the tile kernel writes, cleared here: after
    // the search the engine stream's next launch must be the tile kernel
    // itself, or the side stream's kernels start first and take the CUs (a
    // 66-us kernel in between cost 2 ms)
    if (!deps_only)
      FH_HIP(hipMemsetAsync(kdiff.ensure(n + 2), 0, size_t(n + 1) * sizeof(uint32_t), stream));
    auto go = [&](auto kern) {
      probed_launch("cmd_search", double(n) * (16.0 + 16.0 + 4.0 * fq + 4.0 + 1.0), kern,
                    dim3(stiles), dim3(sth), stream, n, cm, K, np, (const uint32_t *)ks,
                    (const V3 *)vs, lat, codes, rec4, rcur, tm, mr, pcode, pd32, pe8);
    };
    if (fq == 2)
      go(k_cmd_search<2, kKoSrchThreads, V3, true>);
    else
      go(k_cmd_search<3, kKoSrchThreads, V3, true>);
    mark("keydeps_views");
    // The command-order half -- the records' entries to their commands
    // (region by region), the tails, the committed deps -- needs nothing the
    // graph computes, and the graph needs none of it: it runs on the side
    // stream while the tile kernel (latency bound, one workgroup per CU)
    // runs here.
    hipStream_t cs = side_off ? stream : side;
    ScanWorkspace &cws = side_off ? scan_ws : scan_ws2;
    if (!side_off) {
      FH_HIP(hipEventRecord(ev_fork, stream));
      FH_HIP(hipStreamWaitEvent(side, ev_fork, 0));
    }
    auto join = [&] {
      if (side_off) return;
      FH_HIP(hipEventRecord(ev_join, side));
      FH_HIP(hipStreamWaitEvent(stream, ev_join, 0));
    };
    const unsigned sg = side_off ? ~0u : side_grid;
    const dim3 gs(grid_for(n, B, std::min(sg, 1u << 30)));
    const dim3 gs8(grid_for(n, B, std::min(sg, 8192u)));
    // committed deps (QuorumDeps union, deps/quorum.rs:28-98): the records'
    // entries are dots already, so each command's row is written in one pass
    // (round 5: a scatter of the entries to command order, a count pass, a
    // scan and the union, 4.5 ms alone)
    // the union's error word (results() checks it)
    FH_HIP(hipMemsetAsync(scal.get(), 0, 2 * sizeof(uint32_t), cs));
    // rows of 32-bit packed dots when every dot of the log packs with this
    // batch's layout (any earlier batch's dot a row may name): half the
    // scattered row bytes, and the tile kernel beside them waits less on the
    // write path -- C4 11.87 against 12.79 ms per step with u64 rows
    // (k_row_place 3.82 -> 2.63 ms, the tile kernel 5.22 -> 4.35 ms; same
    // box, r06r32)
    rows32 = bits_for(log_mq + 1) <= sb && sb + bits_for(log_ms + 1) <= 31;
    rows_sb = sb;
    const uint64_t *dl = dot.get();
    if (rows32) {
      uint32_t *rows = o_rows32.ensure(size_t(n) * fq + 1);
      if (fq == 2)
        probed_launch("row_place", double(n) * (16.0 + 8.0), k_row_place<2, uint32_t>, gs, dim3(B),
                      cs, n, (const uint4 *)rec4, dl, sb, rows, scal.get() + 1);
      else
        probed_launch("row_place", double(n) * (16.0 + 12.0), k_row_place<3, uint32_t>, gs,
                      dim3(B), cs, n, (const uint4 *)rec4, dl, sb, rows, scal.get() + 1);
    } else {
      uint64_t *rows = o_rows.ensure(size_t(n) * fq + 1);
      if (fq == 2)
        probed_launch("row_place", double(n) * (16.0 + 16.0), k_row_place<2>, gs, dim3(B), cs, n,
                      (const uint4 *)rec4, dl, sb, rows, scal.get() + 1);
      else
        probed_launch("row_place", double(n) * (16.0 + 24.0), k_row_place<3>, gs, dim3(B), cs, n,
                      (const uint4 *)rec4, dl, sb, rows, scal.get() + 1);
    }
    k_cmd_tails<V3><<<gs8, B, 0, cs>>>(n, cm, K, ks, vs, tm,
                                                 reinterpret_cast<const uint8_t *>(mr),
                                                 views_latest(), bbase);
    deps_rows = fq;
    // per-key offsets: a lower bound per key over the sorted keys (they
    // need nothing else; the side stream has slack beside the tile kernel)
    if (!deps_only)
      k_key_offsets<<<grid_for(uint32_t(key_space) + 1, B), B, 0, cs>>>(
          n, ks, uint32_t(key_space), key_offs.ensure(key_space + 2), cm.kmask);
    if (deps_only) {
      join();
      mark("keydeps_union");
      return true;
    }
    // the key-order graph on the tile path
    GraphInput gin;
    gin.V = n;
    gin.stride = fq;
    gin.dst = pe8;
    gin.dst_codes = true;
    gin.dst_esc = pcode;
    // (C4: 14.91 against 14.94 ms at normal priority, r05u)
    gin.tile_prio = !side_off;
    gin.dot32 = pd32;
    gin.dot32_sb = sb;
    gin.k = 1;
    gin.key_bits = key_bits;
    gin.want_per_key = false;
    gin.tiles_only = true;
    // the tiles write the per-key sequence and the command-order records
    uint64_t *sq = seq_dot.ensure(n + 1);
    uint32_t *diff = kdiff.ensure(n + 2);  // (cleared before the search)
    uint4 *hl = khl.ensure(n + 1);
    gin.ko_seq = sq;
    gin.ko_hl = hl;
    gin.ko_diff = diff;
    gin.ko_cmd = reinterpret_cast<const uint32_t *>(vs);
    gin.ko_cstride = 3;
    gin.ko_cmask = uint32_t(cm.cmask);
    // (tried: the tile kernel at 5120-vertex contexts, two workgroups per
    // CU, R0 = 256, T = 4096: 4.45 against 3.2 ms per C4 step -- twice the
    // tiles and their barrier-bound fixed phases)
    graph.run(gin, gout);
    if (gout.nexec == 0) {
      // certificate failure: command-order codes for the general path
      join();
      deps_rows = 0;
      // the records' entries to command order (the general path's codes)
      if (fq == 2)
        k_code_scatter<2><<<grid_for(n, B), B, 0, stream>>>(n, (const uint4 *)rec4, codes);
      else
        k_code_scatter<3><<<grid_for(n, B), B, 0, stream>>>(n, (const uint4 *)rec4, codes);
      if (fq == 2)
        k_pcode_to_vid<2><<<grid_for(n, B), B, 0, stream>>>(n, vs, cm.cmask, pe8, pcode, codes);
      else
        k_pcode_to_vid<3><<<grid_for(n, B), B, 0, stream>>>(n, vs, cm.cmask, pe8, pcode, codes);
      return false;
    }
    unsigned long long *stt = srcstats.ensure(4 * 256);
    FH_HIP(hipMemsetAsync(stt + 256, 0, 512 * sizeof(unsigned long long), stream));
    uint32_t *ss = kss.ensure(n + 2);
    exclusive_scan_u32(diff, ss, n + 1, scan_ws, stream);
    mark("ko_straddle");
    uint64_t *lb = lab.ensure(n + 1);
    uint32_t *rk = rank_tmp.ensure(n + 1);
    probed_launch("ko_final", double(n) * (4.0 + 8.0 + 8.0 + 4.0), k_ko_final,
                  dim3(grid_for(n, 256, 8192)), dim3(256), stream, n, (const uint32_t *)diff,
                  (const uint4 *)hl, (const uint32_t *)ss, bdot, lb, rk, stt + 256,
                  reinterpret_cast<unsigned int *>(stt + 512));
    k_frontier_update<<<1, 256, 0, stream>>>(stt + 256, reinterpret_cast<unsigned int *>(stt + 512),
                                             frontier.get(), excount_ptr());
    o_label = lb;
    o_rank = rk;
    o_seq = sq;
    o_nelem = n;
    mark("out_per_key");
    join();
    mark("keydeps_union");
    return true;
  }

  // (units: element logs through the pair-level search, n commands of k
  // keys = n·k units; cm.us = log2 k; every array below is per unit)
  void cmd_views(size_t b, uint32_t nc, uint32_t fq, uint32_t M, const uint32_t *bkey,
                 uint64_t bbase, const CmdMeta &cm) {
    const uint32_t np = desc.nproc;
    const uint32_t n = nc << cm.us;  // units
    // replica ids the search indexes its per-replica slots by: the logs, or
    // their colouring (units; unit_meta)
    const uint32_t nrep = cm.us || (desc.flags & FH_STREAM_ELEMENT_LOGS) ? unit_colors : np;
    FH_CHECK(nrep >= 1 && nrep <= uint32_t(kSrchMaxRep), FH_EINVARIANT, "search replicas");
    LogOffs lo{};
    const uint32_t *bl = h_loff.data() + b * size_t(np + 1);
    for (uint32_t r = 0; r <= np; r++) lo.off[r] = bl[r];
    for (uint32_t r = 0; r < np; r++) lo.rid[r] = h_rid[r];
    const uint32_t *bent = lent.get() + b * size_t(M);
    uint32_t *rec = vrec.ensure(M + 1);
    // ~4800 commands per workgroup: fq·4800 + slack positions fit the window
    // (tried: 8K windows 1391 us per C4 launch, 32K 1072, 16K 935); element
    // logs hold fq·k elements per command
    const uint32_t epc = fq << cm.us;
    const uint32_t per = std::max<uint32_t>(1, (kRecWin - 2 * rec_slack(kRecWin)) / epc);
    const uint32_t G = std::max<uint32_t>(1, (nc + per - 1) / per);
    const uint32_t *vb = nullptr;
    if (cm.us || (desc.flags & FH_STREAM_ELEMENT_LOGS)) {
      FH_CHECK(b < h_vbnd_g.size() && h_vbnd_g[b] == G, FH_EINVARIANT, "view record slices");
      vb = vbnd.get() + h_vbnd_off[b];
    }
    probed_launch("view_records", double(M) * (4.0 + 4.0), k_view_records<kRecWin>, dim3(G),
                  dim3(1024), stream, nc, epc, np, G, lo, bent, rec, vb);
    mark(cm.us ? "unit_records" : "cmd_records");
    const uint32_t tiles = (n + kTile - 1) / kTile;
    sort_ws.prepare(tiles, 1, stream);
    const int db = sort_digit_bits(key_bits, 4);
    uint32_t *kwa = sk32a.ensure(n + 1);
    uint64_t *va = cv64a.ensure(n + 1);
    // reads the key and fq records, writes the key word and the value
    probed_launch("cmd_pack", double(n) * (4.0 + 4.0 * fq + 4.0 + 8.0), k_cmd_pack, dim3(tiles),
                  dim3(kThreads), stream, n, cm, bkey, (const uint32_t *)rec, kwa, va,
                  sort_ws.meta.get(), (1u << db) - 1);
    uint32_t *ks = nullptr;
    uint64_t *vs = nullptr;
    sort_pairs_counted<uint32_t, uint64_t>(kwa, va, sk32b.ensure(n + 1), cv64b.ensure(n + 1), n,
                                           key_bits, sort_ws, stream, &ks, &vs, db);
    mark(cm.us ? "unit_sort" : "cmd_sort");
    uint8_t *tm = tailm.ensure(n + 16);  // (k_cmd_tails reads it 16 bytes at a time)
    // predecessor marks from other tiles (k_cmd_search, k_cmd_tails)
    const size_t mwords = (size_t(n) + 3) / 4;
    uint32_t *mr = mrem.ensure(mwords);
    FH_HIP(hipMemsetAsync(mr, 0, mwords * sizeof(uint32_t), stream));
    // reads the sorted key words and values (12 B, neighbours from LDS) and
    // the heads' latest entries, writes fq codes (through region records when
    // fq <= 3) and the tail mask.  1024 threads (tried 256 / 512: flat)
    uint32_t *codes = dep32.ensure(size_t(M) + 1);
    // units (element logs): 512-unit tiles, four workgroups per CU, as the
    // key-order path measured faster than 1024 (§5.1 item 4)
    const bool t512 = (cm.us || (desc.flags & FH_STREAM_ELEMENT_LOGS)) && (fq == 2 || fq == 3);
    const uint32_t sth = t512 ? 512u : uint32_t(kSrchThreads);
    const uint32_t stiles = (n + sth - 1) / sth;
    const uint32_t nreg = uint32_t((uint64_t(n) - 1) >> cm.rsh) + 1;
    FH_CHECK(nreg <= kMaxRegions, FH_EINVARIANT, "command regions");
    uint4 *rec4 = nullptr;
    uint32_t *rcur = nullptr;
    if (fq <= 3) {
      rec4 = crec.ensure(size_t(n) + 1);
      rcur = ctoff.ensure(kMaxRegions);
      FH_HIP(hipMemsetAsync(rcur, 0, kMaxRegions * sizeof(uint32_t), stream));
    }
    const double sb = double(n) * (12.0 + (rec4 ? 16.0 : fq * 4.0) + 1.0);
    const uint32_t K = uint32_t(key_space);
    const uint64_t *lat = views_latest();
    auto go = [&](auto kern) {
      probed_launch("cmd_search", sb, kern, dim3(stiles), dim3(sth), stream, n, cm, K, nrep,
                    (const uint32_t *)ks, (const uint64_t *)vs, lat, codes, rec4, rcur, tm, mr,
                    (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr);
    };
    if (t512 && fq == 3)
      go(k_cmd_search<3, 512, uint64_t, false>);
    else if (t512 && fq == 2)
      go(k_cmd_search<2, 512, uint64_t, false>);
    else
      switch (fq) {
        case 1: go(k_cmd_search<1, kSrchThreads, uint64_t, false>); break;
        case 2: go(k_cmd_search<2, kSrchThreads, uint64_t, false>); break;
        case 3: go(k_cmd_search<3, kSrchThreads, uint64_t, false>); break;
        default: go(k_cmd_search<4, kSrchThreads, uint64_t, false>); break;
      }
    mark(cm.us ? "unit_search" : "cmd_search");
    if (rec4) {
      auto sc = [&](auto kern) {
        probed_launch("code_scatter", double(n) * (16.0 + 4.0 * fq), kern,
                      dim3((n + 255) / 256), dim3(256), stream, n, (const uint4 *)rec4, codes);
      };
      switch (fq) {
        case 1: sc(k_code_scatter<1>); break;
        case 2: sc(k_code_scatter<2>); break;
        default: sc(k_code_scatter<3>); break;
      }
    }
    k_cmd_tails<uint64_t><<<grid_for(n, B), B, 0, stream>>>(n, cm, uint32_t(key_space), ks, vs, tm,
                                                  reinterpret_cast<const uint8_t *>(mr),
                                                  views_latest(), bbase);
  }

  // The chunk's dependency codes -> dep32 through the placement pass: bucket
  // (position - base, code) by the position's bits [15, 23) with the radix
  // kernels (PrevSrc computes each code on the fly), then k_place per bucket.
  // The bucketing pass also makes the segment tails the latest entries (log
  // references log_base + command).
  void place_codes(uint32_t Mc, const uint32_t *ks, const uint32_t *vs, uint32_t per_cmd,
                   const uint32_t *ebase, uint32_t *bk, uint32_t *bv, uint32_t *out,
                   hipStream_t s, uint64_t log_base) {
    if (Mc == 0) return;
    const PrevSrc src{ks, vs, ebase, (const uint64_t *)views_latest(), per_cmd};
    const uint32_t tiles = (Mc + kTile - 1) / kTile;
    const uint32_t groups = (tiles + kGroup - 1) / kGroup;
    sort_ws.prepare(tiles, 1, s);
    constexpr uint32_t R = kPlaceBuckets;
    uint32_t *counts = sort_ws.meta.get();
    uint32_t *gsum = counts + size_t(tiles) * R;
    uint32_t *dbase = gsum + size_t(std::max<uint32_t>(groups, 4)) * R;
    // runs of a key's consecutive elements mostly share a bucket: one atomic
    // per run (k_up)
    k_up<uint32_t, uint32_t, kPlaceDB, PrevSrc><<<tiles, kThreads, 0, s>>>(src, Mc, kPlaceShift,
                                                                            counts);
    k_scan_a<kPlaceDB><<<dim3(groups, R / 256), 256, 0, s>>>(counts, tiles, gsum);
    scan_b<kPlaceDB>(gsum, groups, dbase, s);
    // reads (key, arrival) keys + positions, the previous element's, and the
    // latest table at heads; writes 8 B per element
    const uint32_t nb = (tiles + 1) / 2;
    uint32_t *defer = tail_defer.ensure(2 * size_t(nb));
    probed_launch("prev_bucket", double(Mc) * (4.0 + 4.0 + 8.0), k_bucket_codes,
                  dim3(nb), dim3(kBucketThreads), s, src, bk, bv, Mc, (const uint32_t *)counts,
                  (const uint32_t *)gsum, uint32_t(kGroup), (const uint32_t *)dbase,
                  views_latest(), log_base, defer);
    FH_CHECK(nb <= size_t(R) * 1024, FH_EINVAL, "placement: too many bucketing workgroups");
    probed_launch("place", double(Mc) * (8.0 + 4.0), k_place, dim3(R), dim3(1024), s, Mc,
                  (const uint32_t *)dbase, (const uint32_t *)bk, (const uint32_t *)bv, ebase, out,
                  (const uint32_t *)defer, nb, views_latest(), log_base);
  }

  void run_general(uint32_t n, uint32_t k, uint32_t fq, uint32_t S, uint32_t M, bool views,
                   const uint32_t *bkey, const uint64_t *bdot, uint64_t bbase) {
    uint32_t *svid = sorted_vid.get();
    mark("keydeps_prev");
    uint32_t *dcnt = dep_cnt.ensure(n + 1);
    uint32_t *dd = dst.ensure(M + 1);
    FH_HIP(hipMemsetAsync(scal.get(), 0, 2 * sizeof(uint32_t), stream));
    uint32_t *ecnt = views && S >= 8 ? edge_cnt.ensure(n + 1) : (uint32_t *)nullptr;
    // rows of <= kRegSlots slots: count, scan, and the union writes the
    // committed-deps CSR directly; wider rows go through fixed-stride rows.
    // (Tried, round 3: the committed dots -- an output nothing later in the
    // step reads -- on a second stream beside the graph stage, which needs
    // only the edges.  The graph kernels slowed down more than the union's
    // 3.3 ms they would hide: 21.8 against 21.6 ms per C4 step.)
    deps_direct = S <= kRegSlots;
    uint64_t *ddot = nullptr;
    const uint32_t *doff = nullptr;
    if (deps_direct) {
      doff = o_dep_off.ensure(n + 1);
      ddot = o_dep.ensure(M + 1);
      if (views)
        k_cmd_count<uint32_t><<<grid_for(n, B), B, 0, stream>>>(
            n, S, (const uint32_t *)dep32.get(), (const uint64_t *)dot.get(), bbase, dcnt);
      else
        k_cmd_count<uint64_t><<<grid_for(n, B), B, 0, stream>>>(
            n, S, (const uint64_t *)dep_ext.get(), (const uint64_t *)dot.get(), bbase, dcnt);
      exclusive_scan_u32(dcnt, o_dep_off.get(), n, scan_ws, stream);
      mark("keydeps_count");
    } else {
      ddot = dep_dot.ensure(M + 1);
    }
    // rows of <= 4 slots: XCD-contiguous blocks (k_cmd_engine)
    const uint32_t g = S <= 4 ? (grid_for(n, B, 1u << 22) + 7) / 8 * 8 : grid_for(n, B);
    // the batch's packed dots (staged), when they fit 32 bits
    const size_t bcur = cursor - 1;
    const bool packed = bcur < h_dpack.size() && h_dpack[bcur].second > 0 && dot32.get();
    const uint32_t *bdot32 = packed ? dot32.get() + bcur * size_t(n) : nullptr;
    const int bsb32 = packed ? h_dpack[bcur].first : 0;
    // wide rows (C5: 12 slots) write their edges into the committed-deps CSR
    // rows (the in-batch deps are a subset), so no edge compaction pass; the
    // union also counts the forward edges for the graph stage
    const bool edges_at_deps = views && S >= 8 && deps_direct;
    unsigned long long *fwd = views && S >= 8 ? fwd_ctr.ensure(64) : nullptr;
    if (fwd) FH_HIP(hipMemsetAsync(fwd, 0, 64 * sizeof(unsigned long long), stream));
    if (views)
      probed_launch("cmd_union", double(n) * (S * 4.0 + 8.0 * S + 4.0 * S + 4.0),
                    k_cmd_engine<uint32_t>, dim3(g), dim3(B), stream, n, S, bdot,
                    (const uint32_t *)dep32.get(), (const uint64_t *)dot.get(),
                    (const uint64_t *)frontier.get(), ddot, dcnt, dd, (uint8_t *)nullptr,
                    scal.get(), edges_at_deps ? (uint32_t *)nullptr : ecnt, bbase, doff,
                    scal.get() + 1, 0u, uint32_t(edges_at_deps), fwd, bdot32, bsb32);
    else
      probed_launch("cmd_union", double(n) * (S * 8.0 + 8.0 * S + 4.0 * S + 4.0),
                    k_cmd_engine<uint64_t>, dim3(grid_for(n, B)), dim3(B), stream, n, S, bdot,
                    (const uint64_t *)dep_ext.get(), (const uint64_t *)dot.get(),
                    (const uint64_t *)frontier.get(), ddot, dcnt, dd, (uint8_t *)nullptr,
                    scal.get(), ecnt, bbase, doff, scal.get() + 1, 0u, 0u,
                    (unsigned long long *)nullptr, (const uint32_t *)nullptr, 0);
    mark("keydeps_union");
    if (deps_only) return;  // the committed deps are the output (partial replication)
    const uint32_t *gdst = dd, *goff = nullptr;
    if (edges_at_deps) {
      goff = doff;
    } else if (views && S >= 8) {  // measured: a win at S = 12 (C5), flat or worse at 3 and 6
      uint32_t *eo = edge_off.ensure(n + 1);
      exclusive_scan_u32(edge_cnt.get(), eo, n, scan_ws, stream);
      uint32_t *ec = edge_csr.ensure(size_t(n) * S + 1);
      k_edges_csr<<<grid_for(n, B), B, 0, stream>>>(n, S, dd, eo, ec);
      gdst = ec;
      goff = eo;
      mark("edges_csr");
    }
    // graph stage
    GraphInput gin;
    gin.V = n;
    gin.off = goff;
    gin.stride = goff ? 0 : S;
    gin.dst = gdst;
    gin.blocked0 = nullptr;  // see k_cmd_engine: no pending carried by the fused engine
    gin.fwd_counts = fwd;    // forward edges, counted by the union
    gin.dot = bdot;
    gin.k = k;
    gin.key32 = bkey;
    gin.key_bits = key_bits;
    if (!views) {
      gin.no_forward_hint = true;  // single view: deps always point backwards
      gin.sorted_keys = sorted_keys32;
      gin.sorted_vid = svid;
    }
    gin.per_key_dots = true;
    if (cursor >= 1 && cursor - 1 < h_dpack.size()) {
      gin.dot_sb = h_dpack[cursor - 1].first;
      gin.dot_pbits = h_dpack[cursor - 1].second;
    }
    // the executed-clock stats ride on the per-key pass's dot reads
    unsigned long long *stt = srcstats.ensure(4 * 256);
    FH_HIP(hipMemsetAsync(stt + 256, 0, 512 * sizeof(unsigned long long), stream));
    gin.src_mx = stt + 256;
    gin.src_cnt = reinterpret_cast<unsigned int *>(stt + 512);
    graph.run(gin, gout);
    FH_CHECK(gout.npending == 0, FH_EINVARIANT, "fused engine batch left pending vertices");
    // per-key sequence of dots (ExecutionOrderMonitor::add order)
    if (gout.pk_dot) {
      o_seq = gout.pk_dot;
    } else {
      uint64_t *sq = seq_dot.ensure(gout.nelem + 1);
      k_seq_dots<<<grid_for(gout.nelem, B), B, 0, stream>>>(gout.nelem, gout.pk_vid, bdot, sq);
      o_seq = sq;
      mark("per_key_dots");
    }
    // executed clock: the whole batch executed
    unsigned long long *st = srcstats.get();
    if (!gout.src_stats_done)
      k_src_stats<<<grid_for(n, B, 1024), B, 0, stream>>>(n, bdot, st + 256,
                                                      reinterpret_cast<unsigned int *>(st + 512));
    k_frontier_update<<<1, 256, 0, stream>>>(st + 256, reinterpret_cast<unsigned int *>(st + 512),
                                             frontier.get(), excount_ptr());
    mark("executed_clock");
  }

  // The run's outputs, materialised on the device before run() returns:
  // committed deps as CSR of dots (o_dep_off, o_dep), SCC labels and
  // execution ranks (o_label, o_rank), per-key offsets over the key space
  // (key_offs) and the per-key execution sequences of dots (seq_dot).
  // results() only copies them to the host.
  void materialize(uint32_t n, uint32_t S, const uint64_t *bdot) {
    uint32_t *off = o_dep_off.ensure(n + 1);
    if (!sv_fused && deps_direct) {
      // written by the union (k_cmd_count sized the rows)
    } else {
    if (sv_fused && bucket_order) {
      // the order launch wrote each command's row (one slot per command)
      deps_rows = 1;
      sv_labels_done = false;
    } else if (sv_fused) {
      // one dependency slot per command: the rows themselves; the trivial
      // order's labels and ranks in one coalesced pass
      uint64_t *lb = gout.trivial ? lab.ensure(n + 1) : nullptr;
      uint32_t *rk = gout.trivial ? rank_tmp.ensure(n + 1) : nullptr;
      k_sv_rows<<<grid_for(n, B), B, 0, stream>>>(n, sv_vs, dep_ext.get(), bdot, dot.get(),
                                                   o_rows.ensure(n + 1), lb, rk);
      deps_rows = 1;
      sv_labels_done = gout.trivial;
    } else {
      exclusive_scan_u32(dep_cnt.get(), off, n, scan_ws, stream);
      k_compact_deps<<<grid_for(n, B), B, 0, stream>>>(n, S, dep_dot.get(), off,
                                                        o_dep.ensure(size_t(n) * S + 1));
    }
    }
    mark("out_deps");
    if (deps_only) return;
    if (gout.trivial && sv_fused && bucket_order) {
      // (written with the per-key sequence below)
      o_label = lab.ensure(n + 1);
      o_rank = rank_tmp.ensure(n + 1);
    } else if (gout.trivial && sv_fused && sv_labels_done) {
      o_label = lab.get();
      o_rank = rank_tmp.get();
    } else if (gout.trivial) {
      // singleton SCCs in arrival order: label = own dot, rank = position
      uint64_t *lb = lab.ensure(n + 1);
      uint32_t *rk = rank_tmp.ensure(n + 1);
      k_identity_labels<<<grid_for(n, B), B, 0, stream>>>(n, bdot, lb, rk);
      o_label = lb;
      o_rank = rk;
    } else {
      o_label = gout.scc_label;
      o_rank = gout.exec_rank;
    }
    // per-key offsets over the ascending key space (histogram + scan)
    o_nelem = gout.nelem;
    uint32_t *o = key_offs.ensure(key_space + 2);
    uint32_t *dl = nullptr;
    if (sv_fused && bucket_order) {
      // key-grouped runs (not ascending): one scan over the run bounds the
      // order launch wrote gives the offsets and each run's shift
      dl = kb_delta.ensure(key_space + 1);
      run_offsets(kb_runs.get(), kb_run_tag, o, dl, key_space, scan_ws, stream);
    } else {
      k_key_offsets<<<grid_for(uint32_t(key_space) + 1, B), B, 0, stream>>>(
          o_nelem, gout.pk_key, uint32_t(key_space), o);
    }
    if (sv_fused) {
      uint64_t *sq = seq_dot.ensure(o_nelem + 1);
      if (bucket_order) {
        // key-grouped runs -> ascending keys; the trivial labels and ranks
        // in the same pass
        k_run_place<<<grid_for(o_nelem, B), B, 0, stream>>>(o_nelem, gout.pk_key, dl, kb_seq.get(),
                                                             sq, bdot, lab.get(), rank_tmp.get());
      } else {  // (sorted keys, sorted vids): gather the dots
        k_seq_dots<<<grid_for(o_nelem, B), B, 0, stream>>>(o_nelem, gout.pk_vid, bdot, sq);
      }
      o_seq = sq;
    }  // else: run_general set o_seq
    mark("out_per_key");
  }

  void collect_times() {
    FH_HIP(hipStreamSynchronize(stream));
    last_times.clear();
    for (size_t i = 1; i < marks.size(); i++) {
      float t = 0;
      FH_HIP(hipEventElapsedTime(&t, marks[i - 1].second, marks[i].second));
      last_times.push_back({marks[i].first, t});
    }
  }

  // results of the last run (materialised by run()): device -> host copies
  void results(uint32_t *dep_off, uint64_t *dep_out, size_t dep_cap, size_t *dep_len,
               uint64_t *scc_label, uint32_t *exec_rank, uint32_t *key_off, uint64_t *key_seq) {
    FH_HIP(hipSetDevice(device));
    FH_CHECK(staged && cursor > 0, FH_EINVAL, "no run to read results from");
    FH_CHECK(!codes_only, FH_EINVAL, "subset logs: the run computed KeyDeps codes only");
    FH_CHECK(!last_deps_only || (!scc_label && !exec_rank && !key_off && !key_seq), FH_EINVAL,
             "deps-only run: only the committed deps are materialised");
    FH_HIP(hipStreamSynchronize(stream));
    const uint32_t n = uint32_t(desc.n);
    if (deps_rows && !rows_packed) {
      // the rows -> the ABI's CSR (o_dep_off, o_dep) on the device, once
      uint32_t *cnt = dep_cnt.ensure(n + 1);
      uint32_t *off = o_dep_off.ensure(n + 1);
      uint64_t *dep = o_dep.ensure(size_t(n) * deps_rows + 1);
      if (rows32) {
        k_rows32_count<<<grid_for(n, B), B, 0, stream>>>(n, deps_rows, o_rows32.get(), cnt);
        exclusive_scan_u32(cnt, off, n, scan_ws, stream);
        k_rows32_compact<<<grid_for(n, B), B, 0, stream>>>(n, deps_rows, o_rows32.get(), rows_sb,
                                                            off, dep);
      } else {
        k_rows_count<<<grid_for(n, B), B, 0, stream>>>(n, deps_rows, o_rows.get(), cnt);
        exclusive_scan_u32(cnt, off, n, scan_ws, stream);
        k_rows_compact<<<grid_for(n, B), B, 0, stream>>>(n, deps_rows, o_rows.get(), off, dep);
      }
      FH_HIP(hipStreamSynchronize(stream));
      rows_packed = true;
    }
    if (!sv_fused && (deps_direct || deps_rows)) {
      uint32_t bad = 0;
      FH_HIP(hipMemcpy(&bad, scal.get() + 1, sizeof(bad), hipMemcpyDeviceToHost));
      FH_CHECK(!(bad & 2), FH_EINVARIANT, "packed dependency rows: a log dot does not pack");
      FH_CHECK(bad == 0, FH_EINVARIANT, "a dot of the batch repeats a dot of an earlier batch");
    }
    if (dep_off || dep_out || dep_len) {
      uint32_t total = 0;
      FH_HIP(hipMemcpyAsync(&total, o_dep_off.get() + n, sizeof(total), hipMemcpyDeviceToHost,
                            stream));
      FH_HIP(hipStreamSynchronize(stream));
      if (dep_len) *dep_len = total;
      if (dep_out) FH_CHECK(dep_cap >= total, FH_ECAP, "dep output capacity too small");
      // (read back through pinned chunks, several host threads copying out:
      // hoststage.h)
      if (dep_off) ring.download(dep_off, o_dep_off.get(), size_t(n) + 1, stream);
      if (dep_out) ring.download(dep_out, o_dep.get(), size_t(total), stream);
    }
    if (scc_label) ring.download(scc_label, o_label, size_t(n), stream);
    if (exec_rank) ring.download(exec_rank, o_rank, size_t(n), stream);
    if (key_off) ring.download(key_off, key_offs.get(), size_t(key_space) + 1, stream);
    if (key_seq) ring.download(key_seq, o_seq, size_t(o_nelem), stream);
    FH_HIP(hipStreamSynchronize(stream));
  }
};

// ---- internal interface for fh_dgraph (engine_internal.h) ------------------
EngineDevice *engine_new(const fh_config &cfg) { return new EngineDevice(cfg); }
void engine_free(EngineDevice *e) { delete e; }
void engine_stage_subset(EngineDevice *e, const fh_stream_desc &d, const uint64_t *dot,
                         const uint64_t *key, const uint64_t *off, const uint32_t *ent) {
  // the range codes are log references relative to a command log that starts
  // at 0 (k_gather_codes): a re-stage starts a fresh log and fresh tables
  e->reset();
  e->stage_logs(d, 1, dot, key, off, ent, true);
}
const uint32_t *engine_run_codes(EngineDevice *e, float *ms) {
  FH_HIP(hipSetDevice(e->device));
  e->rewind();
  e->run(ms);
  return e->dep32.get();
}
hipStream_t engine_stream(EngineDevice *e) { return e->stream; }
void engine_set_profiling(EngineDevice *e, bool on) { e->profile = on; }
std::vector<std::pair<std::string, float>> engine_times(EngineDevice *e) { return e->last_times; }

void union_rows(uint32_t n, uint32_t S, const uint32_t *codes, const uint64_t *dot,
                uint32_t vbase, uint32_t *dcnt, uint32_t *dep_off, uint64_t *dep_dot,
                uint32_t *dst, uint32_t *ecnt, uint32_t *scal, ScanWorkspace &ws, hipStream_t s) {
  FH_CHECK(S <= kRegSlots, FH_ENOTIMPL, "range union: at most 16 slots per command");
  FH_HIP(hipMemsetAsync(scal, 0, 2 * sizeof(uint32_t), s));
  k_cmd_count<uint32_t><<<grid_for(n, B), B, 0, s>>>(n, S, codes, dot, 0, dcnt);
  exclusive_scan_u32(dcnt, dep_off, n, ws, s);
  const uint32_t g = S <= 4 ? (grid_for(n, B, 1u << 22) + 7) / 8 * 8 : grid_for(n, B);
  probed_launch("cmd_union", double(n) * (S * 4.0 + 8.0 * S + 4.0 * S + 4.0),
                k_cmd_engine<uint32_t>, dim3(g), dim3(B), s, n, S, dot, codes, dot,
                (const uint64_t *)nullptr, dep_dot, dcnt, dst, (uint8_t *)nullptr, scal, ecnt,
                uint64_t(0), (const uint32_t *)dep_off, scal + 1, vbase, 0u,
                (unsigned long long *)nullptr, (const uint32_t *)nullptr, 0);
}

}  // namespace fh

struct fh_engine {
  fh::EngineDevice dev;
  explicit fh_engine(const fh_config &c) : dev(c) {}
};

extern "C" {

fh_status fh_engine_create(const fh_config *cfg, fh_engine **out) {
  FH_API_BEGIN
  FH_CHECK(cfg && out, FH_EINVAL, "null argument");
  *out = new fh_engine(*cfg);
  FH_API_END
}

fh_status fh_engine_destroy(fh_engine *h) {
  FH_API_BEGIN
  delete h;
  FH_API_END
}

fh_status fh_engine_reset(fh_engine *h) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.reset();
  FH_API_END
}

fh_status fh_engine_stage(fh_engine *h, const fh_stream_desc *desc, const uint64_t *dot,
                          const uint64_t *key_id, const uint8_t *fq_proc, const uint64_t *fq_time) {
  FH_API_BEGIN
  FH_CHECK(h && desc, FH_EINVAL, "null argument");
  h->dev.stage(*desc, 1, dot, key_id, fq_proc, fq_time);
  FH_API_END
}

fh_status fh_engine_stage_many(fh_engine *h, const fh_stream_desc *desc, size_t nbatches,
                               const uint64_t *dot, const uint64_t *key_id,
                               const uint8_t *fq_proc, const uint64_t *fq_time) {
  FH_API_BEGIN
  FH_CHECK(h && desc, FH_EINVAL, "null argument");
  h->dev.stage(*desc, nbatches, dot, key_id, fq_proc, fq_time);
  FH_API_END
}

fh_status fh_engine_stage_logs(fh_engine *h, const fh_stream_desc *desc, size_t nbatches,
                               const uint64_t *dot, const uint64_t *key_id,
                               const uint64_t *log_off, const uint32_t *log_cmd) {
  FH_API_BEGIN
  FH_CHECK(h && desc, FH_EINVAL, "null argument");
  FH_CHECK(desc->views >= 1, FH_EINVAL, "stage_logs: views must be >= 1");
  h->dev.stage_logs(*desc, nbatches, dot, key_id, log_off, log_cmd);
  FH_API_END
}

fh_status fh_engine_rewind(fh_engine *h) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.rewind();
  FH_API_END
}

fh_status fh_engine_sync(fh_engine *h) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_HIP(hipSetDevice(h->dev.device));
  FH_HIP(hipStreamSynchronize(h->dev.stream));
  FH_API_END
}

fh_status fh_engine_run(fh_engine *h, float *device_ms) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.run(device_ms);
  FH_API_END
}

fh_status fh_engine_results(fh_engine *h, uint32_t *dep_off, uint64_t *dep_dot, size_t dep_cap,
                            size_t *dep_len, uint64_t *scc_label, uint32_t *exec_rank,
                            uint32_t *key_off, uint64_t *key_seq) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.results(dep_off, dep_dot, dep_cap, dep_len, scc_label, exec_rank, key_off, key_seq);
  FH_API_END
}

fh_status fh_engine_kernel_times(fh_engine *h, const char **names, float *ms, size_t cap,
                                 size_t *len) {
  FH_API_BEGIN
  FH_CHECK(h && len, FH_EINVAL, "null argument");
  const auto &t = h->dev.last_times;
  *len = t.size();
  for (size_t i = 0; i < t.size() && i < cap; i++) {
    if (names) names[i] = t[i].first.c_str();
    if (ms) ms[i] = t[i].second;
  }
  FH_API_END
}

fh_status fh_engine_set_probe(fh_engine *h, const char *kernel) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_HIP(hipStreamSynchronize(h->dev.stream));
  h->dev.probe.set(kernel ? kernel : "");
  FH_API_END
}

fh_status fh_engine_probe_stats_for(fh_engine *h, const char *kernel, float *avg_ms,
                                    size_t *launches, double *bytes_per_launch) {
  FH_API_BEGIN
  FH_CHECK(h && avg_ms && launches && bytes_per_launch, FH_EINVAL, "null argument");
  FH_HIP(hipStreamSynchronize(h->dev.stream));
  auto &pr = h->dev.probe;
  fh::ProbeSlot *p = kernel ? pr.find(kernel) : (pr.slots.empty() ? nullptr : &pr.slots[0]);
  FH_CHECK(p, FH_EINVAL, "kernel is not probed");
  const size_t n = p->next / 2;
  double tot = 0;
  for (size_t i = 0; i < n; i++) {
    float ms = 0;
    FH_HIP(hipEventElapsedTime(&ms, p->ev[2 * i], p->ev[2 * i + 1]));
    tot += ms;
  }
  *launches = n;
  *avg_ms = n ? float(tot / double(n)) : 0.f;
  *bytes_per_launch = n ? p->bytes / double(n) : 0.0;
  FH_API_END
}

fh_status fh_engine_probe_stats(fh_engine *h, float *avg_ms, size_t *launches,
                                double *bytes_per_launch) {
  return fh_engine_probe_stats_for(h, nullptr, avg_ms, launches, bytes_per_launch);
}

fh_status fh_engine_set_profiling(fh_engine *h, int on) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.profile = on != 0;
  FH_API_END
}

fh_status fh_engine_forget_tuning(fh_engine *h) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  FH_HIP(hipStreamSynchronize(h->dev.stream));
  h->dev.graph.forget_tuning();
  FH_API_END
}

fh_status fh_engine_set_deps_only(fh_engine *h, int on) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.deps_only = on != 0;
  FH_API_END
}

}  // extern "C"
