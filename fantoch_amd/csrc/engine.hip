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
#include <cstring>
#include <string>
#include <vector>

#include "graph_core.h"
#include "keybucket.h"

namespace fh {
namespace {

constexpr unsigned B = 256;
#define GRID_STRIDE(i, n) \
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += gridDim.x * blockDim.x)

// composite sort key for replica views: ((replica * K + key) << tb) | time
__global__ void k_view_keys(uint32_t M, uint32_t k, uint32_t fq, uint64_t K,
                            const uint32_t *__restrict__ key32, const uint8_t *__restrict__ fq_proc,
                            const uint64_t *__restrict__ fq_time, uint64_t tmin, int tb,
                            uint64_t *__restrict__ out) {
  GRID_STRIDE(e, M) {
    const uint32_t s = e % k;
    const uint32_t ij = e / k;  // i * fq + j
    const uint32_t i = ij / fq;
    const uint64_t seg = uint64_t(fq_proc[ij]) * K + key32[i * k + s];
    out[e] = (seg << tb) | (fq_time[ij] - tmin);
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
__device__ __forceinline__ bool dep_in_batch(uint64_t c, uint32_t *v) {
  if (c != 0 && c < kLogFlag) {
    *v = uint32_t(c - 1);
    return true;
  }
  return false;
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
__device__ __forceinline__ void cmd_union_regs(
    uint32_t i, uint32_t S, const uint64_t *__restrict__ dot,
    const uint64_t *__restrict__ dep_code, const uint64_t *__restrict__ dlog,
    const uint64_t *__restrict__ frontier, uint64_t *__restrict__ dep_dot,
    uint32_t *__restrict__ dep_cnt, uint32_t *__restrict__ dst, uint8_t *__restrict__ blocked0,
    uint32_t *nblocked, uint32_t *__restrict__ nv_out) {
  uint64_t r[kRegSlots];
  uint32_t vv[kRegSlots];
  bool missing = false;
#pragma unroll
  for (uint32_t t = 0; t < kRegSlots; t++) {
    r[t] = ~0ull;
    vv[t] = ~0u;
    if (t < S) {
      uint64_t x = dep_code[size_t(i) * S + t];
      uint32_t v;
      if (dep_in_batch(x, &v)) {
        vv[t] = v;
        r[t] = dot[v];
      } else {
        if (is_log_ref(x)) x = dlog[x - kLogFlag];  // single view: command-log reference
        if (x) {
          r[t] = x;
          if ((x & 0x00FFFFFFFFFFFFFFull) > frontier[x >> 56]) missing = true;
        }
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
  uint64_t *dd = dep_dot + size_t(i) * S;
  uint32_t m = 0;
  uint64_t prev = 0;  // dots are never 0
#pragma unroll
  for (uint32_t t = 0; t < kRegSlots; t++) {
    if (r[t] != ~0ull && r[t] != prev) {
      dd[m++] = r[t];
      prev = r[t];
    }
  }
  for (uint32_t q = m; q < S; q++) dd[q] = 0;
  uint32_t *ds = dst + size_t(i) * S;
  uint32_t nv = 0;
#pragma unroll
  for (uint32_t t = 0; t < kRegSlots; t++) {
    if (vv[t] != ~0u) {
      bool dup = false;
#pragma unroll
      for (uint32_t q = 0; q < t; q++) dup |= vv[q] == vv[t];
      if (!dup) ds[nv++] = vv[t];
    }
  }
  for (uint32_t q = nv; q < S; q++) ds[q] = i;  // padding: self loops are ignored
  if (nv_out) nv_out[i] = nv;
  dep_cnt[i] = m;
  if (blocked0) blocked0[i] = missing;
  if (missing) atomicAdd(nblocked, 1u);
}

// Per command: union of its fast-quorum members' element deps (vids and
// external dots), committed dep dots (sorted, fixed stride S), graph edges
// (vids, padded with the vertex itself), latest-table update at tails and the
// missing-dependency flag for external deps that are not executed.
__global__ void k_cmd_engine(uint32_t n, uint32_t S, const uint64_t *__restrict__ dot,
                             const uint64_t *__restrict__ dep_code,
                             const uint64_t *__restrict__ dlog,
                             const uint64_t *__restrict__ frontier,
                             uint64_t *__restrict__ dep_dot, uint32_t *__restrict__ dep_cnt,
                             uint32_t *__restrict__ dst, uint8_t *__restrict__ blocked0,
                             uint32_t *nblocked, uint32_t *__restrict__ nv_out) {
  if (S <= kRegSlots) {  // uniform: the register path
    GRID_STRIDE(i, n) {
      cmd_union_regs(i, S, dot, dep_code, dlog, frontier, dep_dot, dep_cnt, dst, blocked0,
                     nblocked, nv_out);
    }
    return;
  }
  GRID_STRIDE(i, n) {
    uint64_t *dd = dep_dot + size_t(i) * S;
    uint32_t *ds = dst + size_t(i) * S;
    uint32_t nv = 0, nd = 0;
    bool missing = false;
    for (uint32_t t = 0; t < S; t++) {
      uint64_t x = dep_code[size_t(i) * S + t];
      uint32_t v;
      if (dep_in_batch(x, &v)) {
        bool dup = false;
        for (uint32_t q = 0; q < nv; q++) dup |= ds[q] == v;
        if (!dup) ds[nv++] = v;
        dd[nd++] = dot[v];
      } else {
        if (is_log_ref(x)) x = dlog[x - kLogFlag];  // single view: command-log reference
        if (x) {
          dd[nd++] = x;
          // executed? (AEClock frontier; exceptions are not carried by the
          // fused engine: every earlier batch executed completely)
          if ((x & 0x00FFFFFFFFFFFFFFull) > frontier[x >> 56]) missing = true;
        }
      }
    }
    for (uint32_t q = nv; q < S; q++) ds[q] = i;  // padding: self loops are ignored
    if (nv_out) nv_out[i] = nv;
    const uint32_t m = S == 1 ? nd : sort_unique_u64(dd, nd);
    for (uint32_t q = m; q < S; q++) dd[q] = 0;
    dep_cnt[i] = m;
    if (blocked0) blocked0[i] = missing;
    if (missing) atomicAdd(nblocked, 1u);
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
__global__ void k_sv_unpermute(uint32_t M, const uint32_t *__restrict__ vs,
                               const uint64_t *__restrict__ dep_sorted,
                               const uint64_t *__restrict__ dot, const uint64_t *__restrict__ dlog,
                               uint64_t *__restrict__ dep_dot) {
  GRID_STRIDE(j, M) {
    const uint64_t x = dep_sorted[j];
    dep_dot[vs[j]] = is_log_ref(x) ? dlog[x - kLogFlag]  // an earlier batch
                     : (x != 0 && (x >> 56) == 0) ? dot[x - 1]  // in-batch index + 1
                     : x;
  }
}

__global__ void k_seq_dots(uint32_t m, const uint32_t *__restrict__ pk_vid,
                           const uint64_t *__restrict__ dot, uint64_t *__restrict__ seq) {
  GRID_STRIDE(j, m) seq[j] = dot[pk_vid[j]];
}

// executed-clock frontier advance for a fully executed batch: per-source
// min / max / count of the batch's sequences, reduced in LDS first
__global__ void __launch_bounds__(256)
    k_src_stats(uint32_t n, const uint64_t *__restrict__ dot, unsigned long long *__restrict__ mn,
                unsigned long long *__restrict__ mx, unsigned int *__restrict__ cnt) {
  __shared__ unsigned long long s_mn[256], s_mx[256];
  __shared__ unsigned int s_cnt[256];
  s_mn[threadIdx.x] = ~0ull;
  s_mx[threadIdx.x] = 0;
  s_cnt[threadIdx.x] = 0;
  __syncthreads();
  GRID_STRIDE(i, n) {
    const uint64_t d = dot[i];
    const uint32_t s = uint32_t(d >> 56);
    const unsigned long long q = d & 0x00FFFFFFFFFFFFFFull;
    atomicMin(&s_mn[s], q);
    atomicMax(&s_mx[s], q);
    atomicAdd(&s_cnt[s], 1u);
  }
  __syncthreads();
  const uint32_t s = threadIdx.x;
  if (s_cnt[s]) {
    atomicMin(&mn[s], s_mn[s]);
    atomicMax(&mx[s], s_mx[s]);
    atomicAdd(&cnt[s], s_cnt[s]);
  }
}

__global__ void k_frontier_update(const unsigned long long *__restrict__ mn,
                                  const unsigned long long *__restrict__ mx,
                                  const unsigned int *__restrict__ cnt, uint64_t *frontier,
                                  unsigned long long *excount, uint32_t *err) {
  const uint32_t s = threadIdx.x;
  if (s >= 256 || cnt[s] == 0) return;
  if (mn[s] == frontier[s] + 1 && mx[s] - mn[s] + 1 == cnt[s]) {
    frontier[s] = mx[s];
    excount[s] += cnt[s];
  } else {
    atomicOr(err, 1u);  // non-contiguous executed set: needs exceptions
  }
}

// per-key sequence in key-grouped (not key-ascending) order -> ascending
// layout: the first position of each key's run, then every element moves to
// off[key] + (its position - the run's first position)
__global__ void k_run_heads(uint32_t m, const uint32_t *__restrict__ keys, uint32_t *__restrict__ hp) {
  GRID_STRIDE(j, m) if (j == 0 || keys[j - 1] != keys[j]) hp[keys[j]] = j;
}

__global__ void k_run_scatter(uint32_t m, const uint32_t *__restrict__ keys,
                              const uint32_t *__restrict__ vids, const uint32_t *__restrict__ hp,
                              const uint32_t *__restrict__ off, const uint64_t *__restrict__ dot,
                              uint64_t *__restrict__ out) {
  GRID_STRIDE(j, m) {
    const uint32_t k = keys[j];
    out[off[k] + (j - hp[k])] = dot[vids[j]];
  }
}

__global__ void k_cnt_nonzero(uint32_t n, const uint64_t *__restrict__ d, uint32_t *__restrict__ c) {
  GRID_STRIDE(i, n) c[i] = d[i] != 0;
}

__global__ void k_bcast_u32(uint32_t n, uint32_t *p, uint32_t v) { GRID_STRIDE(i, n) p[i] = v; }

__global__ void k_identity_labels(uint32_t n, const uint64_t *__restrict__ dot,
                                  uint64_t *__restrict__ lab, uint32_t *__restrict__ rank) {
  GRID_STRIDE(i, n) {
    lab[i] = dot[i];
    rank[i] = i;
  }
}

// Key histogram of the per-key sequence.  Its keys come in runs (each key's
// elements are contiguous), so one atomic per run within a wave: the run's
// head lane adds the run length (C3's 20M elements on 17 keys took 125 ms
// with one atomic per element).
__global__ void k_key_hist(uint32_t m, const uint32_t *__restrict__ keys, uint32_t *__restrict__ h) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t b = blockIdx.x * blockDim.x; b < m; b += gridDim.x * blockDim.x) {
    const uint32_t j = b + threadIdx.x;
    const bool valid = j < m;
    const uint32_t k = valid ? keys[j] : ~0u;
    const uint32_t kp = __shfl_up(k, 1, 64);
    const bool head = valid && (lane == 0 || kp != k);
    const uint64_t heads = __ballot(head);
    const uint64_t vmask = __ballot(valid);
    if (head) {
      const uint64_t later = lane == 63 ? 0ull : heads >> (lane + 1);
      const uint32_t nvalid = uint32_t(__popcll(vmask));  // valid lanes are a prefix
      const uint32_t end = later ? lane + 1 + uint32_t(__ffsll((long long)later) - 1) : nvalid;
      atomicAdd(&h[k], end - lane);
    }
  }
}

// fixed-stride in-batch edges (S slots, the first cnt[i] real) -> CSR: the
// graph's fixpoint passes then read only real edges (C5: 6.3 of 12 slots)
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
  DBuf<uint32_t> key_hist, key_offs, headpos;
  // persistent state
  DBuf<uint64_t> latest;     // [(nproc+1) * K]
  DBuf<uint64_t> frontier;   // [256] executed-clock frontier per source
  uint32_t latest_slots = 1; // replica slots allocated in `latest`
  DBuf<uint32_t> err;
  // staged batches
  fh_stream_desc desc{};
  bool staged = false;
  size_t nbatches = 0, cursor = 0, last = 0;
  std::vector<uint64_t> tmins;
  uint64_t tmin = 0;
  int tbits = 0;
  DBuf<uint64_t> dot, fq_time;  // dot: the command log (every staged batch, appended)
  size_t log_len = 0;            // dots in the log
  size_t stage_base = 0;         // log position of the first staged batch
  DBuf<uint32_t> key32;
  DBuf<uint8_t> fq_proc;
  // scratch / outputs
  DBuf<uint64_t> vkeys, sk64a, sk64b, dep_ext, dep_dot, seq_dot, lab;
  DBuf<uint32_t> sk32a, sk32b, sva, svb, dep_cnt, dst, sorted_vid, rank_tmp, u32tmp;
  DBuf<uint32_t> edge_cnt, edge_off, edge_csr;  // replica views: in-batch edges as CSR
  DBuf<uint8_t> blocked0;
  DBuf<uint32_t> scal;
  DBuf<unsigned long long> srcstats;
  SortWorkspace sort_ws;
  ScanWorkspace scan_ws;
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
    FH_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    FH_HIP(hipEventCreate(&ev0));
    FH_HIP(hipEventCreate(&ev1));

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
    staged = false;
  }

  void stage(const fh_stream_desc &d, size_t nb, const uint64_t *h_dot, const uint64_t *h_key,
             const uint8_t *h_proc, const uint64_t *h_time) {
    FH_CHECK(h_dot && h_key && nb >= 1, FH_EINVAL, "null argument");
    FH_CHECK(d.keys_per_cmd >= 1 && d.keys_per_cmd <= 8, FH_EINVAL, "keys_per_cmd in [1, 8]");
    const uint32_t fq = d.views ? d.views : 1;
    FH_CHECK(fq <= 16, FH_EINVAL, "views <= 16");
    FH_CHECK(size_t(d.n) * fq * d.keys_per_cmd < (size_t(1) << 30), FH_EINVAL,
             "batch too large (elements >= 2^30)");
    FH_CHECK(!d.views || (h_proc && h_time && d.nproc >= 1 && d.nproc <= 255), FH_EINVAL,
             "replica views need fq_proc, fq_time and nproc");
    FH_HIP(hipSetDevice(device));
    sync_all();
    const size_t n = d.n, nk = n * d.keys_per_cmd;
    std::vector<uint32_t> k32(nk * nb);
    for (size_t e = 0; e < nk * nb; e++) {
      FH_CHECK(h_key[e] < key_space, FH_EINVAL, "stage: key id >= key_space");
      k32[e] = uint32_t(h_key[e]);
    }
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
    FH_HIP(hipMemcpyAsync(dot.get() + log_len, h_dot, n * nb * sizeof(uint64_t),
                          hipMemcpyHostToDevice, stream));
    stage_base = log_len;
    log_len += n * nb;
    FH_HIP(hipMemcpyAsync(key32.ensure(nk * nb + 1), k32.data(), nk * nb * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    tmins.assign(nb, 0);
    tbits = 0;
    if (d.views) {
      const size_t nv = n * fq;
      for (size_t b = 0; b < nb; b++) {
        uint64_t lo = ~0ull, hi = 0;
        for (size_t i = b * nv; i < (b + 1) * nv; i++) {
          FH_CHECK(h_proc[i] >= 1 && h_proc[i] <= d.nproc, FH_EINVAL, "fq_proc out of range");
          lo = std::min(lo, h_time[i]);
          hi = std::max(hi, h_time[i]);
        }
        tmins[b] = n ? lo : 0;
        tbits = std::max(tbits, bits_for(n ? hi - lo + 1 : 1));
      }
      FH_CHECK(bits_for(uint64_t(d.nproc + 1) * key_space) + tbits <= 64, FH_ENOTIMPL,
               "replica-view sort key wider than 64 bits");
      FH_HIP(hipMemcpyAsync(fq_proc.ensure(nv * nb + 1), h_proc, nv * nb, hipMemcpyHostToDevice,
                            stream));
      FH_HIP(hipMemcpyAsync(fq_time.ensure(nv * nb + 1), h_time, nv * nb * sizeof(uint64_t),
                            hipMemcpyHostToDevice, stream));
      ensure_latest(d.nproc + 1);
    }
    FH_HIP(hipStreamSynchronize(stream));
    desc = d;
    nbatches = nb;
    cursor = 0;
    staged = true;
  }

  // The device run of one batch: everything below is the timed hot path.
  void run(float *ms) {
    FH_CHECK(staged && cursor < nbatches, FH_EINVAL, "no staged batch left to run");
    FH_HIP(hipSetDevice(device));
    clear_marks();
    graph.profile = profile;
    const uint32_t n = uint32_t(desc.n), k = desc.keys_per_cmd;
    const uint32_t fq = desc.views ? desc.views : 1;
    const uint32_t S = fq * k;
    const uint32_t M = n * S;
    const bool views = desc.views != 0;
    const size_t b = cursor++;
    last = b;
    const uint64_t bbase = stage_base + b * n;  // log position of this batch
    const uint64_t *bdot = dot.get() + bbase;
    const uint32_t *bkey = key32.get() + b * size_t(n) * k;
    const uint8_t *bproc = views ? fq_proc.get() + b * size_t(n) * fq : nullptr;
    const uint64_t *btime = views ? fq_time.get() + b * size_t(n) * fq : nullptr;
    tmin = tmins[b];
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
        vs = sva.ensure(M + 1);
        // one launch per step: order this batch (partitioned by the previous
        // step, or now) and partition the next staged batch in the same grid
        const size_t q = b & 1;
        const KeyBucketClock clock = kb_clock(b);
        if (kb_next_part != b)
          keybucket_partition(plan, M, bkey, bdot, clock.fold, kb_ws[q], stream, &kb_sched);
        kb_next_part = ~size_t(0);
        if (b + 1 < nbatches) {
          keybucket_step(plan, M, bbase, latest.get(), kb_ws[q], ks, vs, dsorted, clock, plan, M,
                         bkey + M, bdot + M, kb_clock(b + 1).fold, kb_ws[q ^ 1], stream,
                         &kb_sched);
          kb_next_part = b + 1;
        } else {
          keybucket_order(plan, M, bbase, latest.get(), kb_ws[q], ks, vs, dsorted, clock, stream,
                          &kb_sched);
        }
        // refresh the schedule from the sizes just recorded: after the first
        // launch, then every 32 (the key distribution drifts slowly)
        if ((kb_launches++ & 31) == 0) keybucket_sched(kb_sched, stream);
        mark("keydeps_bucket");
        bucket_order = true;
      } else {
        sort_pairs<uint32_t>(bkey, nullptr, sk32a.ensure(M + 1), sva.ensure(M + 1),
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
      sort_pairs<uint32_t>(bkey, nullptr, sk32a.ensure(M + 1), sva.ensure(M + 1),
                           sk32b.ensure(M + 1), svb.ensure(M + 1), M, key_bits, sort_ws, stream,
                           &ks, &vs);
      mark("keydeps_sort");
      k_prev_engine<uint32_t><<<grid_for(M, B), B, 0, stream>>>(
          M, ks, vs, 0, S, latest.get(), uint64_t(lmul), uint64_t(lmask), dext,
          k == 1 ? nullptr : svid);
      k_tail_engine<uint32_t><<<grid_for(M, B), B, 0, stream>>>(
          M, ks, vs, 0, S, latest.get(), uint64_t(lmul), uint64_t(lmask), nullptr, bbase);
      sorted_keys32 = ks;
    } else {
      sv_fused = false;
      uint64_t *vk = vkeys.ensure(M + 1);
      k_view_keys<<<grid_for(M, B), B, 0, stream>>>(M, k, fq, key_space, bkey, bproc, btime, tmin,
                                                     tbits, vk);
      uint64_t *ks = nullptr;
      const int bits = bits_for(uint64_t(desc.nproc + 1) * key_space) + tbits;
      sort_pairs<uint64_t>(vk, nullptr, sk64a.ensure(M + 1), sva.ensure(M + 1),
                           sk64b.ensure(M + 1), svb.ensure(M + 1), M, bits, sort_ws, stream, &ks,
                           &vs);
      mark("keydeps_sort");
      k_prev_engine<uint64_t><<<grid_for(M, B), B, 0, stream>>>(
          M, ks, vs, tbits, S, views_latest(), 1ull, ~0ull, dext, nullptr);
      k_tail_engine<uint64_t><<<grid_for(M, B), B, 0, stream>>>(
          M, ks, vs, tbits, S, views_latest(), 1ull, ~0ull, bdot, 0);
    }
    if (!sv_fused) run_general(n, k, fq, S, M, views, bkey, bproc, bdot, bbase);
    if (ms || profile) FH_HIP(hipEventRecord(ev1, stream));
    if (ms) {
      FH_HIP(hipEventSynchronize(ev1));
      FH_HIP(hipEventElapsedTime(ms, ev0, ev1));
    }
    if (profile) collect_times();
  }

  void run_general(uint32_t n, uint32_t k, uint32_t fq, uint32_t S, uint32_t M, bool views,
                   const uint32_t *bkey, const uint8_t *bproc, const uint64_t *bdot,
                   uint64_t bbase) {
    const uint64_t *dcode = dep_ext.get();
    uint32_t *svid = sorted_vid.get();
    mark("keydeps_prev");
    uint64_t *ddot = dep_dot.ensure(M + 1);
    uint32_t *dcnt = dep_cnt.ensure(n + 1);
    uint32_t *dd = dst.ensure(M + 1);
    FH_HIP(hipMemsetAsync(scal.get(), 0, sizeof(uint32_t), stream));
    k_cmd_engine<<<grid_for(n, B), B, 0, stream>>>(
        n, S, bdot, dcode, (const uint64_t *)dot.get(), frontier.get(), ddot, dcnt, dd, nullptr,
        scal.get(), views && S >= 8 ? edge_cnt.ensure(n + 1) : nullptr);
    mark("keydeps_union");
    const uint32_t *gdst = dd, *goff = nullptr;
    if (views && S >= 8) {  // measured: a win at S = 12 (C5), flat or worse at 3 and 6
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
    gin.dot = bdot;
    gin.k = k;
    gin.key32 = bkey;
    gin.key_bits = key_bits;
    if (!views) {
      gin.no_forward_hint = true;  // single view: deps always point backwards
      gin.sorted_keys = sorted_keys32;
      gin.sorted_vid = svid;
    }
    graph.run(gin, gout);
    FH_CHECK(gout.npending == 0, FH_EINVARIANT, "fused engine batch left pending vertices");
    // per-key sequence of dots (ExecutionOrderMonitor::add order)
    uint64_t *sq = seq_dot.ensure(gout.nelem + 1);
    k_seq_dots<<<grid_for(gout.nelem, B), B, 0, stream>>>(gout.nelem, gout.pk_vid, bdot, sq);
    mark("per_key_dots");
    // executed clock: the whole batch executed
    unsigned long long *st = srcstats.ensure(4 * 256);
    FH_HIP(hipMemsetAsync(st, 0xFF, 256 * sizeof(unsigned long long), stream));
    FH_HIP(hipMemsetAsync(st + 256, 0, 512 * sizeof(unsigned long long), stream));
    k_src_stats<<<grid_for(n, B, 512), B, 0, stream>>>(n, bdot, st, st + 256,
                                                   reinterpret_cast<unsigned int *>(st + 512));
    k_frontier_update<<<1, 256, 0, stream>>>(st, st + 256,
                                             reinterpret_cast<unsigned int *>(st + 512),
                                             frontier.get(), excount_ptr(), err.get());
    mark("executed_clock");
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

  void check_err() {
    uint32_t e = 0;
    FH_HIP(hipMemcpyAsync(&e, err.get(), sizeof(e), hipMemcpyDeviceToHost, stream));
    if (excount.get()) {
      uint64_t f[256], c[256];
      FH_HIP(hipMemcpyAsync(f, frontier.get(), sizeof(f), hipMemcpyDeviceToHost, stream));
      FH_HIP(hipMemcpyAsync(c, excount.get(), sizeof(c), hipMemcpyDeviceToHost, stream));
      FH_HIP(hipStreamSynchronize(stream));
      for (int s = 0; s < 256; s++)
        if (c[s] != f[s]) e = 1;  // executed set not contiguous from 1
    }
    FH_HIP(hipStreamSynchronize(stream));
    FH_CHECK(e == 0, FH_ENOTIMPL,
             "executed clock: non-contiguous executed dots per process (exceptions not supported "
             "by the fused engine)");
  }

  void results(uint32_t *dep_off, uint64_t *dep_out, size_t dep_cap, size_t *dep_len,
               uint64_t *scc_label, uint32_t *exec_rank, uint32_t *key_off, uint64_t *key_seq) {
    FH_HIP(hipSetDevice(device));
    FH_HIP(hipStreamSynchronize(stream));
    check_err();
    const uint32_t n = uint32_t(desc.n), k = desc.keys_per_cmd;
    const uint32_t S = (desc.views ? desc.views : 1) * k;
    if (dep_off || dep_out || dep_len) {
      uint32_t *off = u32tmp.ensure(n + 1);
      if (sv_fused) {  // one dependency slot per command: decode, count = slot used
        k_sv_unpermute<<<grid_for(n, B), B, 0, stream>>>(n, sv_vs, dep_ext.get(),
                                                          dot.get() + stage_base + last * n,
                                                          dot.get(), dep_dot.ensure(n + 1));
        k_cnt_nonzero<<<grid_for(n, B), B, 0, stream>>>(n, dep_dot.get(), dep_cnt.ensure(n + 1));
      }
      exclusive_scan_u32(dep_cnt.get(), off, n, scan_ws, stream);
      uint32_t total = 0;
      FH_HIP(hipMemcpyAsync(&total, off + n, sizeof(total), hipMemcpyDeviceToHost, stream));
      FH_HIP(hipStreamSynchronize(stream));
      if (dep_len) *dep_len = total;
      if (dep_off)
        FH_HIP(hipMemcpyAsync(dep_off, off, (n + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                              stream));
      if (dep_out) {
        FH_CHECK(dep_cap >= total, FH_ECAP, "dep output capacity too small");
        uint64_t *c = sk64a.ensure(total + 1);
        k_compact_deps<<<grid_for(n, B), B, 0, stream>>>(n, S, dep_dot.get(), off, c);
        FH_HIP(hipMemcpyAsync(dep_out, c, size_t(total) * sizeof(uint64_t),
                              hipMemcpyDeviceToHost, stream));
      }
    }
    if (scc_label || exec_rank) {
      uint64_t *lb = gout.scc_label;
      uint32_t *rk = gout.exec_rank;
      if (gout.trivial) {
        lb = lab.ensure(n + 1);
        rk = rank_tmp.ensure(n + 1);
        k_identity_labels<<<grid_for(n, B), B, 0, stream>>>(n, dot.get() + stage_base + last * n, lb, rk);
      }
      if (scc_label)
        FH_HIP(hipMemcpyAsync(scc_label, lb, size_t(n) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                              stream));
      if (exec_rank)
        FH_HIP(hipMemcpyAsync(exec_rank, rk, size_t(n) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                              stream));
    }
    if (key_off || key_seq) {
      // per-key offsets over the ascending key space (histogram + scan)
      uint32_t *h = key_hist.ensure(key_space + 1);
      uint32_t *o = key_offs.ensure(key_space + 2);
      FH_HIP(hipMemsetAsync(h, 0, key_space * sizeof(uint32_t), stream));
      k_key_hist<<<grid_for(gout.nelem, B), B, 0, stream>>>(gout.nelem, gout.pk_key, h);
      exclusive_scan_u32(h, o, key_space, scan_ws, stream);
      if (key_off)
        FH_HIP(hipMemcpyAsync(key_off, o, (key_space + 1) * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, stream));
      if (key_seq) {
        uint64_t *sq = seq_dot.ensure(gout.nelem + 1);
        const uint64_t *bd = dot.get() + stage_base + last * n;
        if (sv_fused && bucket_order) {
          // key-grouped runs -> ascending keys
          uint32_t *hp = headpos.ensure(key_space + 1);
          k_run_heads<<<grid_for(gout.nelem, B), B, 0, stream>>>(gout.nelem, gout.pk_key, hp);
          k_run_scatter<<<grid_for(gout.nelem, B), B, 0, stream>>>(gout.nelem, gout.pk_key,
                                                                    gout.pk_vid, hp, o, bd, sq);
        } else if (sv_fused) {  // (sorted keys, sorted vids): gather the dots
          k_seq_dots<<<grid_for(gout.nelem, B), B, 0, stream>>>(gout.nelem, gout.pk_vid, bd, sq);
        }
        FH_HIP(hipMemcpyAsync(key_seq, sq, size_t(gout.nelem) * sizeof(uint64_t),
                              hipMemcpyDeviceToHost, stream));
      }
    }
    FH_HIP(hipStreamSynchronize(stream));
  }
};

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

}  // extern "C"
