// graph_small.hip -- one executor pass of a small graph in one workgroup
// (fh_graph streaming at small batches: SURVEY §8f rank 1).
//
// GraphExecutor::handle(Add) runs per command inside the simulator and the
// runner (fantoch/src/sim/runner.rs:407-413, run/task/executor.rs:150-175),
// so a drop-in must take batches of one.  The general pass (graph_api.hip:
// dot sort, resolve, GraphCore's fixpoints, compaction) is a few dozen
// launches with several host round trips; for V <= kSmallV vertices and
// E <= kSmallE dependency entries everything happens here, in LDS, in one
// launch, reading the batch from and writing its results to mapped pinned
// host memory:
//  0. the batch's rows appended after the carried prefix (read over PCIe
//     from the mapped upload block, every load of a thread issued before its
//     first store), and the executed-clock mirror when it changed;
//  1. the dot -> vid index: an LDS hash table (duplicate check,
//     mod.rs:235-240);
//  2. dependencies resolved once, a thread per entry: self and executed ones
//     ignored (tarjan.rs:131-148), others are vertices or missing (the
//     vertex is blocked, tarjan.rs:150-170); missing dots listed;
//  3. blocked closure: a vertex reaching a missing dependency stays pending
//     (check_pending, mod.rs:558-644);
//  4. the rest as GraphCore orders it (graph_core.h): H = max vid reachable
//     (pointer jumping), SCCs by rounds of reach from each ready group's root
//     (an SCC's representative is its minimum vid), depth over same-H edges,
//     labels = min dot;
//  5. execution order by (H, depth, representative, dot): a counting sort by
//     H, then each vertex's rank inside its group;
//  6. the survivors compacted, in arrival order, into the next vertex set.
#include "graph_small.h"

#include "dotindex.h"

namespace fh {
namespace {

constexpr int kThreads = 1024;
constexpr uint16_t kNone = 0xFFFF;

// exclusive scan of one value per thread over the block
__device__ uint32_t block_scan(uint32_t v, uint32_t *s_w, uint32_t *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kThreads / 64; i++) {
    const uint32_t c = s_w[i];
    if (i < w) pre += c;
    tot += c;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// dot -> vid hash index in LDS: 2 * kSmallV slots, linear probing; the
// all-ones dot is reserved (the empty slot), as everywhere in the library
constexpr int kHash = 2 * kSmallV;
constexpr uint64_t kEmpty = ~0ull;
constexpr int kSmallExc = 1024;  // executed-clock exceptions staged in LDS
__device__ __forceinline__ uint32_t hash_slot(uint64_t d) {
  return uint32_t((d * 0x9E3779B97F4A7C15ull) >> 52) & (kHash - 1);
}
__device__ __forceinline__ int find_hash(const uint64_t *hk, const uint16_t *hv, uint64_t d) {
  for (uint32_t h = hash_slot(d);; h = (h + 1) & (kHash - 1)) {
    const uint64_t k = hk[h];
    if (k == d) return hv[h];
    if (k == kEmpty) return -1;
  }
}

// sweep to the fixpoint: body(x) returns true on a change
template <class F>
__device__ void sweep(int n, uint32_t *s_ch, F body) {
  for (int it = 0;; it++) {
    bool ch = false;
    for (int x = threadIdx.x; x < n; x += kThreads) ch |= body(x);
    if (ch) s_ch[it % 3] = 1;
    if (threadIdx.x == 0) s_ch[(it + 1) % 3] = 0;
    __syncthreads();
    if (!s_ch[it % 3]) break;
  }
  __syncthreads();
  if (threadIdx.x < 3) s_ch[threadIdx.x] = 0;
  __syncthreads();
}

__global__ void __launch_bounds__(kThreads)
    k_graph_small(SmallPass p) {
  // phase stamps (FH_GRAPH_DEBUG): wall clock (100 MHz) at 10 points into
  // header[8 + 2i] (host prints the phase times)
  auto stamp = [&](int i) {
    if (p.stamps && threadIdx.x == 0) {
      const uint64_t t = wall_clock64();
      p.header[8 + 2 * i] = uint32_t(t);
      p.header[9 + 2 * i] = uint32_t(t >> 32);
    }
  };
  stamp(0);
  if (p.delay_us) {  // fault injection: a pass that takes delay_us longer
    if (threadIdx.x == 0) {
      const uint64_t t0 = wall_clock64(), t1 = t0 + uint64_t(p.delay_us) * 100;  // 100 MHz
      while (wall_clock64() < t1) __builtin_amdgcn_s_sleep(127);
    }
    __syncthreads();
  }
  // the batch's rows after the carried prefix, and the clock mirror
  // (k_append's job on the general path); the pass below reads them back
  // from global memory after the barrier
  {
    // four items per thread per round, every load issued before a store: one
    // PCIe round trip per 4096 items instead of one per 1024
    const uint32_t m = append_items(p.up);
    for (uint32_t i0 = 0; i0 < m; i0 += 4 * kThreads) {
      AppendVals av[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t i = i0 + uint32_t(k) * kThreads + threadIdx.x;
        if (i < m) append_load(p.up, i, av[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t i = i0 + uint32_t(k) * kThreads + threadIdx.x;
        if (i < m) append_store(p.up, p.dst, i, av[k]);
      }
    }
  }
  __syncthreads();
  stamp(9);
  __shared__ uint64_t s_dot[kSmallV], s_key[kSmallV];
  // dot -> vid hash index (open addressing, load <= 1/2); after the resolve
  // its key words are scratch for the order's group counts
  __shared__ uint64_t s_hk[kHash];
  __shared__ uint16_t s_hv[kHash];
  __shared__ uint16_t s_off[kSmallV + 1], s_dst[kSmallE], s_tgt[kSmallE];
  __shared__ uint64_t s_front[256];  // executed clock frontier (AEClock)
  // its exceptions, staged when they fit: the resolve's binary search per
  // dependency then runs in LDS instead of ~8 dependent global loads
  __shared__ uint64_t s_exc[kSmallExc];
  __shared__ uint16_t s_H[kSmallV], s_R[kSmallV], s_W[kSmallV], s_min[kSmallV];
  __shared__ uint32_t s_D[kSmallV];
  __shared__ uint8_t s_blk[kSmallV], s_F[kSmallV];
  __shared__ uint32_t s_w[kThreads / 64], s_ch[3], s_nmiss, s_err;
  const int tid = threadIdx.x, V = int(p.V);
  if (tid < 3) s_ch[tid] = 0;
  if (tid == 0) s_nmiss = s_err = 0;
  if (tid < 256) s_front[tid] = p.frontier[tid];
  for (int x = tid; x < kHash; x += kThreads) s_hk[x] = kEmpty;
  for (int x = tid; x < V; x += kThreads) s_dot[x] = p.dot[x];
  const bool exc_lds = p.nexc <= uint32_t(kSmallExc);
  if (exc_lds)
    for (uint32_t x = tid; x < p.nexc; x += kThreads) s_exc[x] = p.exc[x];
  const uint64_t *exc = exc_lds ? s_exc : p.exc;
  __syncthreads();
  // 1. dot -> vid index; a dot indexed twice (mod.rs:235-240)
  for (int x = tid; x < V; x += kThreads) {
    const uint64_t d = s_dot[x];
    for (uint32_t h = hash_slot(d);; h = (h + 1) & (kHash - 1)) {
      const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long *>(&s_hk[h]),
                                      (unsigned long long)kEmpty, (unsigned long long)d);
      if (prev == kEmpty) {
        s_hv[h] = uint16_t(x);
        break;
      }
      if (prev == d) {
        s_err = 1;
        break;
      }
    }
  }
  __syncthreads();
  stamp(1);
  // 2. resolve: one pass over the dependency entries, a thread per entry
  // (coalesced loads, no per-vertex chains of dependent global loads),
  // writes each entry's target vid into LDS at its list position: kNone for
  // executed, kMiss for missing; an entry naming its own vertex is dropped
  // by the per-vertex pass below (its own dot is always a vertex)
  constexpr uint16_t kMiss = 0xFFFE;
  const uint32_t e0 = p.doff[0], DT = p.doff[V] - e0;
  for (uint32_t e = tid; e < DT; e += kThreads) {
    const uint64_t d = p.ddot[e0 + e];
    uint16_t t = kNone;
    if (!executed_dev(d, s_front, exc, p.nexc)) {
      const int u = find_hash(s_hk, s_hv, d);
      if (u >= 0) {
        t = uint16_t(u);
      } else {
        t = kMiss;
        const uint32_t q = atomicAdd(&s_nmiss, 1u);
        if (q < p.miss_cap) p.miss[q] = d;
      }
    }
    s_tgt[e] = t;
  }
  __syncthreads();
  uint32_t cnt[2] = {0, 0};
  for (int j = 0; j < 2; j++) {
    const int v = 2 * tid + j;  // a thread's vertices are adjacent: scans follow vid order
    if (v >= V) continue;
    bool missing = false;
    const uint32_t eb = p.doff[v] - e0, ee = p.doff[v + 1] - e0;
    for (uint32_t e = eb; e < ee; e++) {
      const uint16_t t = s_tgt[e];
      if (t == uint16_t(v)) {
        s_tgt[e] = kNone;  // self (graph/mod.rs skips the vertex's own dot)
      } else if (t == kMiss) {
        missing = true;
      } else if (t != kNone) {
        cnt[j]++;
      }
    }
    s_blk[v] = missing;
  }
  uint32_t etot = 0;
  const uint32_t o0 = block_scan(cnt[0] + cnt[1], s_w, &etot);
  {
    uint32_t o = o0;
    for (int j = 0; j < 2; j++) {
      const int v = 2 * tid + j;
      if (v >= V) continue;
      s_off[v] = uint16_t(o);
      const uint32_t eb = p.doff[v] - e0, ee = p.doff[v + 1] - e0;
      for (uint32_t e = eb; e < ee; e++) {
        const uint16_t t = s_tgt[e];
        if (t < kMiss) s_dst[o++] = t;
      }
    }
    if (tid == 0) s_off[V] = uint16_t(etot);
  }
  __syncthreads();
  stamp(2);
  // 3. blocked closure
  sweep(V, s_ch, [&](int v) {
    if (s_blk[v]) return false;
    for (int e = s_off[v]; e < s_off[v + 1]; e++)
      if (s_blk[s_dst[e]]) {
        s_blk[v] = 1;
        return true;
      }
    return false;
  });
  stamp(3);
  // 4. H = max vid reachable (executable vertices reach only executable ones)
  for (int v = tid; v < V; v += kThreads) {
    s_H[v] = uint16_t(v);
    s_R[v] = kNone;
    s_F[v] = 0;
  }
  __syncthreads();
  sweep(V, s_ch, [&](int v) {
    if (s_blk[v]) return false;
    uint32_t h = s_H[v];
    const uint32_t h0 = h;
    for (int e = s_off[v]; e < s_off[v + 1]; e++) h = max(h, uint32_t(s_H[s_dst[e]]));
    h = max(h, uint32_t(s_H[h]));
    if (h > h0) {
      s_H[v] = uint16_t(h);
      return true;
    }
    return false;
  });
  stamp(4);
  // SCC rounds over the unassigned vertices: W = max unassigned vid reachable
  // through unassigned vertices; roots (W(v) = v) reach their class members
  for (int round = 0;; round++) {
    uint32_t left = 0;
    {
      uint32_t mine = 0;
      for (int v = tid; v < V; v += kThreads)
        if (!s_blk[v] && s_R[v] == kNone) {
          mine++;
          s_W[v] = uint16_t(v);
          s_F[v] = 0;
        }
      block_scan(mine, s_w, &left);
    }
    if (!left) break;
    // round 0: nothing is assigned yet, so W over the unassigned vertices is
    // H itself
    if (round == 0) {
      for (int v = tid; v < V; v += kThreads)
        if (!s_blk[v]) s_W[v] = s_H[v];
      __syncthreads();
    } else
    sweep(V, s_ch, [&](int v) {
      if (s_blk[v] || s_R[v] != kNone) return false;
      uint32_t h = s_W[v];
      const uint32_t h0 = h;
      for (int e = s_off[v]; e < s_off[v + 1]; e++) {
        const uint16_t y = s_dst[e];
        if (s_R[y] == kNone) h = max(h, uint32_t(s_W[y]));
      }
      h = max(h, uint32_t(s_W[h]));
      if (h > h0) {
        s_W[v] = uint16_t(h);
        return true;
      }
      return false;
    });
    for (int v = tid; v < V; v += kThreads)
      if (!s_blk[v] && s_R[v] == kNone && s_W[v] == v) s_F[v] = 1;
    __syncthreads();
    sweep(V, s_ch, [&](int v) {
      if (s_F[v] != 1) return false;
      s_F[v] = 2;
      const uint16_t g = s_W[v];
      for (int e = s_off[v]; e < s_off[v + 1]; e++) {
        const uint16_t y = s_dst[e];
        if (s_R[y] == kNone && s_F[y] == 0 && s_W[y] == g) s_F[y] = 1;
      }
      return true;
    });
    for (int v = tid; v < V; v += kThreads)
      if (!s_blk[v] && s_R[v] == kNone && s_F[v]) s_R[v] = s_W[v];
    __syncthreads();
  }
  stamp(5);
  // representative = min member; labels = min dot; depth over same-H edges
  for (int v = tid; v < V; v += kThreads) {
    s_min[v] = kNone;
    s_D[v] = 0;
    s_key[v] = ~0ull;  // per representative: min dot (label)
  }
  __syncthreads();
  for (int v = tid; v < V; v += kThreads)
    if (!s_blk[v]) {
      // 16-bit min through the 32-bit word: s_min is reread after the barrier
      uint32_t *w = reinterpret_cast<uint32_t *>(reinterpret_cast<uintptr_t>(&s_min[s_R[v]]) & ~uintptr_t(3));
      const int sh = int(reinterpret_cast<uintptr_t>(&s_min[s_R[v]]) & 2) * 8;
      uint32_t old = *w;
      for (;;) {
        if (uint16_t(old >> sh) <= uint16_t(v)) break;
        const uint32_t nw = (old & ~(0xFFFFu << sh)) | (uint32_t(v) << sh);
        const uint32_t prev = atomicCAS(w, old, nw);
        if (prev == old) break;
        old = prev;
      }
    }
  __syncthreads();
  for (int v = tid; v < V; v += kThreads)
    if (!s_blk[v]) {
      s_R[v] = s_min[s_R[v]];
      atomicMin(reinterpret_cast<unsigned long long *>(&s_key[s_R[v]]),
                (unsigned long long)s_dot[v]);
    }
  __syncthreads();
  sweep(V, s_ch, [&](int v) {
    if (s_blk[v]) return false;
    const uint16_t r = s_R[v], h = s_H[v];
    uint32_t best = 0;
    for (int e = s_off[v]; e < s_off[v + 1]; e++) {
      const uint16_t y = s_dst[e];
      if (s_H[y] == h && s_R[y] != r) best = max(best, s_D[s_R[y]] + 1);
    }
    return best > s_D[r] && atomicMax(&s_D[r], best) < best;
  });
  stamp(6);
  // 5. execution order: (H, depth, representative, dot) -- the executed
  // vertices counting-sorted by ready time H (groups in H order), then each
  // one's rank inside its group by (depth, representative, dot); labels
  uint64_t lab[2];
  for (int j = 0; j < 2; j++) {
    const int v = 2 * tid + j;  // a thread's vertices are adjacent: scans follow vid order
    lab[j] = v < V && !s_blk[v] ? s_key[s_R[v]] : 0ull;
  }
  // group counts and cursors in the hash keys' space (the resolve is done)
  uint32_t *s_gs = reinterpret_cast<uint32_t *>(s_hk), *s_gc = s_gs + kSmallV;
  for (int v = tid; v < V; v += kThreads) s_gs[v] = 0;
  __syncthreads();
  for (int j = 0; j < 2; j++) {
    const int v = 2 * tid + j;
    if (v < V) {
      s_key[v] = lab[j];  // label per vertex
      if (!s_blk[v]) atomicAdd(&s_gs[s_H[v]], 1u);
    }
  }
  __syncthreads();
  uint32_t nexec = 0;
  {
    const int v0 = 2 * tid;
    const uint32_t c0 = v0 < V ? s_gs[v0] : 0u, c1 = v0 + 1 < V ? s_gs[v0 + 1] : 0u;
    const uint32_t o = block_scan(c0 + c1, s_w, &nexec);
    if (v0 < V) s_gs[v0] = s_gc[v0] = o;
    if (v0 + 1 < V) s_gs[v0 + 1] = s_gc[v0 + 1] = o + c0;
  }
  __syncthreads();
  // members listed group by group (s_W: the SCC rounds are done)
  for (int v = tid; v < V; v += kThreads)
    if (!s_blk[v]) s_W[atomicAdd(&s_gc[s_H[v]], 1u)] = uint16_t(v);
  __syncthreads();
  for (int v = tid; v < V; v += kThreads) {
    if (s_blk[v]) continue;
    const uint32_t g = s_H[v], b0 = s_gs[g], b1 = s_gc[g];
    const uint32_t rv = s_R[v], dv = s_D[rv];
    const uint64_t xv = s_dot[v];
    uint32_t rk = 0;
    for (uint32_t i = b0; i < b1; i++) {
      const uint32_t y = s_W[i];
      const uint32_t ry = s_R[y], dy = s_D[ry];
      rk += dy != dv ? dy < dv : ry != rv ? ry < rv : s_dot[y] < xv;
    }
    const uint32_t pos = b0 + rk;
    p.xdot[pos] = xv;
    p.xlab[pos] = s_key[v];
    p.xcar[pos] = uint32_t(v) < p.P ? 1 : 0;
  }
  for (int v = tid; v < V; v += kThreads) p.blocked[v] = s_blk[v];
  stamp(7);
  // survivors, compacted in arrival order into the next vertex set
  uint32_t kc[2] = {0, 0}, dc[2] = {0, 0}, kv[2] = {0, 0};
  for (int j = 0; j < 2; j++) {
    const int v = 2 * tid + j;  // a thread's vertices are adjacent: scans follow vid order
    if (v < V && s_blk[v]) {
      kv[j] = 1;
      kc[j] = p.koff[v + 1] - p.koff[v];
      dc[j] = p.doff[v + 1] - p.doff[v];
    }
  }
  uint32_t tv = 0, tk = 0, td = 0;
  uint32_t ov = block_scan(kv[0] + kv[1], s_w, &tv);
  uint32_t okk = block_scan(kc[0] + kc[1], s_w, &tk);
  uint32_t od = block_scan(dc[0] + dc[1], s_w, &td);
  for (int j = 0; j < 2; j++) {
    const int v = 2 * tid + j;  // a thread's vertices are adjacent: scans follow vid order
    if (!kv[j]) continue;
    p.ndot[ov] = s_dot[v];
    p.nkoff[ov] = okk;
    p.ndoff[ov] = od;
    for (uint32_t e = p.koff[v]; e < p.koff[v + 1]; e++) p.nkey32[okk++] = p.key32[e];
    for (uint32_t e = p.doff[v]; e < p.doff[v + 1]; e++) p.nddot[od++] = p.ddot[e];
    ov++;
  }
  if (tid == 0) {
    p.nkoff[tv] = tk;
    p.ndoff[tv] = td;
    p.header[0] = nexec;
    p.header[1] = s_nmiss;
    p.header[2] = s_err;
    p.header[3] = tv;
    p.header[4] = tk;
    p.header[5] = td;
  }
  stamp(8);
  // completion word for a host that polls the mapped block: every thread's
  // stores are made visible system-wide before it
  __threadfence_system();
  __syncthreads();
  if (tid == 0) __hip_atomic_store(&p.header[31], p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

void launch_graph_small(const SmallPass &p, hipStream_t s) {
  FH_CHECK(p.V >= 1 && p.V <= uint32_t(kSmallV), FH_EINVARIANT, "graph_small: vertex count");
  k_graph_small<<<1, kThreads, 0, s>>>(p);
  FH_HIP(hipGetLastError());  // a failed launch, before the host polls for its completion word
}

}  // namespace fh
