// graph_tile.hip -- tile-local SCC + execution order for graphs whose
// structure is position-local (replica views with a bounded reorder window).
//
// Reference semantics (graph_core.h): the incremental DependencyGraph +
// TarjanSCCFinder (fantoch_ps/src/executor/graph/mod.rs:215-644,
// tarjan.rs:98-319) executes SCC S when the last vertex it reaches arrives:
// its ready time H(S) = the maximum arrival position reachable from S.  SCCs
// that become ready together run deps first (Tarjan pops them in reverse
// topological order), members of an SCC in dot order (tarjan.rs:14-15).  The
// execution order is therefore sorted by (H, depth, tie, dot) where depth is
// the longest dependency path to the group's root SCC among the SCCs sharing
// H, and tie separates unconnected SCCs (min member vid).
//
// Locality certificate.  Let excess(v) = H(v) - v.  If every vertex has
// excess < R0 and every forward edge (a dependency that arrived later) spans
// fewer than L - R0 positions, with L = 2·R0, then for a tile core [a, b) and
// its context [a - L, b + L):
//  * a path from any vertex of [a - R0, b + R0) that leaves the context
//    below can never climb back (that would need a climb > L - R0 >= R0),
//    and one cannot leave above (H(v) < v + R0 <= b + L);
//  * so H, the SCCs, the depths and the ready groups G_t = {v : H(v) = t}
//    of every group with a member in the core (G_t lies in [t - R0, t]) are
//    the same in the context subgraph as in the whole graph.
// Conversely if some vertex has excess >= R0, take a shortest path climbing
// >= R0: it stays in [x, x + R0 + span) and x's own tile sees it (or a long
// forward edge).  Each tile checks both conditions for its core vertices; any
// failure sends the batch to the global path (graph_core.hip).
//
// Per tile, in LDS (1024 threads, context <= 8192 vertices, u16 local ids):
//  1. context edges (in-batch deps with both ends in the context);
//  2. H by max-propagation sweeps to the fixpoint;
//  3. certificate for the core;
//  4. SCCs: round 1 = the members of each group reachable from its root t
//     (H(t) = t) inside the group; later rounds recompute H over the vertices
//     left and repeat (a group holds few SCCs: the measured C4 maximum is 4);
//  5. SCC slot = min member; depth by max-propagation over same-group edges;
//  6. ready groups: count of each core root's group, and each core vertex's
//     rank in its group by (depth, min member, dot), scanning the compacted
//     list of raised vertices (H(v) > v) of the group's window.
// Global epilogue (graph_core.hip): exclusive scan of the group counts gives
// each group's first execution position, exec_rank = start[H] + rank.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "graph_core.h"

namespace fh {
namespace {

constexpr int kTileThreads = 1024;
constexpr int kTileC = 10240;  // max context vertices (LDS: 15 B per vertex)
constexpr uint16_t kNone = 0xFFFF;
constexpr int kMaxCore = 10;    // core vertices per thread (T <= 10240)
constexpr uint32_t kMixR1 = 512;  // pass-1 reach bound of the mixed tiling

// R0 rounded up to a multiple of 64 (at least 256)
// (floor: 256, or 128 for the key-order graph, whose edges span a handful of
// positions: C4 excess 102 -> R0 128, T 9728 instead of 9216)
static uint32_t round_r0(uint32_t x, uint32_t floor = 256) {
  return std::max<uint32_t>(floor, (x + 63) & ~63u);
}

// exclusive scan of one value per thread over the TH-thread block
template <int TH>
__device__ __forceinline__ uint32_t tile_scan(uint32_t v, uint32_t *s_w, uint32_t *total) {
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
  for (int i = 0; i < TH / 64; i++) {
    const uint32_t c = s_w[i];
    if (i < w) pre += c;
    tot += c;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// 16-bit LDS min / max through a CAS on the aligned 32-bit word
__device__ __forceinline__ void lds_min_u16(uint16_t *p, uint16_t v) {
  uint32_t *w = reinterpret_cast<uint32_t *>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(3));
  const int sh = int(reinterpret_cast<uintptr_t>(p) & 2) * 8;
  uint32_t old = *w;
  for (;;) {
    if (uint16_t(old >> sh) <= v) return;
    const uint32_t nw = (old & ~(0xFFFFu << sh)) | (uint32_t(v) << sh);
    const uint32_t prev = atomicCAS(w, old, nw);
    if (prev == old) return;
    old = prev;
  }
}
__device__ __forceinline__ bool lds_max_u16(uint16_t *p, uint16_t v) {
  uint32_t *w = reinterpret_cast<uint32_t *>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(3));
  const int sh = int(reinterpret_cast<uintptr_t>(p) & 2) * 8;
  uint32_t old = *w;
  for (;;) {
    if (uint16_t(old >> sh) >= v) return false;
    const uint32_t nw = (old & ~(0xFFFFu << sh)) | (uint32_t(v) << sh);
    const uint32_t prev = atomicCAS(w, old, nw);
    if (prev == old) return true;
    old = prev;
  }
}

__device__ __forceinline__ uint16_t lds_add_u16(uint16_t *p, uint16_t v) {
  uint32_t *w = reinterpret_cast<uint32_t *>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(3));
  const int sh = int(reinterpret_cast<uintptr_t>(p) & 2) * 8;
  // a 32-bit add of v << sh: the low half never carries into the high half
  // because every count stays below 2^16
  return uint16_t(atomicAdd(w, uint32_t(v) << sh) >> sh);
}

__device__ __forceinline__ uint16_t lds_xchg_u16(uint16_t *p, uint16_t v) {
  uint32_t *w = reinterpret_cast<uint32_t *>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(3));
  const int sh = int(reinterpret_cast<uintptr_t>(p) & 2) * 8;
  uint32_t old = *w;
  for (;;) {
    const uint32_t nw = (old & ~(0xFFFFu << sh)) | (uint32_t(v) << sh);
    const uint32_t prev = atomicCAS(w, old, nw);
    if (prev == old) return uint16_t(old >> sh);
    old = prev;
  }
}

}  // namespace

// graph_tile's outputs and launch parameters (named: GraphCore::tiles_mixed
// takes it)
struct TileOut {
  uint32_t *rep;     // [V] global vid of the SCC's min member, or null (not written)
  uint64_t *label;   // [V] min dot of the SCC
  uint32_t *hgrp;    // [V] ready time H (a vertex position)
  uint32_t *grank;   // [V] rank inside the ready group
  uint32_t *gcount;  // [V] size of the group rooted at v (0 if H(v) != v)
  uint32_t *stat;    // [0] failed tiles, [1] max core local excess,
                     // [2] core vertices over R0, [3] long forward edges,
                     // [4] max H sweeps, [5] max SCC rounds, [6] max group
  const uint8_t *redo;  // [tiles] or null: only tiles with redo[t] run
  const uint32_t *cores;  // [2·tiles] or null: tile t's core is [cores[2t], + cores[2t+1])
  uint8_t *failf;         // [tiles] or null: 1 for each tile whose certificate fails
  unsigned long long *prof;  // [8] or null: per-phase clock sums (FH_GRAPH_DEBUG)
  int r0;      // certified reach bound R0 (L = 2·R0)
  int core;    // core vertices per tile T (T + 2L <= tile_ctx(th), T <= kMaxCore·th)
  int th = kTileThreads;  // threads per workgroup (1024, or 512: half the context)
  // the engine's key-order graph (GraphInput::dst_codes / dot32): edges as
  // one u32 of 8-bit distances per vertex (GraphInput::dst_codes) and the
  // dots packed src << dot_sb | seq
  bool codes = false;
  const uint32_t *dot32 = nullptr;
  int dot_sb = 0;
  const uint32_t *esc = nullptr;  // codes: escaped targets (GraphInput::dst_esc)
  bool prio = false;              // raise the waves' issue priority
  // key-order outputs (GraphInput::ko_seq; the engine's key-order path):
  // each core vertex writes its dot at its key-order execution position
  // (the per-key sequence), and a vertex of a multi-member ready group its
  // command-order record and straddle difference (engine.hip k_ko_final);
  // label / hgrp / grank / gcount are then not written.  cmd: the sorted
  // values (command index in the low word, stride cstride words).
  uint64_t *ko_seq = nullptr;
  uint4 *ko_hl = nullptr;
  uint32_t *ko_diff = nullptr;
  const uint32_t *ko_cmd = nullptr;
  uint32_t ko_cstride = 0, ko_cmask = 0;
  __device__ __forceinline__ uint64_t vdot(const uint64_t *dot, uint32_t v) const {
    if (!dot32) return dot[v];
    const uint32_t d = dot32[v];
    return (uint64_t(d >> dot_sb) << 56) | (d & ((1u << dot_sb) - 1));
  }
};

namespace {


// One tile: core [a, a + T), context [a - L, a + T + L) with L = 2·R0 and
// T + 2L <= kTileC.
template <int S, int TH, bool D32>
__global__ void __launch_bounds__(TH, 4)
    k_graph_tile(uint32_t V, const uint32_t *__restrict__ dst, const uint64_t *__restrict__ dot,
                 TileOut out) {
  constexpr int CTX = TH * (kTileC / kTileThreads);  // context vertices: 10 per thread
  const int R0 = out.r0, T = out.core, L = 2 * R0;  // host: T + 2L <= CTX
  if (out.redo && !out.redo[blockIdx.x]) return;
  __shared__ __align__(16) uint16_t eL[S][CTX];
  __shared__ uint16_t sH[CTX];
  __shared__ uint16_t sR[CTX];
  __shared__ uint8_t sF[CTX];
  __shared__ uint16_t W1[CTX];
  __shared__ __align__(16) uint16_t W2[CTX];
  // rank-phase member keys: S = 3 reuses the third edge row, S = 2 has room
  __shared__ uint32_t gkey_s[S == 3 ? 1 : CTX / 2];
  __shared__ uint32_t s_w[TH / 64];
  __shared__ uint32_t s_ch[3];
  __shared__ uint32_t s_fail, s_maxex, s_over, s_long;

  const int tid = threadIdx.x;
  // issue priority over co-resident waves (the engine's key-order path runs
  // its command-order kernels on a side stream beside this one)
  if (out.prio) __builtin_amdgcn_s_setprio(3);
  uint64_t t_last = wall_clock64();
  auto phase = [&](int i) {  // after a barrier: thread 0 accounts the phase
    if (out.prof && tid == 0) {
      const uint64_t now = wall_clock64();
      atomicAdd(&out.prof[i], (unsigned long long)(now - t_last));
      t_last = now;
    }
  };
  const uint32_t a = out.cores ? out.cores[2 * blockIdx.x] : blockIdx.x * uint32_t(T);
  const uint32_t b = min(V, a + (out.cores ? out.cores[2 * blockIdx.x + 1] : uint32_t(T)));
  const uint32_t lo = a > uint32_t(L) ? a - L : 0u;
  const uint32_t hi = min(V, b + uint32_t(L));
  const int C = int(hi - lo);
  const int ca = int(a - lo), cb = int(b - lo);  // core, local
  if (tid < 3) s_ch[tid] = 0;
  if (tid == 0) s_fail = s_maxex = s_over = s_long = 0;
  // the core vertices' own dots, loaded now and used by the last phase (its
  // labels and dot tie-breaks): the loads complete behind the LDS phases
  // (D32: the dots packed to 32 bits, GraphInput::dot32 -- half the
  // registers, which pays for the group roots' dots prefetched below)
  using DotT = std::conditional_t<D32, uint32_t, uint64_t>;
  auto unpack = [&](DotT d) -> uint64_t {
    if constexpr (D32)
      return (uint64_t(d >> out.dot_sb) << 56) | (d & ((1u << out.dot_sb) - 1));
    else
      return d;
  };
  auto ldot = [&](uint32_t v) -> DotT {
    if constexpr (D32)
      return out.dot32[v];
    else
      return dot[v];
  };
  DotT pdot[kMaxCore];
  uint32_t pcmd[kMaxCore];
  // issued after the edge words (with codes), so that the edge decode waits
  // for those alone (vmcnt retires in issue order)
  auto prefetch_core = [&]() {
#pragma unroll
    for (int j = 0; j < kMaxCore; j++) {
      const int x = ca + tid + j * TH;
      pdot[j] = x < cb ? ldot(lo + x) : DotT(0);
      pcmd[j] = out.ko_seq && x < cb ? out.ko_cmd[size_t(lo + x) * out.ko_cstride] & out.ko_cmask
                                     : 0u;
    }
  };

  // 1. context edges; certificate part 2: forward spans of core vertices
  uint32_t nlong = 0;
  auto put_edge = [&](int x, int s, uint32_t v, uint32_t u) {
    uint16_t l = kNone;
    if (u != v && u >= lo && u < hi) l = uint16_t(u - lo);
    if (x >= ca && x < cb && u > v && u - v >= uint32_t(L - R0)) nlong++;
    eL[s][x] = l;
  };
  if (out.codes) {
    // one word per vertex: all of the thread's words in flight at once
    constexpr int kPI = CTX / TH;
    uint32_t ew[kPI];
#pragma unroll
    for (int j = 0; j < kPI; j++) {
      const int x = tid + j * TH;
      ew[j] = x < C ? dst[lo + x] : 0u;
    }
    prefetch_core();
#pragma unroll
    for (int j = 0; j < kPI; j++) {
      const int x = tid + j * TH;
      if (x >= C) break;
      const uint32_t v = lo + x;
#pragma unroll
      for (int s = 0; s < S; s++) {
        const int d = int(int8_t(uint8_t(ew[j] >> (8 * s))));
        const uint32_t u =
            d == 0 ? v : d == -128 ? out.esc[size_t(v) * S + s] - 1u : uint32_t(int(v) - d);
        put_edge(x, s, v, u);
      }
      sH[x] = uint16_t(x);
    }
  } else {
    prefetch_core();
    for (int x = tid; x < C; x += TH) {
      const uint32_t v = lo + x;
#pragma unroll
      for (int s = 0; s < S; s++) put_edge(x, s, v, dst[size_t(v) * S + s]);
      sH[x] = uint16_t(x);
    }
  }
  __syncthreads();
  phase(0);
  if (nlong) atomicAdd(&s_long, nlong);

  // sweep helper: body(x) returns true if it changed something; loops until
  // a sweep changes nothing (rotating flags: one barrier per sweep)
  auto sweeps = [&](auto body, int n, const uint16_t *list) {
    int it = 0;
    for (;; it++) {
      bool ch = false;
      for (int i = tid; i < n; i += TH) ch |= body(list ? int(list[i]) : i);
      if (ch) s_ch[it % 3] = 1;
      if (tid == 0) s_ch[(it + 1) % 3] = 0;
      __syncthreads();
      if (!s_ch[it % 3]) break;
    }
    __syncthreads();
    if (tid < 3) s_ch[tid] = 0;
    __syncthreads();
    return it + 1;
  };

  // 2. H: max arrival position reachable (context subgraph).  H(x) is a
  // vertex x reaches, so H(H(x)) is reachable too: pointer jumping collapses
  // chains of forward dependencies in logarithmically many sweeps.
  const int hP = 64 * ((C + TH - 1) / TH);  // per-wave block
  // Each wave walks a contiguous block in ascending steps of 64 (updates of a
  // block's earlier vertices are seen by its later ones in the same sweep),
  // with each thread's vertices' context edges and own H in registers: the thread owning x is the only writer of sH[x], so its
  // register copy stays exact, and a sweep's LDS traffic is the random
  // sH[y] / sH[H] reads alone (the edge rows and own H were conflict-free
  // re-reads of the same words every sweep)
  auto h_sweeps_regs = [&]() {
    constexpr int kHI = CTX / TH;
    const int w = tid >> 6, lane = tid & 63, nk = hP / 64;
    uint16_t ey[kHI][S];
    uint32_t hv[kHI];
#pragma unroll
    for (int j = 0; j < kHI; j++) {
      const int x = w * hP + j * 64 + lane;
      const bool ok = j < nk && x < C;
      hv[j] = ok ? uint32_t(x) : 0xFFFFFFFFu;  // sH[x] starts at x; ~0: no vertex
#pragma unroll
      for (int q = 0; q < S; q++) ey[j][q] = ok ? eL[q][x] : kNone;
    }
    int it = 0;
    for (;; it++) {
      bool ch = false;
#pragma unroll
      for (int j = 0; j < kHI; j++) {
        if (hv[j] == 0xFFFFFFFFu) continue;
        uint32_t h = hv[j];
        const uint32_t h0 = h;
#pragma unroll
        for (int q = 0; q < S; q++)
          if (ey[j][q] != kNone) h = max(h, uint32_t(sH[ey[j][q]]));
        h = max(h, uint32_t(sH[h]));
        if (h > h0) {
          sH[w * hP + j * 64 + lane] = uint16_t(h);
          hv[j] = h;
          ch = true;
        }
      }
      if (ch) s_ch[it % 3] = 1;
      if (tid == 0) s_ch[(it + 1) % 3] = 0;
      __syncthreads();
      if (!s_ch[it % 3]) break;
    }
    __syncthreads();
    if (tid < 3) s_ch[tid] = 0;
    __syncthreads();
    return it + 1;
  };
  const int hs = h_sweeps_regs();
  phase(1);

  // 3. certificate part 1: core excess < R0
  {
    uint32_t mx = 0, over = 0;
    for (int x = ca + tid; x < cb; x += TH) {
      const uint32_t ex = uint32_t(sH[x]) - uint32_t(x);
      mx = max(mx, ex);
      over += ex >= uint32_t(R0);
    }
    if (mx) atomicMax(&s_maxex, mx);
    if (over) atomicAdd(&s_over, over);
  }
  __syncthreads();
  if (tid == 0) {
    atomicMax(&out.stat[1], s_maxex);
    if (s_over) atomicAdd(&out.stat[2], s_over);
    if (s_long) atomicAdd(&out.stat[3], s_long);
    atomicMax(&out.stat[4], uint32_t(hs));
    if (s_over || s_long) atomicAdd(&out.stat[0], 1u);
    if ((s_over || s_long) && out.failf) out.failf[blockIdx.x] = 1;
  }
  if (s_over || s_long) return;

  // 4. raised vertices (H(v) > v), ascending, into W2 (an ordered
  // compaction: each thread takes consecutive positions).  Every vertex of a
  // multi-vertex ready group except its root is raised, so the later phases
  // work on this list only.  sF bits: 1 reached, 2 processed, 4 the group
  // rooted here has raised members.
  constexpr int kPer = CTX / TH;
  uint32_t nraised = 0;
  for (int x = tid; x < C; x += TH) {
    sF[x] = 0;
    sR[x] = kNone;
  }
  __syncthreads();
  {
    uint32_t mine = 0;
    const int x0 = tid * kPer;
    for (int x = x0; x < x0 + kPer && x < C; x++) mine += sH[x] > x;
    uint32_t o = tile_scan<TH>(mine, s_w, &nraised);
    for (int x = x0; x < x0 + kPer && x < C; x++)
      if (sH[x] > x) W2[o++] = uint16_t(x);
  }
  __syncthreads();
  for (uint32_t i = tid; i < nraised; i += TH) sF[sH[W2[i]]] = 4;
  __syncthreads();
  phase(2);

  // 5. SCCs.  Round 1: the members of each ready group reachable from its
  // root t (H(t) = t) inside the group are t's SCC.  Roots push once; then
  // the raised vertices reached push until nothing new is reached.
  for (int x = tid; x < C; x += TH) {
    if (sH[x] != x) continue;
    sF[x] |= 3;
    sR[x] = uint16_t(x);
    if (!(sF[x] & 4)) continue;  // no raised member: a singleton group
#pragma unroll
    for (int s = 0; s < S; s++) {
      const uint16_t y = eL[s][x];
      if (y != kNone && sH[y] == x) sF[y] |= 1;
    }
  }
  __syncthreads();
  auto reach = [&](const uint16_t *grp) {
    // grp: the group label array (sH in round 1, W1 later); only unassigned
    // (sR == kNone) raised vertices take part
    sweeps(
        [&](int i) {
          const uint16_t x = W2[i];
          const uint8_t f = sF[x];
          if ((f & 3) != 1 || sR[x] != kNone) return false;
          sF[x] = f | 2;
          const uint16_t g = grp[x];
#pragma unroll
          for (int s = 0; s < S; s++) {
            const uint16_t y = eL[s][x];
            if (y != kNone && sR[y] == kNone && grp[y] == g) sF[y] |= 1;
          }
          return true;
        },
        int(nraised), nullptr);
  };
  reach(sH);
  // assign round 1; count the raised vertices left
  uint32_t left = 0;
  {
    uint32_t mine = 0;
    for (uint32_t i = tid; i < nraised; i += TH) {
      const uint16_t x = W2[i];
      if (sF[x] & 1)
        sR[x] = sH[x];
      else
        mine++;
    }
    tile_scan<TH>(mine, s_w, &left);
  }
  phase(3);
  // later rounds over the raised vertices left: H' over the unassigned
  // subgraph (W1, pointer jumping), roots H'(x) = x, reach inside the H'
  // group, assign
  int round = 0;
  for (; left; round++) {
    if (round >= 64) {  // adversarial nesting: leave it to the global path
      if (tid == 0) {
        atomicAdd(&out.stat[0], 1u);
        if (out.failf) out.failf[blockIdx.x] = 1;
      }
      return;
    }
    for (uint32_t i = tid; i < nraised; i += TH) {
      const uint16_t x = W2[i];
      if (sR[x] == kNone) {
        W1[x] = x;
        sF[x] &= 4;
      }
    }
    __syncthreads();
    sweeps(
        [&](int i) {
          const uint16_t x = W2[i];
          if (sR[x] != kNone) return false;
          uint32_t h = W1[x];
          const uint32_t h0 = h;
#pragma unroll
          for (int s = 0; s < S; s++) {
            const uint16_t y = eL[s][x];
            if (y != kNone && sR[y] == kNone) h = max(h, uint32_t(W1[y]));
          }
          h = max(h, uint32_t(W1[h]));
          if (h > h0) {
            W1[x] = uint16_t(h);
            return true;
          }
          return false;
        },
        int(nraised), nullptr);
    for (uint32_t i = tid; i < nraised; i += TH) {
      const uint16_t x = W2[i];
      if (sR[x] == kNone && W1[x] == x) sF[x] |= 1;
    }
    __syncthreads();
    reach(W1);
    uint32_t mine = 0;
    for (uint32_t i = tid; i < nraised; i += TH) {
      const uint16_t x = W2[i];
      if (sR[x] != kNone) continue;
      if (sF[x] & 1)
        sR[x] = W1[x];  // (W1[x] is unassigned until this pass ends)
      else
        mine++;
    }
    __syncthreads();
    tile_scan<TH>(mine, s_w, &left);
  }
  if (tid == 0 && round) atomicMax(&out.stat[5], uint32_t(round));

  // 6. SCC slot = min member; depth over same-group edges (W1, per slot).
  // Only raised vertices can have an edge to another SCC of their group (a
  // root's same-group dependencies reach it back), so the sweeps run over W2.
  for (int x = tid; x < C; x += TH) W1[x] = kNone;
  __syncthreads();
  for (int x = tid; x < C; x += TH) lds_min_u16(&W1[sR[x]], uint16_t(x));
  __syncthreads();
  for (int x = tid; x < C; x += TH) sR[x] = W1[sR[x]];
  __syncthreads();
  for (int x = tid; x < C; x += TH) W1[x] = 0;
  __syncthreads();
  sweeps(
      [&](int i) {
        const uint16_t x = W2[i];
        const uint16_t r = sR[x], hx = sH[x];
        uint32_t best = 0;
#pragma unroll
        for (int s = 0; s < S; s++) {
          const uint16_t y = eL[s][x];
          if (y != kNone && sH[y] == hx) {
            const uint16_t r2 = sR[y];
            if (r2 != r) best = max(best, uint32_t(W1[r2]) + 1);
          }
        }
        return best > W1[r] && lds_max_u16(&W1[r], uint16_t(best));
      },
      int(nraised), nullptr);
  phase(4);

  // 7. ready groups: the raised vertices counting-sorted by group root into
  // eL[1] (group t's members at [end(t-1), end(t)), ends in eL[0]; the edges
  // are no longer needed), then each core vertex's rank in its group by
  // (depth, min member, dot) and each core root's group size
  uint16_t *gend = eL[0], *gmem = eL[1];
  for (int x = tid; x < C; x += TH) gend[x] = 0;
  __syncthreads();
  for (uint32_t i = tid; i < nraised; i += TH) lds_add_u16(&gend[sH[W2[i]]], 1);
  __syncthreads();
  {
    const int x0 = tid * kPer;
    uint32_t sum = 0;
    for (int x = x0; x < x0 + kPer && x < C; x++) sum += gend[x];
    uint32_t tot = 0;
    uint32_t base = tile_scan<TH>(sum, s_w, &tot);
    for (int x = x0; x < x0 + kPer && x < C; x++) {
      const uint32_t c = gend[x];
      gend[x] = uint16_t(base);
      base += c;
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < nraised; i += TH) {
    const uint16_t y = W2[i];
    gmem[lds_add_u16(&gend[sH[y]], 1)] = y;
  }
  __syncthreads();
  // the group members' dots, staged once in W2's space (the raised list is
  // consumed): members of one SCC tie on (depth, min member) and compare
  // dots, which would otherwise be one round of global loads per 8 members
  // for every vertex of a large SCC
  // With them each member's order key (depth << 16 | SCC slot), so the rank
  // loop reads two independent arrays instead of a gmem -> sR -> W1 chain.
  // key order: rp[j] = raised context vertices below the root t of core
  // vertex j's group (W2 is still the ascending raised list); with b0 =
  // gend[t - 1] = raised vertices whose group root is below t, rp - b0 =
  // straddle(t) = vertices u < t with H(u) >= t (all within R0 below t, in
  // the context, with exact H: the certificate), so t's group starts at
  // lo + t - straddle(t) in the key-order execution.
  uint32_t rpv[kMaxCore];
  if (out.ko_seq) {
#pragma unroll
    for (int j = 0; j < kMaxCore; j++) {
      const int x = ca + tid + j * TH;
      uint32_t l0 = 0, h0 = nraised;
      if (x < cb) {
        const uint16_t t = sH[x];
        while (l0 < h0) {
          const uint32_t mid = (l0 + h0) >> 1;
          if (W2[mid] < t)
            l0 = mid + 1;
          else
            h0 = mid;
        }
      }
      rpv[j] = l0;
    }
    __syncthreads();  // W2 becomes gdot below
  }
  uint64_t *gdot = reinterpret_cast<uint64_t *>(W2);
  uint32_t *gkey = S == 3 ? reinterpret_cast<uint32_t *>(&eL[S - 1][0]) : gkey_s;
  const bool lds_dots = nraised <= uint32_t(CTX / 4);
  if (lds_dots)
    for (uint32_t i = tid; i < nraised; i += TH) {
      const uint16_t y = gmem[i];
      gdot[i] = out.vdot(dot, lo + y);
      gkey[i] = (uint32_t(W1[sR[y]]) << 16) | sR[y];
    }
  __syncthreads();
  phase(5);
  // the root's command (key-order outputs) for every core vertex of the
  // thread first, the loads all in flight together (inside the loop each was
  // a serialised round trip per vertex; phase 6: 50 -> 20 us per tile with
  // the root's dot prefetched too, but that took the kernel to 125 VGPRs, and
  // 4 waves x 128 registers fill each SIMD's file: the side stream's kernels
  // could no longer run beside the tile workgroup, C4 14.5 -> 16.4 ms.  With
  // the command alone: 105 VGPRs, C4 14.52 against 14.55 ms, r05ai)
  // With D32 the roots' dots too: the rank loop below then issues no load.
  // (Its stores -- the per-key sequence, the command-order records -- count
  // in vmcnt like loads on gfx9, so a load inside the loop waited for every
  // earlier iteration's stores: one loaded-HBM round trip per core vertex,
  // ~65 us per tile of 128.)
  uint32_t rcv[kMaxCore];
  DotT rdv[D32 ? kMaxCore : 1];
#pragma unroll
  for (int j = 0; j < kMaxCore; j++) {
    const int x = ca + tid + j * TH;
    rcv[j] = pcmd[j];
    if constexpr (D32) rdv[j] = 0;
    if (x < cb) {
      const uint16_t t = sH[x];
      if (t != uint32_t(x)) {
        if (out.ko_seq) rcv[j] = out.ko_cmd[size_t(lo + t) * out.ko_cstride] & out.ko_cmask;
        if constexpr (D32) rdv[j] = out.dot32[lo + t];
      }
    }
  }
  uint32_t gmax = 0;
#pragma unroll
  for (int j = 0; j < kMaxCore; j++) {
    const int x = ca + tid + j * TH;
    if (x >= cb) break;
    const uint32_t v = lo + x;
    const uint64_t dotx = unpack(pdot[j]);
    const uint16_t t = sH[x];
    uint32_t cnt = 0, rk = 0;
    uint64_t lab = 0;  // min dot of x's SCC (0 = x's own: a singleton group)
    if (sF[t] & 4) {
      const uint32_t b0 = t ? gend[t - 1] : 0u, b1 = gend[t];
      cnt = b1 - b0;
      const uint32_t dx = W1[sR[x]], mx = sR[x];
      // the root's dot (prefetched with D32)
      auto root_dot = [&]() -> uint64_t {
        if constexpr (D32)
          return unpack(rdv[j]);
        else
          return out.vdot(dot, lo + t);
      };
      if (t != uint32_t(x)) {
        const uint32_t dy = W1[sR[t]], my = sR[t];
        rk += dy != dx ? dy < dx : my != mx ? my < mx : root_dot() < dotx;
      }
      if (lds_dots) {
        // x's own entry (if raised) ties with itself on the dot: not before
        // x, and its dot is x's own in the label minimum
        const uint32_t kx = (dx << 16) | mx;
        for (uint32_t j = b0; j < b1; j += 8) {
          uint32_t kk[8];
#pragma unroll
          for (int u = 0; u < 8; u++) kk[u] = j + u < b1 ? gkey[j + u] : 0xFFFFFFFFu;
#pragma unroll
          for (int u = 0; u < 8; u++) {
            rk += kk[u] < kx;
            if (kk[u] == kx) {
              const uint64_t dy = gdot[j + u];
              rk += dy < dotx;
              if (lab == 0 || dy < lab) lab = dy;
            }
          }
        }
      } else
      // members 8 at a time: (depth, min member) from LDS, and the dots of
      // same-SCC members loaded together (independent L2 loads in flight)
      for (uint32_t j = b0; j < b1; j += 8) {
        uint32_t ys[8];
        int st[8];  // -1 before x, 1 after x, 0 tie on the SCC (dot decides)
        uint64_t dy[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          ys[u] = j + u < b1 ? gmem[j + u] : uint32_t(x);
          const uint32_t d2 = W1[sR[ys[u]]], m2 = sR[ys[u]];
          st[u] = ys[u] == uint32_t(x) ? 1 : d2 != dx ? (d2 < dx ? -1 : 1)
                                       : m2 != mx ? (m2 < mx ? -1 : 1) : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
          dy[u] = st[u] != 0 ? 0ull : lds_dots ? gdot[j + u] : out.vdot(dot, lo + ys[u]);
#pragma unroll
        for (int u = 0; u < 8; u++) {
          rk += st[u] < 0 || (st[u] == 0 && dy[u] < dotx);
          if (st[u] == 0 && (lab == 0 || dy[u] < lab)) lab = dy[u];
        }
      }
      // the root t is in x's SCC iff it shares the SCC slot (the root test above
      // compared it; its dot was not kept)
      if (t != uint32_t(x) && sR[t] == mx) {
        const uint64_t dt = root_dot();
        if (lab == 0 || dt < lab) lab = dt;
      }
      gmax = max(gmax, cnt + 1);
    }
    const uint64_t label = (lab == 0 || dotx < lab) ? dotx : lab;
    if (out.ko_seq) {
      const uint32_t b0 = t ? uint32_t(gend[t - 1]) : 0u;
      out.ko_seq[lo + t - rpv[j] + b0 + rk] = dotx;
      if (t != uint32_t(x) || cnt > 0) {
        const uint32_t c = pcmd[j];
        const uint32_t ct = rcv[j];
        out.ko_hl[c] = make_uint4(ct, rk, uint32_t(label), uint32_t(label >> 32));
        out.ko_diff[c + 1] = t != uint32_t(x) ? 1u : 0u - cnt;
      }
      continue;
    }
    out.label[v] = label;
    if (out.rep) out.rep[v] = lo + sR[x];
    out.hgrp[v] = lo + t;
    out.grank[v] = rk;
    out.gcount[v] = t == uint32_t(x) ? cnt + 1 : 0u;
  }
  if (gmax) atomicMax(&out.stat[6], gmax);
  // no trailing barrier outside the phase profile: a barrier waits for every
  // wave's stores to complete (a workgroup-scope release), and beside the
  // side stream's row stores that drain took ~40 us of the tile's ~117
  if (out.prof) {
    __syncthreads();
    phase(6);
  }
}

__global__ void k_exec_from_groups(uint32_t V, const uint32_t *__restrict__ hgrp,
                                   const uint32_t *__restrict__ grank,
                                   const uint32_t *__restrict__ gstart, uint32_t *__restrict__ rank,
                                   uint32_t *__restrict__ order) {
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x) {
    const uint32_t r = gstart[hgrp[v]] + grank[v];
    rank[v] = r;
    order[r] = v;
  }
}

}  // namespace

// Cores up to 10240 vertices (kMaxCore = 10): on the key-order graph the reach
// bound is small, so T = kTileC - 4·R0 exceeds 8192 and fewer tiles carry
// the fixed per-tile phases (C4: 14.83 against 14.94 ms at T <= 8192, r05z)
static int tile_core_cap(int th = kTileThreads) { return kMaxCore * th; }
// context vertices of a th-thread tile (10 per thread; the LDS: 15 B each)
static int tile_ctx(int th) { return th * (kTileC / kTileThreads); }

static void launch_tiles(uint32_t V, uint32_t S, const uint32_t *dst, const uint64_t *dot,
                         const TileOut &to, hipStream_t stream, uint32_t ncores = 0,
                         bool count_bytes = true) {
  FH_CHECK(to.core >= 1024 && to.core <= kMaxCore * to.th &&
               to.core + 4 * to.r0 <= tile_ctx(to.th) && to.r0 >= 64 &&
               (to.th == 1024 || to.th == 512),
           FH_EINVARIANT, "graph_tile: bad tile geometry");
  const uint32_t tiles = to.cores ? ncores : (V + to.core - 1) / to.core;
  if (tiles == 0) return;
  // algorithmic bytes: read the vertex's S edge slots and its dot (labels and
  // dot tie-breaks), write H, rank, group count and the label (rep too when
  // asked for; the context halo re-reads are overhead, not algorithmic; so is
  // a redo pass over cores already ordered once: count_bytes = false)
  const double bytes =
      count_bytes ? double(V) * (4.0 * S + 8.0 + (to.rep ? 16.0 : 12.0) + 8.0) : 0.0;
  auto go = [&](auto kern) {
    probed_launch("graph_tile", bytes, kern, dim3(tiles), dim3(to.th), stream, V, dst, dot, to);
  };
  const bool d32 = to.dot32 != nullptr;
  if (S == 2) {
    if (to.th == 512)
      d32 ? go(k_graph_tile<2, 512, true>) : go(k_graph_tile<2, 512, false>);
    else
      d32 ? go(k_graph_tile<2, 1024, true>) : go(k_graph_tile<2, 1024, false>);
  } else {
    if (to.th == 512)
      d32 ? go(k_graph_tile<3, 512, true>) : go(k_graph_tile<3, 512, false>);
    else
      d32 ? go(k_graph_tile<3, 1024, true>) : go(k_graph_tile<3, 1024, false>);
  }
}

// Mixed reach bounds.  Pass 1 runs every tile at R1 = kMixR1 (T1 = 8192);
// pass 2 reruns, at R2 (T2 = kTileC - 4·R2), the cores of every failed tile
// and of its two neighbours.  Why the kept tiles are right: with global
// excess < R2 (pass 2's certificate, below), a vertex whose excess is >= R1
// climbs through the lowest vertex y of its climbing path, whose own tile
// (or the tile of a long forward edge within R1 above y) sees the climb in
// its context and fails; so such vertices lie less than R1 + R2 above a
// failed core.  A kept tile's proof (file header, at R1) needs excess < R1
// on [a - R1, b + R1), no climb back from below a - L1 (a vertex there with
// excess > L1 - R1 = R1 would lie within R1 + R2 above a failed core, i.e.
// within 2·R1 + 2·R2 <= 5120 below a), and its ready groups' members within
// R1 below their roots (members of excess >= R1 again lie near a failed
// core); a neighbour on each side keeps every failed core >= T1 = 8192 away.
// Pass 2's proof at R2 needs excess < R2 everywhere: the lowest vertex with
// excess >= R2 would be seen by its own tile -- a pass-2 tile (fails the
// pass, and the run falls back to uniform bounds) or a kept tile, which sees
// its climb past R1 inside its context and would have failed in pass 1.
// Forward spans: kept tiles certify < L1 - R1 = R1 < R2.  Each pass writes
// only certified cores; pass 2 overwrites its cores.
bool GraphCore::tiles_mixed(const GraphInput &in, TileOut &to, uint32_t r2, uint32_t *st) {
  const uint32_t V = in.V;
  const uint32_t r1 = kMixR1;
  uint32_t *stat = to.stat;
  to.r0 = int(r1);
  to.th = kTileThreads;
  to.core = std::min(kTileC - 4 * int(r1), kMaxCore * kTileThreads);
  const uint32_t t1 = uint32_t(to.core), tiles1 = (V + t1 - 1) / t1;
  uint8_t *ff = t_fail.ensure(tiles1 + 1);
  FH_HIP(hipMemsetAsync(ff, 0, tiles1, stream));
  FH_HIP(hipMemsetAsync(stat, 0, 7 * sizeof(uint32_t), stream));
  if (to.prof) FH_HIP(hipMemsetAsync(to.prof, 0, 8 * sizeof(unsigned long long), stream));
  to.failf = ff;
  to.cores = nullptr;
  launch_tiles(V, in.stride, in.dst, in.dot, to, stream);
  fetch_u32(stat, st, 7, stream);
  to.failf = nullptr;
  if (st[0] == 0) return true;
  // the pass-2 bound: the requested one, at least what pass 1 saw
  r2 = std::max(r2, round_r0(st[1] + st[1] / 32 + 16));
  if (r2 > 2048) return false;
  // the proof below keeps failed cores >= T1 >= 2·R1 + 2·R2 from a kept tile
  if (2 * r1 + 2 * r2 > t1) return false;
  std::vector<uint8_t> hf(tiles1);
  FH_HIP(hipMemcpyAsync(hf.data(), ff, tiles1, hipMemcpyDeviceToHost, stream));
  FH_HIP(hipStreamSynchronize(stream));
  std::vector<uint8_t> redo(tiles1, 0);
  for (uint32_t t = 0; t < tiles1; t++)
    if (hf[t])
      for (int d = -1; d <= 1; d++)
        if (int64_t(t) + d >= 0 && int64_t(t) + d < int64_t(tiles1)) redo[t + d] = 1;
  const uint32_t t2 = uint32_t(std::min(kTileC - 4 * int(r2), tile_core_cap()));
  std::vector<uint32_t> cores;
  for (uint32_t t = 0; t < tiles1;) {
    if (!redo[t]) {
      t++;
      continue;
    }
    uint32_t e = t;
    while (e < tiles1 && redo[e]) e++;
    const uint32_t lo = t * t1, hi = std::min(V, e * t1);
    for (uint32_t x = lo; x < hi; x += t2) {
      cores.push_back(x);
      cores.push_back(std::min(t2, hi - x));
    }
    t = e;
  }
  uint32_t *dc = t_cores.ensure(cores.size() + 1);
  FH_HIP(hipMemcpyAsync(dc, cores.data(), cores.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                        stream));
  const uint32_t pass1_max = st[1];
  FH_HIP(hipMemsetAsync(stat, 0, 7 * sizeof(uint32_t), stream));
  to.r0 = int(r2);
  to.core = int(t2);
  to.cores = dc;
  launch_tiles(V, in.stride, in.dst, in.dot, to, stream, uint32_t(cores.size() / 2), false);
  fetch_u32(stat, st, 7, stream);
  to.cores = nullptr;
  dbg_mixed_redo = uint32_t(cores.size() / 2);
  st[1] = std::max(st[1], pass1_max);
  return st[0] == 0;
}

bool GraphCore::run_tiles(const GraphInput &in, GraphOutput &out) {
  const uint32_t V = in.V;
  uint32_t *stat = scalars.get() + 24;
  TileOut to;
  to.rep = nullptr;  // (no consumer: the engine and the executor read labels and ranks)
  to.label = tmp64c.ensure(V + 1);
  to.hgrp = t_h.ensure(V + 1);
  to.grank = t_rank.ensure(V + 1);
  to.gcount = t_cnt.ensure(V + 1);
  to.stat = stat;
  to.redo = nullptr;
  to.cores = nullptr;
  to.failf = nullptr;
  to.codes = in.dst_codes;
  to.esc = in.dst_esc;
  to.prio = in.tile_prio;
  to.dot32 = in.dot32;
  to.dot_sb = in.dot32_sb;
  to.ko_seq = in.ko_seq;
  to.ko_hl = in.ko_hl;
  to.ko_diff = in.ko_diff;
  to.ko_cmd = in.ko_cmd;
  to.ko_cstride = in.ko_cstride;
  to.ko_cmask = in.ko_cmask;
  static const bool debug = getenv("FH_GRAPH_DEBUG") != nullptr;
  // the key-order graph's tiles: 512 threads (C4, ms per step, three boxes:
  // 12.30 / 12.60 / 12.81 against 12.22 / 12.95 / 12.94 at 1024, r06b/d/e)
  constexpr int ko_tile_threads = 512;
  to.prof = nullptr;
  if (debug) {
    to.prof = reinterpret_cast<unsigned long long *>(t_prof.ensure(16));
    FH_HIP(hipMemsetAsync(to.prof, 0, 8 * sizeof(unsigned long long), stream));
  }
  // Certified reach bound R0 and core T = min(kTileC - 4·R0, 8192): a run
  // starts from the bound the last run's maximum excess calls for (a tighter
  // R0 = longer cores, less halo per core vertex); a certificate failure
  // retries with a larger bound (the kernel reports the excess it saw), up to
  // R0 = 2048, then the global path.
  bool ok = false;
  uint32_t st[7] = {0, 0, 0, 0, 0, 0, 0};
  uint32_t r0 = tile_r0;
  // mixed bounds: when the last run needed a bound above kMixR1, every tile
  // first runs at kMixR1 (longer cores) and only the failed tiles and their
  // neighbours run again at the larger bound
  if (tile_r0 > kMixR1) {
    dbg_mixed_redo = 0;
    ok = tiles_mixed(in, to, tile_r0, st);
    if (debug)
      fprintf(stderr,
              "fh graph_tile mixed: V=%u R1=%u R2=%u redo_cores=%u ok=%d max_excess=%u "
              "max_sweeps=%u max_rounds=%u max_group=%u\n",
              V, kMixR1, uint32_t(to.r0), dbg_mixed_redo, int(ok), st[1], st[4], st[5], st[6]);
  }
  for (int attempt = 0; attempt < 4 && !ok; attempt++) {
    to.r0 = int(r0);
    // the key-order graph: half-size tiles (two workgroups per CU, so one
    // tile's loads overlap another's LDS phases) while the bound leaves a
    // core of >= 1024 vertices
    to.th = in.ko_seq && tile_ctx(ko_tile_threads) - 4 * int(r0) >= 1024 ? ko_tile_threads
                                                                         : kTileThreads;
    to.core = std::min(tile_ctx(to.th) - 4 * int(r0), tile_core_cap(to.th));
    FH_HIP(hipMemsetAsync(stat, 0, 7 * sizeof(uint32_t), stream));
    if (to.prof) FH_HIP(hipMemsetAsync(to.prof, 0, 8 * sizeof(unsigned long long), stream));
    launch_tiles(V, in.stride, in.dst, in.dot, to, stream);
    fetch_u32(stat, st, 7, stream);
    ok = st[0] == 0;
    if (debug)
      fprintf(stderr,
              "fh graph_tile: V=%u R0=%u T=%d failed_tiles=%u max_excess=%u over=%u "
              "long_fwd=%u max_sweeps=%u max_rounds=%u max_group=%u\n",
              V, r0, to.core, st[0], st[1], st[2], st[3], st[4], st[5], st[6]);
    if (ok || r0 >= 2048) break;
    r0 = std::min<uint32_t>(2048, std::max<uint32_t>(r0 + r0 / 4, round_r0(st[1] + st[1] / 8)));
  }
  // next run: this run's excess with a small margin (a failure there only
  // costs one retry)
  tile_r0 = ok ? std::min<uint32_t>(2048, round_r0(st[1] + st[1] / 32 + 16, in.tiles_only ? 128u : 256u))
                : 1536;
  if (debug && ok) {
    unsigned long long pr[8];
    FH_HIP(hipMemcpyAsync(pr, to.prof, sizeof(pr), hipMemcpyDeviceToHost, stream));
    FH_HIP(hipStreamSynchronize(stream));
    // wall_clock64 runs at 100 MHz on gfx9: ticks * 10 ns, per tile average
    // (the profile sums every launch of this run)
    const double tiles = double((V + to.core - 1) / to.core);
    fprintf(stderr, "fh graph_tile phases (us per tile, T=%d): load %.1f H %.1f raised %.1f "
            "reach1 %.1f rounds+depth %.1f groups %.1f rank %.1f\n", to.core,
            pr[0] * 0.01 / tiles, pr[1] * 0.01 / tiles, pr[2] * 0.01 / tiles,
            pr[3] * 0.01 / tiles, pr[4] * 0.01 / tiles, pr[5] * 0.01 / tiles,
            pr[6] * 0.01 / tiles);
  }
  mark("graph_tile");
  if (!ok) {
    dbg_tile_fail++;
    return false;
  }
  if (in.ko_seq) {  // the tiles wrote the caller's outputs themselves
    out.exec_rank = nullptr;
    out.exec_order = nullptr;
    out.nexec = V;
    out.npending = 0;
    out.rep = nullptr;
    out.scc_label = nullptr;
    return true;
  }
  // execution order: groups in ready-time order, ranks inside a group
  uint32_t *gs = t_start.ensure(V + 1);
  exclusive_scan_u32(t_cnt.get(), gs, V, scan_ws, stream);
  if (in.tiles_only) {
    // the caller takes (H, rank in group, group starts, labels) as they are
    out.exec_rank = nullptr;
    out.exec_order = nullptr;
    out.nexec = V;
    out.npending = 0;
    out.rep = nullptr;
    out.scc_label = tmp64c.get();
    mark("exec_order");
    return true;
  }
  uint32_t *er = tmp32d.ensure(V + 1);
  // the per-key pass of dots takes each vertex's rank from its group and
  // writes (key, dot) at it directly (build_per_key): no order array
  fill_from_groups = in.want_per_key && in.per_key_dots && !in.key_off && in.k >= 1 &&
                     size_t(V) * in.k < (size_t(1) << 30);
  if (fill_from_groups) {
    out.exec_order = nullptr;
  } else {
    uint32_t *ord = order.ensure(V + 1);
    k_exec_from_groups<<<grid_for(V, 256), 256, 0, stream>>>(V, t_h.get(), t_rank.get(), gs, er, ord);
    out.exec_order = ord;
  }
  out.exec_rank = er;
  out.nexec = V;
  out.npending = 0;
  out.rep = nullptr;
  out.scc_label = tmp64c.get();
  mark("exec_order");
  return true;
}

bool GraphCore::tiles_eligible(const GraphInput &in) const {
  return !in.off && !in.blocked0 && in.stride >= 2 && in.stride <= 3 && in.V >= 1;
}

}  // namespace fh
