// dgraph.hip -- partial replication across GPUs (fh_dgraph_*, SURVEY §8e,
// BASELINE config C5): one process per GPU, rank q of N.
//
// The reference runs a command's collect on every shard it touches, each
// shard's KeyDeps over the command's keys on that shard only
// (Command::keys(shard), fantoch/src/command.rs:95-100; atlas.rs:214-328),
// commits the union of the shards' reports (MShardCommit, atlas.rs:559-639),
// and orders the committed graph with GraphExecutor, fetching the vertices of
// other shards it reaches through requests (executor/graph/mod.rs:279-408,
// index.rs:171-205).  Here:
//
//  1. KeyDeps by key shard.  Rank q runs the processes of shards h with
//     h % N == q (element logs, a subset of the stream's positions): the
//     fused engine in codes-only mode.
//  2. Union by stream position.  Rank q owns commands [a_q, a_{q+1}); every
//     rank sends the codes of its positions to their range's owner (one
//     all-to-all, 4 B per element), which unions each command's S codes
//     (QuorumDeps + MShardCommit).
//  3. Local SCCs.  The range's graph without its cross-range edges goes
//     through GraphCore's global path: SCCs, ready times H (max position
//     reachable) and depths.  A vertex that reaches no cross-range edge
//     ("settled") has its global SCC, H and depth already.  Escaping
//     vertices (those that do) are contracted to their local SCCs.
//  4. Condensed graph.  Local SCCs of escaping vertices become super vertices
//     keyed by their largest position; an edge to a settled vertex w becomes
//     an edge to a marker vertex keyed H(w) (the largest position w reaches,
//     never an escaping one); cross-range edges are resolved by their owner
//     (an all-to-all of queries and answers).  Every rank gathers all parts
//     (all-gather) and solves the small condensed graph with GraphCore: the
//     escaping vertices' SCCs, ready times and depths.  Markers sort by key
//     with the super vertices, so the condensed ready time (a vid) maps back
//     to a stream position monotonically.
//  5. Order.  A settled SCC never reaches an escaping one, so within a ready
//     group all settled SCCs can run before the escaping ones: the order key
//     is (H, escaping, depth), members of an SCC in dot order.  Same-key
//     commands are always connected by a dependency path, so every key's
//     sequence is fixed by this key (SURVEY §8a parity).  Each (key, command)
//     element goes to its key's owner (all-to-all) and is sorted there.
//
// Exchanges are the caller's (torch.distributed over RCCL): every entry
// point takes and fills device buffers and returns with its stream idle.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "engine_internal.h"
#include "graph_core.h"
#include "scan.h"
#include "sort.h"

namespace fh {
namespace {

constexpr unsigned B = 256;
#define GRID_STRIDE(i, n) \
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += gridDim.x * blockDim.x)

constexpr uint32_t kMarker = 0x80000000u;  // condensed edge target: a marker (ready time)

// codes of this rank's positions in send order (log references into the one
// staged batch become vid + 1: the engine's command log starts at 0)
__global__ void k_gather_codes(uint32_t m, const uint32_t *__restrict__ pos,
                               const uint32_t *__restrict__ codes, uint32_t *__restrict__ out) {
  GRID_STRIDE(i, m) {
    const uint32_t c = codes[pos[i]];
    out[i] = (c & 0x80000000u) ? (c & 0x7FFFFFFFu) + 1u : c;
  }
}

__global__ void k_scatter_codes(uint32_t m, const uint32_t *__restrict__ pos,
                                const uint32_t *__restrict__ in, uint32_t *__restrict__ codes) {
  GRID_STRIDE(i, m) codes[pos[i]] = in[i];
}

// edges of range vertex v (global vids in dst[v*S ..), ecnt[v] of them):
// local ones (as local vids) and cross-range ones
__global__ void k_edge_split_count(uint32_t V, uint32_t S, uint32_t a, const uint32_t *__restrict__ dst,
                                   const uint32_t *__restrict__ ecnt, uint32_t *__restrict__ nloc,
                                   uint32_t *__restrict__ ncross) {
  GRID_STRIDE(v, V) {
    uint32_t l = 0, c = 0;
    for (uint32_t e = 0; e < ecnt[v]; e++) {
      const uint32_t w = dst[size_t(v) * S + e];
      if (w - a < V)
        l++;
      else
        c++;
    }
    nloc[v] = l;
    ncross[v] = c;
  }
}

__global__ void k_edge_split_fill(uint32_t V, uint32_t S, uint32_t a, const uint32_t *__restrict__ dst,
                                  const uint32_t *__restrict__ ecnt, const uint32_t *__restrict__ loff,
                                  const uint32_t *__restrict__ coff, uint32_t *__restrict__ ldst,
                                  uint32_t *__restrict__ csrc, uint32_t *__restrict__ cdst) {
  GRID_STRIDE(v, V) {
    uint32_t l = loff[v], c = coff[v];
    for (uint32_t e = 0; e < ecnt[v]; e++) {
      const uint32_t w = dst[size_t(v) * S + e];
      if (w - a < V) {
        ldst[l++] = w - a;
      } else {
        csrc[c] = v;
        cdst[c++] = w;
      }
    }
  }
}

// escaping: the local SCC of a vertex with a cross-range edge, and every
// vertex reaching one (flags by representative)
__global__ void k_esc_init(uint32_t V, const uint32_t *__restrict__ coff,
                           const uint32_t *__restrict__ rep, uint8_t *__restrict__ esc) {
  GRID_STRIDE(v, V) if (coff[v + 1] != coff[v]) esc[rep[v]] = 1;
}

__global__ void k_esc_iter(uint32_t V, const uint32_t *__restrict__ off,
                           const uint32_t *__restrict__ dst, const uint32_t *__restrict__ rep,
                           uint8_t *esc, uint32_t *changed) {
  GRID_STRIDE(v, V) {
    const uint32_t r = rep[v];
    if (__hip_atomic_load(&esc[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) continue;
    for (uint32_t e = off[v]; e < off[v + 1]; e++) {
      if (__hip_atomic_load(&esc[rep[dst[e]]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(&esc[r], uint8_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *changed = 1;
        break;
      }
    }
  }
}

// super vertex keys: the largest position of each escaping local SCC
__global__ void k_maxpos(uint32_t V, uint32_t a, const uint32_t *__restrict__ rep,
                         const uint8_t *__restrict__ esc, uint32_t *__restrict__ mx) {
  GRID_STRIDE(v, V) {
    const uint32_t r = rep[v];
    if (esc[r]) atomicMax(&mx[r], a + v);
  }
}

// condensed records of escaping vertex v: local edges (to another escaping
// local SCC, or to a settled vertex's ready time), cross edges -> queries
__global__ void k_cond_count(uint32_t V, const uint32_t *__restrict__ off,
                             const uint32_t *__restrict__ dst, const uint32_t *__restrict__ rep,
                             const uint8_t *__restrict__ esc, uint32_t *__restrict__ cnt) {
  GRID_STRIDE(v, V) {
    const uint32_t r = rep[v];
    uint32_t c = 0;
    if (esc[r])
      for (uint32_t e = off[v]; e < off[v + 1]; e++) {
        const uint32_t rw = rep[dst[e]];
        c += (!esc[rw] || rw != r) ? 1u : 0u;
      }
    cnt[v] = c;
  }
}

__global__ void k_cond_fill(uint32_t V, uint32_t a, const uint32_t *__restrict__ off,
                            const uint32_t *__restrict__ dst, const uint32_t *__restrict__ rep,
                            const uint8_t *__restrict__ esc, const uint64_t *__restrict__ kap,
                            const uint32_t *__restrict__ roff, uint64_t *__restrict__ rec) {
  GRID_STRIDE(v, V) {
    const uint32_t r = rep[v];
    if (!esc[r]) continue;
    const uint64_t sv = uint64_t(a + r) << 32;
    uint32_t o = roff[v];
    for (uint32_t e = off[v]; e < off[v + 1]; e++) {
      const uint32_t rw = rep[dst[e]];
      if (esc[rw]) {
        if (rw != r) rec[o++] = sv | (a + rw);
      } else {
        rec[o++] = sv | kMarker | (a + uint32_t(kap[rw] >> 32));
      }
    }
  }
}

// an owner's answer for queried vertex g of its range
__global__ void k_answer(uint32_t m, uint32_t a, const uint32_t *__restrict__ q,
                         const uint32_t *__restrict__ rep, const uint8_t *__restrict__ esc,
                         const uint64_t *__restrict__ kap, uint32_t *__restrict__ ans) {
  GRID_STRIDE(i, m) {
    const uint32_t r = rep[q[i] - a];
    ans[i] = esc[r] ? (a + r) : (kMarker | (a + uint32_t(kap[r] >> 32)));
  }
}

template <class T>
__device__ __forceinline__ uint32_t lower_bound_dev(const T *__restrict__ a, uint32_t n, T x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// cross edges (escaping sources only) -> records with the owners' answers
__global__ void k_cross_records(uint32_t m, uint32_t a, const uint32_t *__restrict__ csrc,
                                const uint32_t *__restrict__ cdst, const uint32_t *__restrict__ rep,
                                const uint32_t *__restrict__ qs, uint32_t nq,
                                const uint32_t *__restrict__ ans, uint64_t *__restrict__ rec) {
  GRID_STRIDE(i, m) {
    const uint32_t r = rep[csrc[i]];  // escaping: it has a cross edge
    rec[i] = (uint64_t(a + r) << 32) | ans[lower_bound_dev(qs, nq, cdst[i])];
  }
}

// The condensed edge records of this rank, sorted (src << 32 | target, a
// marker target carrying kMarker | H): keep the first of each run of equal
// records, and of a source's marker targets only the largest H.  Markers are
// sinks keyed by ready time (a settled vertex never reaches an escaping
// one), so a super vertex's ready time takes only their maximum, and its
// depth counts only successors of its own ready group, which among markers
// is at most the one with the largest H: the dropped edges change no output.
// (A super vertex standing for a large local SCC otherwise carries one edge
// per distinct settled ready time it reaches, which one thread of the solve
// walks on every propagation launch.)
__global__ void k_cond_flags(uint32_t m, const uint64_t *__restrict__ x, uint32_t *__restrict__ fl) {
  GRID_STRIDE(i, m) {
    const uint64_t v = x[i];
    bool keep;
    if (uint32_t(v) & kMarker)
      keep = i + 1 == m || (x[i + 1] >> 32) != (v >> 32);
    else
      keep = i == 0 || x[i - 1] != v;
    fl[i] = keep ? 1u : 0u;
  }
}

// sorted u64 / u32 arrays: keep the first of each run
template <class T>
__global__ void k_first_flags(uint32_t m, const T *__restrict__ x, uint32_t *__restrict__ fl) {
  GRID_STRIDE(i, m) fl[i] = (i == 0 || x[i] != x[i - 1]) ? 1u : 0u;
}
template <class T>
__global__ void k_compact_by(uint32_t m, const T *__restrict__ x, const uint32_t *__restrict__ fl,
                             const uint32_t *__restrict__ pos, T *__restrict__ out) {
  GRID_STRIDE(i, m) if (fl[i]) out[pos[i]] = x[i];
}

// this rank's super vertices: (sid << 32 | maxpos, label)
__global__ void k_super_flags(uint32_t V, const uint32_t *__restrict__ rep,
                              const uint8_t *__restrict__ esc, uint32_t *__restrict__ fl) {
  GRID_STRIDE(v, V) fl[v] = (rep[v] == v && esc[v]) ? 1u : 0u;
}
__global__ void k_super_fill(uint32_t V, uint32_t a, const uint32_t *__restrict__ fl,
                             const uint32_t *__restrict__ pos, const uint32_t *__restrict__ mx,
                             const uint64_t *__restrict__ label, uint64_t *__restrict__ out) {
  GRID_STRIDE(v, V) {
    if (!fl[v]) continue;
    out[2 * size_t(pos[v])] = (uint64_t(a + v) << 32) | mx[v];
    out[2 * size_t(pos[v]) + 1] = label[v];
  }
}

// ---- condensed solve ------------------------------------------------------
// vertex keys: super vertices (maxpos << 1), markers (H << 1 | 1)
__global__ void k_ckeys_super(uint32_t nv, const uint64_t *__restrict__ verts,
                              uint64_t *__restrict__ keys, uint32_t *__restrict__ sid) {
  GRID_STRIDE(i, nv) {
    keys[i] = uint64_t(uint32_t(verts[2 * size_t(i)])) << 1;
    sid[i] = uint32_t(verts[2 * size_t(i)] >> 32);
  }
}
// (non-marker edges get `fill`, above every key: the sort then needs only
// the keys' bits, not 64)
__global__ void k_ckeys_marker(uint32_t ne, const uint64_t *__restrict__ edges,
                               uint64_t *__restrict__ keys, uint64_t fill) {
  GRID_STRIDE(i, ne) {
    const uint32_t t = uint32_t(edges[i]);
    keys[i] = (t & kMarker) ? ((uint64_t(t & ~kMarker) << 1) | 1u) : fill;
  }
}
// super vertex i (in sid order) -> its condensed vid
__global__ void k_sid_vid(uint32_t nv, const uint64_t *__restrict__ verts,
                          const uint32_t *__restrict__ idx, const uint64_t *__restrict__ ck,
                          uint32_t ncv, uint32_t *__restrict__ vid, uint64_t *__restrict__ cdot,
                          const uint32_t *__restrict__ sid_sorted, uint32_t *__restrict__ sid_out) {
  GRID_STRIDE(i, nv) {
    const uint32_t j = idx[i];
    const uint64_t k = uint64_t(uint32_t(verts[2 * size_t(j)])) << 1;
    const uint32_t x = lower_bound_dev(ck, ncv, k);
    vid[i] = x;
    cdot[x] = verts[2 * size_t(j) + 1];
    sid_out[i] = sid_sorted[i];
  }
}
__global__ void k_fill_u64(uint32_t n, uint64_t *p, uint64_t v) { GRID_STRIDE(i, n) p[i] = v; }

// ---- hub split of the condensed graph ---------------------------------------
// A super vertex standing for a large local SCC can carry tens of thousands of
// distinct out-edges (C5 at 8 ranges: up to 22.7K), which one thread of the
// global path walks on every propagation launch.  Each such vertex x becomes
// a group of ids base(x) .. base(x) + nax(x) holding kHubDeg of its edges each,
// x itself last (the group's maximum id, so the class maximum -- the ready
// time -- stays x), the others auxiliary with the largest dot (no label);
// GraphInput::rep0 makes every group one class from the start, and the global
// path works on classes: ready times, depths and the coloring see the
// group's edges as x's.
constexpr uint32_t kHubDeg = 256;  // FH_DGRAPH_HUB (a test switch) overrides
__global__ void k_hub_aux(uint32_t ncv, uint32_t D, const uint32_t *__restrict__ cnt,
                          uint32_t *__restrict__ nax) {
  GRID_STRIDE(x, ncv) {
    const uint32_t d = cnt[x];
    nax[x] = d > D ? (d - 1) / D : 0u;
  }
}
__global__ void k_hub_layout(uint32_t ncv, uint32_t D, const uint32_t *__restrict__ cnt,
                             const uint32_t *__restrict__ nax, const uint32_t *__restrict__ aoff,
                             const uint64_t *__restrict__ cd, const uint64_t *__restrict__ ck,
                             uint32_t *__restrict__ cnt2, uint64_t *__restrict__ cd2,
                             uint64_t *__restrict__ ck2, uint32_t *__restrict__ rep0,
                             uint32_t *__restrict__ vmap) {
  GRID_STRIDE(x, ncv) {
    const uint32_t b = x + aoff[x], na = nax[x], d = cnt[x];
    for (uint32_t j = 0; j <= na; j++) {
      cnt2[b + j] = min(D, d - j * D);
      cd2[b + j] = j == na ? cd[x] : ~0ull;
      ck2[b + j] = ck[x];
      rep0[b + j] = b;
    }
    vmap[x] = b + na;
  }
}
// edges (sorted by source: co[x] = x's first) -> the split CSR, targets mapped
__global__ void k_hub_edges(uint32_t nce, uint32_t D, const uint64_t *__restrict__ eds, int cb,
                            const uint32_t *__restrict__ co, const uint32_t *__restrict__ aoff,
                            const uint32_t *__restrict__ off2, const uint32_t *__restrict__ vmap,
                            uint32_t *__restrict__ dst2) {
  GRID_STRIDE(e, nce) {
    const uint32_t x = uint32_t(eds[e] >> cb);
    const uint32_t d = uint32_t(eds[e] & ((uint64_t(1) << cb) - 1));
    const uint32_t k = e - co[x];
    dst2[off2[x + aoff[x] + k / D] + k % D] = vmap[d];
  }
}
__global__ void k_map_u32(uint32_t n, uint32_t *__restrict__ x, const uint32_t *__restrict__ m) {
  GRID_STRIDE(i, n) x[i] = m[x[i]];
}
__global__ void k_cedges(uint32_t ne, const uint64_t *__restrict__ edges,
                         const uint32_t *__restrict__ sids, const uint32_t *__restrict__ vid,
                         uint32_t nv, const uint64_t *__restrict__ ck, uint32_t ncv, int cb,
                         uint64_t *__restrict__ out) {
  GRID_STRIDE(i, ne) {
    const uint64_t e = edges[i];
    const uint32_t s = vid[lower_bound_dev(sids, nv, uint32_t(e >> 32))];
    const uint32_t t = uint32_t(e);
    const uint32_t d = (t & kMarker) ? lower_bound_dev(ck, ncv, (uint64_t(t & ~kMarker) << 1) | 1u)
                                     : vid[lower_bound_dev(sids, nv, t)];
    out[i] = (uint64_t(s) << cb) | d;
  }
}
__global__ void k_csr_counts(uint32_t ne, const uint64_t *__restrict__ e, int cb,
                             uint32_t *__restrict__ cnt) {
  GRID_STRIDE(i, ne) atomicAdd(&cnt[uint32_t(e[i] >> cb)], 1u);
}
__global__ void k_csr_dst(uint32_t ne, const uint64_t *__restrict__ e, int cb,
                          uint32_t *__restrict__ dst) {
  GRID_STRIDE(i, ne) dst[i] = uint32_t(e[i] & ((uint64_t(1) << cb) - 1));
}

// ---- expansion and per-key elements ----------------------------------------
// order key per range vertex: (H << 32) | escaping << 31 | depth; label
__global__ void k_expand(uint32_t V, uint32_t a, const uint32_t *__restrict__ rep,
                         const uint8_t *__restrict__ esc, const uint64_t *__restrict__ kap,
                         const uint64_t *__restrict__ lab, const uint32_t *__restrict__ sids,
                         const uint32_t *__restrict__ vid, uint32_t nv,
                         const uint32_t *__restrict__ crep, const uint64_t *__restrict__ ckap,
                         const uint64_t *__restrict__ clab, const uint64_t *__restrict__ ck,
                         uint64_t *__restrict__ okey, uint64_t *__restrict__ label,
                         uint32_t *__restrict__ err) {
  GRID_STRIDE(v, V) {
    const uint32_t r = rep[v];
    uint64_t h, d, l;
    if (esc[r]) {
      const uint32_t x = vid[lower_bound_dev(sids, nv, a + r)];
      const uint64_t kp = ckap[crep[x]];
      h = ck[uint32_t(kp >> 32)] >> 1;
      d = uint32_t(kp) | 0x80000000u;
      l = clab[x];
      if (uint32_t(kp) >= 0x80000000u) atomicOr(err, 1u);
    } else {
      const uint64_t kp = kap[r];
      h = a + uint32_t(kp >> 32);
      d = uint32_t(kp);
      l = lab[v];
      if (uint32_t(kp) >= 0x80000000u) atomicOr(err, 1u);
    }
    okey[v] = (h << 32) | d;
    label[v] = l;
  }
}

// elements (key, order) of range vertex v's k keys, by the key's owner:
// e0 = key << hb | H, e1 = (escaping << 31 | depth) << 32 | dot32
struct ElemPack {
  uint32_t k, hb, shards, world, seqb;
  __device__ __forceinline__ uint32_t owner(uint32_t key) const { return (key % shards) % world; }
};
constexpr int kMaxWorld = 64;
__global__ void __launch_bounds__(B)
    k_elem_route(uint32_t V, uint32_t a, ElemPack ep, const uint32_t *__restrict__ key32,
                 const uint64_t *__restrict__ dot, const uint64_t *__restrict__ okey,
                 uint32_t *__restrict__ cursor, const uint32_t *__restrict__ base,
                 uint64_t *__restrict__ out, int fill) {
  __shared__ uint32_t s_c[kMaxWorld], s_b[kMaxWorld];
  if (threadIdx.x < ep.world) s_c[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t v = blockIdx.x * B + threadIdx.x;
  uint32_t rk[8], ow[8];
  if (v < V) {
    for (uint32_t s = 0; s < ep.k; s++) {
      ow[s] = ep.owner(key32[size_t(a + v) * ep.k + s]);
      rk[s] = atomicAdd(&s_c[ow[s]], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < ep.world)
    s_b[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], s_c[threadIdx.x]);
  __syncthreads();
  if (!fill || v >= V) return;
  const uint64_t ok = okey[v], d = dot[a + v];
  const uint64_t d32 = ((d >> 56) << ep.seqb) | (d & 0x00FFFFFFFFFFFFFFull);
  for (uint32_t s = 0; s < ep.k; s++) {
    const uint64_t o = base[ow[s]] + s_b[ow[s]] + rk[s];
    const uint32_t key = key32[size_t(a + v) * ep.k + s];
    out[2 * o] = (uint64_t(key) << ep.hb) | (ok >> 32);
    out[2 * o + 1] = (ok << 32) | d32;
  }
}

__global__ void k_split_elems(uint32_t m, const uint64_t *__restrict__ el, uint64_t *__restrict__ e0,
                              uint64_t *__restrict__ e1) {
  GRID_STRIDE(i, m) {
    e0[i] = el[2 * size_t(i)];
    e1[i] = el[2 * size_t(i) + 1];
  }
}
__global__ void k_gather_u64(uint32_t m, const uint32_t *__restrict__ idx,
                             const uint64_t *__restrict__ in, uint64_t *__restrict__ out) {
  GRID_STRIDE(i, m) out[i] = in[idx[i]];
}
__global__ void k_unpack_elems(uint32_t m, const uint32_t *__restrict__ idx,
                               const uint64_t *__restrict__ e0, const uint64_t *__restrict__ e1,
                               uint32_t hb, uint32_t seqb, uint32_t *__restrict__ key,
                               uint64_t *__restrict__ dot) {
  GRID_STRIDE(i, m) {
    key[i] = uint32_t(e0[i] >> hb);
    const uint32_t d32 = uint32_t(e1[idx[i]]);
    dot[i] = (uint64_t(d32 >> seqb) << 56) | (d32 & ((1u << seqb) - 1u));
  }
}

}  // namespace

struct DistGraph {
  int device = 0;
  uint32_t rank = 0, world = 1, shards = 1;
  fh_config cfg{};
  EngineDevice *eng = nullptr;
  hipStream_t stream = nullptr;
  uint64_t n = 0;     // commands in the stream
  uint32_t k = 0, S = 0, K = 0, hb = 0, seqb = 0;
  std::vector<uint64_t> bound;  // range starts [world + 1]
  uint32_t a = 0, V = 0;        // this rank's range
  // staged
  DBuf<uint64_t> dot;       // [n] the stream's dots
  DBuf<uint32_t> key32;     // [n * k]
  DBuf<uint32_t> send_pos;  // this rank's positions, ascending (= send order)
  DBuf<uint32_t> recv_pos;  // range positions by source rank, range-local
  std::vector<uint64_t> send_cnt, recv_cnt;
  size_t nsend = 0, nrecv = 0;
  // per step
  DBuf<uint32_t> codes, dcnt, dep_off, dst, ecnt, nloc, ncross, loff, coff, ldst, csrc, cdst, scal;
  DBuf<uint64_t> dep_dot;
  DBuf<uint8_t> esc;
  DBuf<uint32_t> mx, tmp_a, tmp_b, tmp_c, tmp_d, queries;
  DBuf<uint64_t> rec_a, rec_b, verts, okey, label;
  uint32_t nq = 0, ncross_e = 0;
  std::vector<uint64_t> q_cnt;
  uint64_t *lkap = nullptr;  // local GraphCore's kap (by rep)
  const uint32_t *lrep = nullptr;
  const uint64_t *llab = nullptr;
  uint32_t nrec = 0, nsuper = 0;
  uint64_t *cond_edges = nullptr;
  // condensed solve
  DBuf<uint64_t> ck, ck2, ce, ce2, cdot;
  DBuf<uint32_t> csid, cvid, cidx, cidx2, coffs, cdst2, ccnt;
  DBuf<uint32_t> hub_nax, hub_aoff, hub_cnt, hub_off, hub_rep0, hub_vmap, hub_dst;
  const uint32_t hub_deg = [] {
    const char *e = getenv("FH_DGRAPH_HUB");
    return e && atoi(e) > 0 ? uint32_t(atoi(e)) : kHubDeg;
  }();
  DBuf<uint64_t> hub_dot, hub_ck;
  // elements
  std::vector<uint64_t> el_cnt;
  DBuf<uint32_t> el_cursor, el_base;
  DBuf<uint64_t> e0a, e0b, e1a, e1b;
  DBuf<uint32_t> ia, ib, pk_key;
  DBuf<uint64_t> pk_dot;
  uint32_t n_pk = 0;
  SortWorkspace sort_ws;
  ScanWorkspace scan_ws;
  GraphCore local, cond;
  GraphOutput lout, cout_;
  // timing (profiling: per-stage device ms)
  bool profile = false;
  std::vector<std::pair<std::string, float>> times;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;

  DistGraph(const fh_config &c, uint32_t r, uint32_t w) : rank(r), world(w), cfg(c) {
    FH_CHECK(w >= 1 && w <= uint32_t(kMaxWorld) && r < w, FH_EINVAL, "dgraph: rank < world <= 64");
    eng = engine_new(c);
    stream = engine_stream(eng);
    FH_HIP(hipGetDevice(&device));
    local.stream = stream;
    cond.stream = stream;
    FH_HIP(hipEventCreate(&ev0));
    FH_HIP(hipEventCreate(&ev1));
  }
  ~DistGraph() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    engine_free(eng);
  }

  void sync() { FH_HIP(hipStreamSynchronize(stream)); }
  void t_begin() {
    if (profile) FH_HIP(hipEventRecord(ev0, stream));
  }
  void t_end(const char *name) {
    if (!profile) return;
    FH_HIP(hipEventRecord(ev1, stream));
    FH_HIP(hipEventSynchronize(ev1));
    float ms = 0;
    FH_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    times.push_back({name, ms});
  }

  uint32_t scan_total(const uint32_t *in, uint32_t *out, uint32_t m) {
    exclusive_scan_u32(in, out, m, scan_ws, stream);
    return fetch_u32(out + m, stream);
  }

  // sorted-unique of m u64 keys in place in (x, spare) -> returns the count;
  // *res = the buffer holding the result
  uint32_t sort_unique_u64(DBuf<uint64_t> &x, DBuf<uint64_t> &spare, uint32_t m, int bits,
                           uint64_t **res, bool cond_records = false) {
    if (m == 0) {
      *res = x.get();
      return 0;
    }
    uint32_t *va = tmp_a.ensure(m + 1), *vb = tmp_b.ensure(m + 1);
    uint64_t *ks = nullptr;
    uint32_t *vs = nullptr;
    spare.ensure(m + 1);
    sort_pairs<uint64_t, uint32_t>(x.get(), nullptr, x.get(), va, spare.get(), vb, m, bits, sort_ws,
                                   stream, &ks, &vs);
    uint64_t *other = ks == x.get() ? spare.get() : x.get();
    uint32_t *fl = tmp_c.ensure(m + 1), *ps = tmp_d.ensure(m + 1);
    if (cond_records)
      k_cond_flags<<<grid_for(m, B), B, 0, stream>>>(m, ks, fl);
    else
      k_first_flags<uint64_t><<<grid_for(m, B), B, 0, stream>>>(m, ks, fl);
    const uint32_t u = scan_total(fl, ps, m);
    k_compact_by<uint64_t><<<grid_for(m, B), B, 0, stream>>>(m, ks, fl, ps, other);
    *res = other;
    return u;
  }

  // ---- staging ---------------------------------------------------------------
  void stage(const fh_stream_desc &d, uint32_t nshards, const uint64_t *h_dot,
             const uint64_t *h_key, const uint64_t *h_off, const uint32_t *h_ent) {
    FH_CHECK(h_dot && h_key && h_off && h_ent, FH_EINVAL, "null argument");
    FH_CHECK(d.views >= 1 && (d.flags & FH_STREAM_ELEMENT_LOGS), FH_EINVAL,
             "dgraph: element logs with replica views");
    FH_CHECK(nshards >= 1 && nshards <= 255, FH_EINVAL, "dgraph: shards in [1, 255]");
    shards = nshards;
    n = d.n;
    k = d.keys_per_cmd;
    S = k * d.views;
    FH_CHECK(S <= 16, FH_ENOTIMPL, "dgraph: at most 16 key slots x views per command");
    FH_CHECK(n * S < (uint64_t(1) << 31) && n >= world, FH_EINVAL, "dgraph: stream size");
    K = uint32_t(cfg.key_space);
    hb = uint32_t(bits_for(n + 1));
    FH_CHECK(uint32_t(bits_for(cfg.key_space)) + hb <= 64, FH_ENOTIMPL, "dgraph: key + position bits");
    uint64_t mseq = 0;
    for (uint64_t i = 0; i < n; i++) mseq = std::max<uint64_t>(mseq, h_dot[i] & 0x00FFFFFFFFFFFFFFull);
    seqb = uint32_t(bits_for(mseq + 1));
    FH_CHECK(seqb <= 24, FH_ENOTIMPL, "dgraph: dot sequences must fit 24 bits");
    bound.resize(world + 1);
    for (uint32_t q = 0; q <= world; q++) bound[q] = n * q / world;
    a = uint32_t(bound[rank]);
    V = uint32_t(bound[rank + 1] - bound[rank]);
    // KeyDeps of this rank's processes (subset element logs)
    engine_stage_subset(eng, d, h_dot, h_key, h_off, h_ent);
    FH_HIP(hipSetDevice(device));
    // send plan: this rank's positions ascending (grouped by destination range)
    const uint32_t np = d.nproc;
    std::vector<uint32_t> mine(h_ent, h_ent + h_off[np]);
    std::sort(mine.begin(), mine.end());
    nsend = mine.size();
    send_cnt.assign(world, 0);
    for (uint32_t p : mine) {
      const uint64_t c = p / S;
      send_cnt[std::upper_bound(bound.begin(), bound.end(), c) - bound.begin() - 1]++;
    }
    FH_HIP(hipMemcpyAsync(send_pos.ensure(nsend + 1), mine.data(), nsend * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    // receive plan: the range's positions of each source's shards, ascending
    recv_cnt.assign(world, 0);
    std::vector<std::vector<uint32_t>> by_src(world);
    for (uint64_t c = a; c < uint64_t(a) + V; c++)
      for (uint32_t s = 0; s < k; s++) {
        const uint32_t src = uint32_t((h_key[c * k + s] % shards) % world);
        for (uint32_t j = 0; j < d.views; j++)
          by_src[src].push_back(uint32_t((((c - a) * d.views + j) * k) + s));
      }
    std::vector<uint32_t> rp;
    rp.reserve(size_t(V) * S);
    for (uint32_t q = 0; q < world; q++) {
      std::sort(by_src[q].begin(), by_src[q].end());
      recv_cnt[q] = by_src[q].size();
      rp.insert(rp.end(), by_src[q].begin(), by_src[q].end());
    }
    nrecv = rp.size();
    FH_CHECK(nrecv == size_t(V) * S, FH_EINVARIANT, "dgraph: receive plan");
    FH_HIP(hipMemcpyAsync(recv_pos.ensure(nrecv + 1), rp.data(), nrecv * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    FH_HIP(hipMemcpyAsync(dot.ensure(n + 1), h_dot, n * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
    std::vector<uint32_t> k32(n * k);
    for (size_t i = 0; i < n * k; i++) {
      FH_CHECK(h_key[i] < cfg.key_space, FH_EINVAL, "dgraph: key id >= key_space");
      k32[i] = uint32_t(h_key[i]);
    }
    FH_HIP(hipMemcpyAsync(key32.ensure(n * k + 1), k32.data(), n * k * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    sync();
  }

  // ---- 1. KeyDeps ----------------------------------------------------------------
  void keydeps(uint32_t *send) {
    times.clear();
    engine_set_profiling(eng, false);
    t_begin();
    const uint32_t *c = engine_run_codes(eng, nullptr);
    if (nsend)
      k_gather_codes<<<grid_for(nsend, B), B, 0, stream>>>(uint32_t(nsend), send_pos.get(), c, send);
    sync();
    t_end("keydeps");
  }

  // ---- 2-3. union + local SCCs + escaping + queries -------------------------------
  void local_stage(const uint32_t *recv) {
    t_begin();
    uint32_t *cd = codes.ensure(size_t(V) * S + 1);
    k_scatter_codes<<<grid_for(nrecv, B), B, 0, stream>>>(uint32_t(nrecv), recv_pos.get(), recv, cd);
    // union: committed deps of the range (dot CSR) + edges
    union_rows(V, S, cd, dot.get(), a, dcnt.ensure(V + 1), dep_off.ensure(V + 1),
               dep_dot.ensure(size_t(V) * S + 1), dst.ensure(size_t(V) * S + 1), ecnt.ensure(V + 1),
               scal.ensure(4), scan_ws, stream);
    t_end("union");
    t_begin();
    // local / cross edges
    k_edge_split_count<<<grid_for(V, B), B, 0, stream>>>(V, S, a, dst.get(), ecnt.get(),
                                                          nloc.ensure(V + 1), ncross.ensure(V + 1));
    const uint32_t nl = scan_total(nloc.get(), loff.ensure(V + 1), V);
    ncross_e = scan_total(ncross.get(), coff.ensure(V + 1), V);
    k_edge_split_fill<<<grid_for(V, B), B, 0, stream>>>(
        V, S, a, dst.get(), ecnt.get(), loff.get(), coff.get(), ldst.ensure(nl + 1),
        csrc.ensure(ncross_e + 1), cdst.ensure(ncross_e + 1));
    // local SCCs, ready times, depths (GraphCore's global path)
    GraphInput gin;
    gin.V = V;
    gin.off = loff.get();
    gin.dst = ldst.get();
    gin.dot = dot.get() + a;
    gin.global_only = true;
    gin.want_orders = false;
    gin.want_per_key = false;
    local.run(gin, lout);
    lrep = lout.rep;
    lkap = lout.kap;
    llab = lout.scc_label;
    FH_CHECK(lrep && lkap && llab, FH_EINVARIANT, "dgraph: local graph outputs");
    t_end("local_scc");
    t_begin();
    // escaping local SCCs
    uint8_t *es = esc.ensure(V + 1);
    FH_HIP(hipMemsetAsync(es, 0, V, stream));
    k_esc_init<<<grid_for(V, B), B, 0, stream>>>(V, coff.get(), lrep, es);
    uint32_t *ch = scal.get() + 2;
    for (int it = 0;; it++) {
      FH_HIP(hipMemsetAsync(ch, 0, sizeof(uint32_t), stream));
      k_esc_iter<<<grid_for(V, B), B, 0, stream>>>(V, loff.get(), ldst.get(), lrep, es, ch);
      if (!fetch_u32(ch, stream)) break;
    }
    // queries: the cross edges' targets, sorted unique (grouped by owner)
    uint32_t *qa = queries.ensure(ncross_e + 1);
    nq = 0;
    if (ncross_e) {
      uint32_t *va = tmp_a.ensure(ncross_e + 1), *kb = tmp_b.ensure(ncross_e + 1),
               *vb = tmp_c.ensure(ncross_e + 1);
      uint32_t *ks = nullptr, *vs = nullptr;
      sort_pairs<uint32_t, uint32_t>(cdst.get(), nullptr, qa, va, kb, vb, ncross_e, bits_for(n + 1),
                                     sort_ws, stream, &ks, &vs);
      uint32_t *fl = tmp_d.ensure(ncross_e + 1), *ps = mx.ensure(ncross_e + 1);
      k_first_flags<uint32_t><<<grid_for(ncross_e, B), B, 0, stream>>>(ncross_e, ks, fl);
      nq = scan_total(fl, ps, ncross_e);
      uint32_t *out = ks == qa ? kb : qa;
      k_compact_by<uint32_t><<<grid_for(ncross_e, B), B, 0, stream>>>(ncross_e, ks, fl, ps, out);
      if (out != qa) FH_HIP(hipMemcpyAsync(qa, out, nq * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream));
    }
    std::vector<uint32_t> hq(nq);
    if (nq) FH_HIP(hipMemcpyAsync(hq.data(), qa, nq * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    sync();
    q_cnt.assign(world, 0);
    for (uint32_t g : hq) q_cnt[std::upper_bound(bound.begin(), bound.end(), uint64_t(g)) - bound.begin() - 1]++;
    FH_CHECK(q_cnt[rank] == 0, FH_EINVARIANT, "dgraph: a cross edge into the own range");
    t_end("escaping");
  }

  void answer(uint32_t m, const uint32_t *q, uint32_t *ans) {
    if (m) k_answer<<<grid_for(m, B), B, 0, stream>>>(m, a, q, lrep, esc.get(), lkap, ans);
    sync();
  }

  // ---- 4. this rank's part of the condensed graph ---------------------------------
  void condense(const uint32_t *ans, uint64_t *nv, uint64_t *ne) {
    t_begin();
    uint32_t *cnt = nloc.get();  // reuse: per-vertex record counts
    k_cond_count<<<grid_for(V, B), B, 0, stream>>>(V, loff.get(), ldst.get(), lrep, esc.get(), cnt);
    uint32_t *ro = ncross.get();
    const uint32_t nl = scan_total(cnt, ro, V);
    const uint32_t tot = nl + ncross_e;
    uint64_t *ra = rec_a.ensure(tot + 1);
    k_cond_fill<<<grid_for(V, B), B, 0, stream>>>(V, a, loff.get(), ldst.get(), lrep, esc.get(),
                                                   lkap, ro, ra);
    if (ncross_e)
      k_cross_records<<<grid_for(ncross_e, B), B, 0, stream>>>(ncross_e, a, csrc.get(), cdst.get(),
                                                                lrep, queries.get(), nq, ans,
                                                                ra + nl);
    nrec = sort_unique_u64(rec_a, rec_b, tot, 64, &cond_edges, true);
    // super vertices
    uint32_t *m = mx.ensure(V + 1);
    FH_HIP(hipMemsetAsync(m, 0, size_t(V) * sizeof(uint32_t), stream));
    k_maxpos<<<grid_for(V, B), B, 0, stream>>>(V, a, lrep, esc.get(), m);
    uint32_t *fl = tmp_c.ensure(V + 1), *ps = tmp_d.ensure(V + 1);
    k_super_flags<<<grid_for(V, B), B, 0, stream>>>(V, lrep, esc.get(), fl);
    nsuper = scan_total(fl, ps, V);
    k_super_fill<<<grid_for(V, B), B, 0, stream>>>(V, a, fl, ps, m, llab, verts.ensure(2 * size_t(nsuper) + 2));
    sync();
    *nv = nsuper;
    *ne = nrec;
    t_end("condense");
  }

  void condensed_part(uint64_t *vout, uint64_t *eout) {
    if (nsuper)
      FH_HIP(hipMemcpyAsync(vout, verts.get(), 2 * size_t(nsuper) * sizeof(uint64_t),
                            hipMemcpyDeviceToDevice, stream));
    if (nrec)
      FH_HIP(hipMemcpyAsync(eout, cond_edges, size_t(nrec) * sizeof(uint64_t),
                            hipMemcpyDeviceToDevice, stream));
    sync();
  }

  // ---- 5. condensed solve, expansion, per-key elements ----------------------------
  void solve(uint32_t nv, const uint64_t *vg, uint32_t ne, const uint64_t *eg, uint64_t *counts) {
    t_begin();
    // condensed vertices: super vertices and markers, sorted by key
    uint64_t *kk = ck.ensure(size_t(nv) + ne + 1);
    uint32_t *sid = csid.ensure(nv + 1);
    if (nv) k_ckeys_super<<<grid_for(nv, B), B, 0, stream>>>(nv, vg, kk, sid);
    // keys: positions (< n) << 1 | marker bit, the filler above them all
    const int kbits = bits_for(uint64_t(n) + 1) + 2;
    const uint64_t fill = (uint64_t(1) << kbits) - 1;
    if (ne) k_ckeys_marker<<<grid_for(ne, B), B, 0, stream>>>(ne, eg, kk + nv, fill);
    uint64_t *cks = nullptr;
    uint32_t ncv = sort_unique_u64(ck, ck2, nv + ne, kbits, &cks);
    // drop the filler (non-marker edges) at the end
    if (ncv) {
      uint64_t last = 0;
      FH_HIP(hipMemcpyAsync(&last, cks + ncv - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
      sync();
      if (last == fill) ncv--;
    }
    // super vertices by sid -> condensed vid; their labels as the vertex dots
    uint32_t *idx = cidx.ensure(nv + 1), *vid = cvid.ensure(nv + 1);
    uint64_t *cd = cdot.ensure(ncv + 1);
    if (ncv) k_fill_u64<<<grid_for(ncv, B), B, 0, stream>>>(ncv, cd, ~0ull);
    uint32_t *sids = cidx2.ensure(nv + 1);
    if (nv) {
      uint32_t *kb = tmp_a.ensure(nv + 1), *vb = tmp_b.ensure(nv + 1), *va = tmp_c.ensure(nv + 1);
      uint32_t *ks = nullptr, *vs = nullptr;
      sort_pairs<uint32_t, uint32_t>(sid, nullptr, sid, va, kb, vb, nv, bits_for(n + 1), sort_ws,
                                     stream, &ks, &vs);
      FH_HIP(hipMemcpyAsync(idx, vs, nv * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream));
      uint32_t *sorted = tmp_d.ensure(nv + 1);
      FH_HIP(hipMemcpyAsync(sorted, ks, nv * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream));
      k_sid_vid<<<grid_for(nv, B), B, 0, stream>>>(nv, vg, idx, cks, ncv, vid, cd, sorted, sids);
    }
    // edges -> (src vid, dst vid), sorted unique -> CSR
    uint64_t *ed = ce.ensure(ne + 1);
    // edges (src vid << cb | dst vid): 2·cb key bits
    const int cb = bits_for(uint64_t(ncv) + 1);
    if (ne) k_cedges<<<grid_for(ne, B), B, 0, stream>>>(ne, eg, sids, vid, nv, cks, ncv, cb, ed);
    uint64_t *eds = nullptr;
    const uint32_t nce = sort_unique_u64(ce, ce2, ne, 2 * cb, &eds);
    uint32_t *cc = ccnt.ensure(ncv + 1), *co = coffs.ensure(ncv + 1);
    FH_HIP(hipMemsetAsync(cc, 0, size_t(ncv + 1) * sizeof(uint32_t), stream));
    if (nce) k_csr_counts<<<grid_for(nce, B), B, 0, stream>>>(nce, eds, cb, cc);
    exclusive_scan_u32(cc, co, ncv, scan_ws, stream);
    uint32_t *cdst_ = cdst2.ensure(nce + 1);
    if (nce) k_csr_dst<<<grid_for(nce, B), B, 0, stream>>>(nce, eds, cb, cdst_);
    // hub split (k_hub_aux above)
    uint32_t V2 = ncv;
    const uint32_t *off_g = co, *dst_g = cdst_, *rep0 = nullptr;
    const uint64_t *dot_g = cd, *ck_g = cks;
    if (nce && ncv) {
      uint32_t *nax = hub_nax.ensure(ncv + 1), *aoff = hub_aoff.ensure(ncv + 1);
      k_hub_aux<<<grid_for(ncv, B), B, 0, stream>>>(ncv, hub_deg, cc, nax);
      const uint32_t na = scan_total(nax, aoff, ncv);
      if (na) {
        V2 = ncv + na;
        uint32_t *cnt2 = hub_cnt.ensure(V2 + 1), *off2 = hub_off.ensure(V2 + 1);
        uint32_t *r0 = hub_rep0.ensure(V2 + 1), *vm = hub_vmap.ensure(ncv + 1);
        uint64_t *cd2 = hub_dot.ensure(V2 + 1), *ck2 = hub_ck.ensure(V2 + 1);
        k_hub_layout<<<grid_for(ncv, B), B, 0, stream>>>(ncv, hub_deg, cc, nax, aoff, cd, cks, cnt2,
                                                         cd2, ck2, r0, vm);
        exclusive_scan_u32(cnt2, off2, V2, scan_ws, stream);
        uint32_t *dst2 = hub_dst.ensure(nce + 1);
        k_hub_edges<<<grid_for(nce, B), B, 0, stream>>>(nce, hub_deg, eds, cb, co, aoff, off2, vm,
                                                         dst2);
        if (nv) k_map_u32<<<grid_for(nv, B), B, 0, stream>>>(nv, vid, vm);
        off_g = off2;
        dst_g = dst2;
        dot_g = cd2;
        ck_g = ck2;
        rep0 = r0;
      }
    }
    GraphInput gin;
    gin.V = V2;
    gin.off = off_g;
    gin.dst = dst_g;
    gin.dot = dot_g;
    gin.rep0 = rep0;
    gin.global_only = true;
    gin.want_orders = false;
    gin.want_per_key = false;
    cond.run(gin, cout_);
    FH_CHECK(ncv == 0 || (cout_.rep && cout_.kap && cout_.scc_label), FH_EINVARIANT,
             "dgraph: condensed graph outputs");
    t_end("condensed_solve");
    t_begin();
    // expansion: order key and label of every range vertex
    uint32_t *err = scal.get() + 3;
    FH_HIP(hipMemsetAsync(err, 0, sizeof(uint32_t), stream));
    k_expand<<<grid_for(V, B), B, 0, stream>>>(V, a, lrep, esc.get(), lkap, llab, sids, vid, nv,
                                               cout_.rep, cout_.kap, cout_.scc_label, ck_g,
                                               okey.ensure(V + 1), label.ensure(V + 1), err);
    // elements by the key's owner: counts, then placement
    const ElemPack ep{k, hb, shards, world, seqb};
    uint32_t *cur = el_cursor.ensure(kMaxWorld);
    FH_HIP(hipMemsetAsync(cur, 0, kMaxWorld * sizeof(uint32_t), stream));
    const unsigned g = (V + B - 1) / B;
    k_elem_route<<<g, B, 0, stream>>>(V, a, ep, key32.get(), dot.get(), okey.get(), cur, nullptr,
                                      nullptr, 0);
    std::vector<uint32_t> hc(world + 1);
    uint32_t herr = 0;
    FH_HIP(hipMemcpyAsync(hc.data(), cur, world * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    FH_HIP(hipMemcpyAsync(&herr, err, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    sync();
    FH_CHECK(herr == 0, FH_ENOTIMPL, "dgraph: depth >= 2^31");
    el_cnt.assign(world, 0);
    std::vector<uint32_t> base(world, 0);
    uint64_t tot = 0;
    for (uint32_t q = 0; q < world; q++) {
      base[q] = uint32_t(tot);
      el_cnt[q] = hc[q];
      tot += hc[q];
      counts[q] = hc[q];
    }
    FH_CHECK(tot == uint64_t(V) * k, FH_EINVARIANT, "dgraph: element count");
    FH_HIP(hipMemcpyAsync(el_base.ensure(kMaxWorld), base.data(), world * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    sync();
    t_end("expand");
  }

  void elements(uint64_t *out) {
    uint32_t *cur = el_cursor.get();
    FH_HIP(hipMemsetAsync(cur, 0, kMaxWorld * sizeof(uint32_t), stream));
    const ElemPack ep{k, hb, shards, world, seqb};
    const unsigned g = (V + B - 1) / B;
    k_elem_route<<<g, B, 0, stream>>>(V, a, ep, key32.get(), dot.get(), okey.get(), cur,
                                      el_base.get(), out, 1);
    sync();
  }

  // ---- 6. per-key sequences of this rank's keys ------------------------------------
  void per_key(uint32_t m, const uint64_t *el) {
    t_begin();
    n_pk = m;
    if (m == 0) {
      t_end("per_key");
      return;
    }
    uint64_t *x0 = e0a.ensure(m + 1), *x1 = e1a.ensure(m + 1);
    k_split_elems<<<grid_for(m, B), B, 0, stream>>>(m, el, x0, x1);
    // LSD: by (escaping|depth, dot32), then stably by (key, H)
    uint32_t *ka = ia.ensure(m + 1), *kb2 = ib.ensure(m + 1);
    uint64_t *ks = nullptr;
    uint32_t *vs = nullptr;
    sort_pairs<uint64_t, uint32_t>(x1, nullptr, x1, ka, e1b.ensure(m + 1), kb2, m, 64, sort_ws,
                                   stream, &ks, &vs);
    const uint64_t *x1s = ks;  // e1 in that order; vs = its source index
    uint64_t *g0 = e0b.ensure(m + 1);
    k_gather_u64<<<grid_for(m, B), B, 0, stream>>>(m, vs, x0, g0);
    // the values of the second sort: positions in the first sort's order
    uint64_t *ks2 = nullptr;
    uint32_t *vs2 = nullptr;
    uint32_t *pa = tmp_a.ensure(m + 1), *pb = tmp_b.ensure(m + 1);
    sort_pairs<uint64_t, uint32_t>(g0, nullptr, g0, pa, x0, pb, m,
                                   bits_for(cfg.key_space) + int(hb), sort_ws, stream, &ks2, &vs2);
    k_unpack_elems<<<grid_for(m, B), B, 0, stream>>>(m, vs2, ks2, x1s, hb, seqb,
                                                     pk_key.ensure(m + 1), pk_dot.ensure(m + 1));
    sync();
    t_end("per_key");
  }

  void results(uint32_t *h_dep_off, uint64_t *h_dep, size_t cap, size_t *dep_len,
               uint64_t *h_label, uint32_t *h_pk_key, uint64_t *h_pk_dot, size_t *pk_len) {
    uint32_t tot = fetch_u32(dep_off.get() + V, stream);
    if (dep_len) *dep_len = tot;
    if (pk_len) *pk_len = n_pk;
    if (h_dep) FH_CHECK(cap >= tot, FH_ECAP, "dgraph: dep capacity");
    if (h_dep_off)
      FH_HIP(hipMemcpyAsync(h_dep_off, dep_off.get(), (size_t(V) + 1) * sizeof(uint32_t),
                            hipMemcpyDeviceToHost, stream));
    if (h_dep && tot)
      FH_HIP(hipMemcpyAsync(h_dep, dep_dot.get(), size_t(tot) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                            stream));
    if (h_label)
      FH_HIP(hipMemcpyAsync(h_label, label.get(), size_t(V) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                            stream));
    if (h_pk_key && n_pk)
      FH_HIP(hipMemcpyAsync(h_pk_key, pk_key.get(), size_t(n_pk) * sizeof(uint32_t),
                            hipMemcpyDeviceToHost, stream));
    if (h_pk_dot && n_pk)
      FH_HIP(hipMemcpyAsync(h_pk_dot, pk_dot.get(), size_t(n_pk) * sizeof(uint64_t),
                            hipMemcpyDeviceToHost, stream));
    sync();
  }
};

}  // namespace fh

struct fh_dgraph {
  fh::DistGraph g;
  fh_dgraph(const fh_config &c, uint32_t r, uint32_t w) : g(c, r, w) {}
};

#define DG_BEGIN        \
  FH_API_BEGIN          \
  FH_CHECK(h, FH_EINVAL, "null handle"); \
  FH_HIP(hipSetDevice(h->g.device));

extern "C" {

fh_status fh_dgraph_create(const fh_config *cfg, uint32_t rank, uint32_t world, fh_dgraph **out) {
  FH_API_BEGIN
  FH_CHECK(cfg && out, FH_EINVAL, "null argument");
  fh_config c = *cfg;
  if (c.device < 0) {
    const char *e = getenv("FANTOCH_HIP_DEVICE");
    c.device = e ? atoi(e) : 0;
  }
  FH_HIP(hipSetDevice(c.device));
  *out = new fh_dgraph(c, rank, world);
  FH_API_END
}

fh_status fh_dgraph_destroy(fh_dgraph *h) {
  FH_API_BEGIN
  delete h;
  FH_API_END
}

fh_status fh_dgraph_stage(fh_dgraph *h, const fh_stream_desc *desc, uint32_t shards,
                          const uint64_t *dot, const uint64_t *key_id, const uint64_t *log_off,
                          const uint32_t *log_elem, uint64_t *send_counts, uint64_t *recv_counts,
                          uint64_t *range) {
  DG_BEGIN
  FH_CHECK(desc, FH_EINVAL, "null argument");
  h->g.stage(*desc, shards, dot, key_id, log_off, log_elem);
  for (uint32_t q = 0; q < h->g.world; q++) {
    if (send_counts) send_counts[q] = h->g.send_cnt[q];
    if (recv_counts) recv_counts[q] = h->g.recv_cnt[q];
  }
  if (range) {
    range[0] = h->g.a;
    range[1] = h->g.V;
  }
  FH_API_END
}

fh_status fh_dgraph_keydeps(fh_dgraph *h, uint32_t *send_dev) {
  DG_BEGIN
  h->g.keydeps(send_dev);
  FH_API_END
}

fh_status fh_dgraph_local(fh_dgraph *h, const uint32_t *recv_dev, uint64_t *query_counts) {
  DG_BEGIN
  h->g.local_stage(recv_dev);
  for (uint32_t q = 0; q < h->g.world; q++)
    if (query_counts) query_counts[q] = h->g.q_cnt[q];
  FH_API_END
}

fh_status fh_dgraph_queries(fh_dgraph *h, uint32_t *query_dev) {
  DG_BEGIN
  if (h->g.nq)
    FH_HIP(hipMemcpyAsync(query_dev, h->g.queries.get(), size_t(h->g.nq) * sizeof(uint32_t),
                          hipMemcpyDeviceToDevice, h->g.stream));
  h->g.sync();
  FH_API_END
}

fh_status fh_dgraph_answer(fh_dgraph *h, size_t n, const uint32_t *in_dev, uint32_t *out_dev) {
  DG_BEGIN
  h->g.answer(uint32_t(n), in_dev, out_dev);
  FH_API_END
}

fh_status fh_dgraph_condense(fh_dgraph *h, const uint32_t *answers_dev, uint64_t *nv,
                             uint64_t *ne) {
  DG_BEGIN
  FH_CHECK(nv && ne, FH_EINVAL, "null argument");
  h->g.condense(answers_dev, nv, ne);
  FH_API_END
}

fh_status fh_dgraph_condensed_part(fh_dgraph *h, uint64_t *verts_dev, uint64_t *edges_dev) {
  DG_BEGIN
  h->g.condensed_part(verts_dev, edges_dev);
  FH_API_END
}

fh_status fh_dgraph_solve(fh_dgraph *h, size_t nv, const uint64_t *verts_dev, size_t ne,
                          const uint64_t *edges_dev, uint64_t *elem_counts) {
  DG_BEGIN
  FH_CHECK(elem_counts, FH_EINVAL, "null argument");
  h->g.solve(uint32_t(nv), verts_dev, uint32_t(ne), edges_dev, elem_counts);
  FH_API_END
}

fh_status fh_dgraph_elements(fh_dgraph *h, uint64_t *elem_dev) {
  DG_BEGIN
  h->g.elements(elem_dev);
  FH_API_END
}

fh_status fh_dgraph_per_key(fh_dgraph *h, size_t n, const uint64_t *elem_dev) {
  DG_BEGIN
  h->g.per_key(uint32_t(n), elem_dev);
  FH_API_END
}

fh_status fh_dgraph_results(fh_dgraph *h, uint32_t *dep_off, uint64_t *dep_dot, size_t dep_cap,
                            size_t *dep_len, uint64_t *scc_label, uint32_t *pk_key,
                            uint64_t *pk_dot, size_t *pk_len) {
  DG_BEGIN
  h->g.results(dep_off, dep_dot, dep_cap, dep_len, scc_label, pk_key, pk_dot, pk_len);
  FH_API_END
}

fh_status fh_dgraph_set_profiling(fh_dgraph *h, int on) {
  DG_BEGIN
  h->g.profile = on != 0;
  FH_API_END
}

fh_status fh_dgraph_stage_times(fh_dgraph *h, const char **names, float *ms, size_t cap,
                                size_t *len) {
  DG_BEGIN
  const auto &t = h->g.times;
  if (len) *len = t.size();
  for (size_t i = 0; i < t.size() && i < cap; i++) {
    if (names) names[i] = t[i].first.c_str();
    if (ms) ms[i] = t[i].second;
  }
  FH_API_END
}

}  // extern "C"
