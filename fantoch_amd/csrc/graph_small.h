// graph_small.h -- one executor pass of a small graph in one workgroup
// (graph_small.hip), used by fh_graph for small batches.
#pragma once

#include "fh_common.h"

namespace fh {

// A batch as the host packs it into one mapped pinned block: dots, dependency
// dots, the executed-clock mirror (frontier[256] + sorted exceptions, nf + ne
// words, only when it changed), key ids, key and dependency offsets.
struct Upload {
  const uint64_t *dot, *dep, *clk;
  const uint32_t *key, *koff, *doff;
  uint32_t n, nk, nd, nf, ne;
};
// Where an Upload goes: the rows after the carried prefix (offsets rebased by
// the carried key / dependency counts) and the device clock mirror.
struct AppendDst {
  uint64_t *dot;
  uint32_t *koff, *key, *doff;
  uint64_t *dep;
  uint32_t kbase, dbase;
  uint64_t *frontier, *exc;
};
// item i of the append (i < append_items(u)): loaded, then stored, so that a
// caller can issue several items' loads (reads of host memory over PCIe)
// before the first store
struct AppendVals {
  uint64_t dot, dep, clk;
  uint32_t key, koff, doff;
};
__device__ __forceinline__ uint32_t append_items(const Upload &u) {
  return max(max(u.n ? u.n + 1 : 0u, u.nk), max(u.nd, u.nf + u.ne));
}
__device__ __forceinline__ void append_load(const Upload &u, uint32_t i, AppendVals &v) {
  v.dot = i < u.n ? u.dot[i] : 0;
  v.koff = u.n && i <= u.n ? u.koff[i] : 0;
  v.doff = u.n && i <= u.n ? u.doff[i] : 0;
  v.key = i < u.nk ? u.key[i] : 0;
  v.dep = i < u.nd ? u.dep[i] : 0;
  v.clk = i < u.nf + u.ne ? u.clk[i] : 0;
}
__device__ __forceinline__ void append_store(const Upload &u, const AppendDst &a, uint32_t i,
                                             const AppendVals &v) {
  // rows only for a non-empty batch: with n == 0 the carried set's end
  // offsets (koff[0] = koff[P] of the set) must stay as they are
  if (i < u.n) a.dot[i] = v.dot;
  if (u.n && i <= u.n) {
    a.koff[i] = v.koff + a.kbase;
    a.doff[i] = v.doff + a.dbase;
  }
  if (i < u.nk) a.key[i] = v.key;
  if (i < u.nd) a.dep[i] = v.dep;
  if (i < u.nf) a.frontier[i] = v.clk;
  else if (i < u.nf + u.ne) a.exc[i - u.nf] = v.clk;
}
__device__ __forceinline__ void append_item(const Upload &u, const AppendDst &a, uint32_t i) {
  AppendVals v;
  append_load(u, i, v);
  append_store(u, a, i, v);
}

constexpr int kSmallV = 2048;  // vertices (carried + batch)
constexpr int kSmallE = 8192;  // dependency entries of those vertices

struct SmallPass {
  // the batch's rows and the clock mirror, appended by the kernel itself
  // before the pass reads the vertex set (one launch instead of two)
  Upload up;
  AppendDst dst;
  uint32_t V;
  uint32_t P;  // the first P vertices are carried pending ones
  // vertices (carried pending, then the batch): dots, key lists, dependency
  // lists (CSR offsets over the key / dependency arrays)
  const uint64_t *dot;
  const uint32_t *koff, *key32, *doff;
  const uint64_t *ddot;
  // executed clock mirror: frontier[256] + sorted exceptions
  const uint64_t *frontier, *exc;
  uint32_t nexc;
  // outputs: executed dots and labels in execution order, per-vertex pending
  // flags, missing dependency dots (repeats allowed, up to miss_cap)
  uint64_t *xdot, *xlab;
  uint8_t *xcar;  // per executed vertex: 1 if carried (host metadata to drop)
  uint8_t *blocked;
  uint64_t *miss;
  uint32_t miss_cap;
  // the survivors, compacted into the next vertex set
  uint64_t *ndot;
  uint32_t *nkoff, *nkey32, *ndoff;
  uint64_t *nddot;
  // [0] executed, [1] missing dots, [2] duplicate dot, [3] survivors,
  // [4] their key entries, [5] their dependency entries
  uint32_t *header;
  int stamps;  // FH_GRAPH_DEBUG: phase clock stamps into header[8..27]
  uint32_t seq;  // written to header[31] last (the host may poll it)
  // fault injection (fh_graph_inject_small_delay, tests): the pass waits
  // this long before it starts, bounded by the wall clock
  uint32_t delay_us;
};

// (host: the completion wait is fh_common.h poll_completion)

void launch_graph_small(const SmallPass &p, hipStream_t s);

}  // namespace fh
