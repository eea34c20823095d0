// graph_small.h -- one executor pass of a small graph in one workgroup
// (graph_small.hip), used by fh_graph for small batches.
#pragma once

#include "fh_common.h"

namespace fh {

constexpr int kSmallV = 2048;  // vertices (carried + batch)
constexpr int kSmallE = 8192;  // dependency entries of those vertices

struct SmallPass {
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
  int stamps;  // FH_GRAPH_DEBUG: phase clock stamps into header[8..25]
  uint32_t seq;  // written to header[31] last (the host may poll it)
};

void launch_graph_small(const SmallPass &p, hipStream_t s);

}  // namespace fh
