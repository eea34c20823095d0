// scan.h -- exclusive prefix sum (reduce-then-scan, three launches).
#pragma once

#include "fh_common.h"

namespace fh {

struct ScanWorkspace {
  DBuf<uint32_t> status;  // per-block sums
};

// out[i] = sum(in[0..i)), out[n] = total.  out must hold n+1 elements.
// Totals must fit in 32 bits.
void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws,
                        hipStream_t s);
// out[i] = max(in[0..i)) (0 for i = 0), out[n] = max of all.
void exclusive_scan_max_u32(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws,
                            hipStream_t s);

// Per-key offsets from run bounds: runs holds n (start, end | tag' << 23)
// u32 pairs, a run of this batch where tag' == tag (1..511); off[i] = the
// total length of the runs before i (off[n] = the total) and delta[i] =
// off[i] - start_i, the shift that moves run i from its position to its
// place in ascending order.
void run_offsets(const uint32_t *runs, uint32_t tag, uint32_t *off, uint32_t *delta, size_t n,
                 ScanWorkspace &ws, hipStream_t s);

// Low-latency read-back of n <= 14 device u32 words (fixpoint flags,
// totals) into host memory: a one-wave kernel stores them into pinned,
// device-mapped host memory followed by a sequence number (system-scope
// release), and the host polls the sequence number (with hipStreamQuery, so
// a failed launch surfaces as an error instead of a hang).  A pageable
// hipMemcpyAsync + hipStreamSynchronize round trip measured ~150-180 us on
// the GPU box; the graph's fixpoint loops take one per iteration.
void fetch_u32(const uint32_t *dev, uint32_t *host, int n, hipStream_t s);
inline uint32_t fetch_u32(const uint32_t *dev, hipStream_t s) {
  uint32_t v = 0;
  fetch_u32(dev, &v, 1, s);
  return v;
}

}  // namespace fh
