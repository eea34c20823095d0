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

}  // namespace fh
