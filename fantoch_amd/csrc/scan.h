// scan.h -- single-pass exclusive prefix sum (decoupled look-back).
#pragma once

#include "fh_common.h"

namespace fh {

struct ScanWorkspace {
  DBuf<uint32_t> status;  // [0]=ticket, [1]=error, [2..] one word per tile
};

// out[i] = sum(in[0..i)), out[n] = total.  out must hold n+1 elements.
// Totals must stay below 2^30 (the look-back granule keeps a 30-bit count).
void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws,
                        hipStream_t s);

}  // namespace fh
