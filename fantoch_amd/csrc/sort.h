// sort.h -- stable LSD radix sort of (key, u32 value) pairs, onesweep style.
//
// One histogram launch computes every 8-bit digit histogram; then one launch
// per digit: each 256-thread workgroup takes a 4096-item tile (tile id from an
// atomic ticket, so a tile only waits on tiles already running), ranks its
// items stably with wave64 ballot matching, publishes per-digit counts and
// resolves its global offsets by decoupled look-back over 32-bit
// {flag, count} granules (single sc1 stores/loads, MI355X_MICROARCH.md
// "Valid forms", R2), and writes its items coalesced from LDS.
#pragma once

#include "fh_common.h"

namespace fh {

constexpr int kSortThreads = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortThreads * kSortItems;  // 4096

struct SortWorkspace {
  DBuf<uint32_t> meta;  // [hist: 8*256][ctr: 16][status: passes*tiles*256]
  size_t meta_words(size_t n, int passes) const;
};

// Sorts n pairs stably by the low `key_bits` bits of the key.  vals_in ==
// nullptr means values are the input positions 0..n-1.  Data ping-pongs
// between (ka, va) and (kb, vb); *kout / *vout point at the sorted result
// (one of the two).  keys_in/vals_in may alias either pair.  n < 2^30.
template <class K>
void sort_pairs(const K *keys_in, const uint32_t *vals_in, K *ka, uint32_t *va,
                K *kb, uint32_t *vb, size_t n, int key_bits, SortWorkspace &ws,
                hipStream_t s, K **kout, uint32_t **vout);

// Device error word of the last sort (look-back spin timeout); 0 = ok.
// Lives at meta[8*256 + 8].
constexpr int kSortErrWord = 8 * 256 + 8;

}  // namespace fh
