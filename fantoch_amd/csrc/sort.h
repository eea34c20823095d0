// sort.h -- stable LSD radix sort of (key, value) pairs, reduce-then-scan.
//
// 8-bit digits (10 or 11 for keys of 17..22 bits: two passes instead of
// three), per pass: tile digit counts, a two-level scan of the counts (no
// inter-workgroup hand-off inside any launch), and a stable LDS-staged
// scatter whose tile ranks come from wave64 ballot matching.
#pragma once

#include "fh_common.h"

namespace fh {

constexpr int kSortThreads = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortThreads * kSortItems;  // 4096

struct SortWorkspace {
  DBuf<uint32_t> meta;  // [tile digit counts: tiles*R][group sums: groups*R], R <= 2048
  size_t meta_words(size_t n, int passes) const;
  void prepare(size_t tiles, int passes, hipStream_t s);
};

// Sorts n pairs stably by the low `key_bits` bits of the key.  vals_in ==
// nullptr means values are the input positions 0..n-1.  Data ping-pongs
// between (ka, va) and (kb, vb); *kout / *vout point at the sorted result
// (one of the two).  keys_in/vals_in may alias either pair.  n < 2^30.
// Values are u32 (element ids) or u64 (dots: the per-key sequences carry
// them through the sort instead of gathering them afterwards).
template <class K, class VT = uint32_t>
void sort_pairs(const K *keys_in, const VT *vals_in, K *ka, VT *va,
                K *kb, VT *vb, size_t n, int key_bits, SortWorkspace &ws,
                hipStream_t s, K **kout, VT **vout);

// sort_pairs of (key, packed 32-bit dot src << sb | seq) whose last pass
// writes the values widened to u64 dots (src << 56 | seq) into dout (no
// separate unpacking pass over the sorted values); *kout: the sorted keys
// (ka or kb).  dout must not alias the value buffers.
void sort_pairs_unpack_dots(const uint32_t *keys_in, const uint32_t *vals_in, uint32_t *ka,
                            uint32_t *va, uint32_t *kb, uint32_t *vb, size_t n, int key_bits,
                            int sb, uint64_t *dout, SortWorkspace &ws, hipStream_t s,
                            uint32_t **kout);


}  // namespace fh
