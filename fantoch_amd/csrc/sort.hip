// sort.hip -- stable LSD radix sort for gfx950, reduce-then-scan (see sort.h).
//
// Per 8-bit digit pass, four launches and no inter-workgroup hand-off inside a
// launch (MI355X's eight XCD L2s are not coherent: a chained look-back costs
// one ~1-3 us hand-off per tile, MI355X_MICROARCH.md "handoff-1to1", which
// serialised a onesweep pass at one tile per hand-off):
//   k_up      tile digit counts           (reads keys once)
//   k_scan_a  per group of 64 tiles: in-place exclusive prefix over its tiles,
//             group totals
//   k_scan_b  one workgroup: prefix over groups + digit bases
//   k_down    stable rank in LDS (wave64 ballot matching), scatter through LDS
//             so global writes are runs of one digit
#include <algorithm>
#include <cstdlib>

#include "sort.h"
#include "sort_impl.h"

namespace fh {

namespace {
constexpr int kWideMax = 9;  // widest digit (R = 512: the code placement's buckets)
}  // namespace

size_t SortWorkspace::meta_words(size_t n, int) const {
  const size_t tiles = (n + kTile - 1) / kTile;
  const size_t groups = (tiles + kGroup - 1) / kGroup;
  return (tiles + groups) * (size_t(1) << kWideMax);
}

void SortWorkspace::prepare(size_t tiles, int, hipStream_t) {
  const size_t groups = std::max<size_t>((tiles + kGroup - 1) / kGroup, 4);
  meta.ensure((tiles + groups + 1) * (size_t(1) << kWideMax));
}

// Digit plan: sort_digit_bits (sort_impl.h), balanced digits of <= 8 bits.
// (Tried: keys of 17..22 bits in two passes of 10 or 11 bits instead of
// three of 8.  No faster on C4 -- KeyDeps 15.75 vs 15.53 ms, per-key 3.40 vs
// 3.29 ms: the wide k_down holds 57-74 KB of LDS, 2 workgroups per CU
// instead of 4, and matches 10 ballots per item.)
template <class K, class VT>
void sort_pairs(const K *keys_in, const VT *vals_in, K *ka, VT *va, K *kb, VT *vb, size_t n,
                int key_bits, SortWorkspace &ws, hipStream_t s, K **kout, VT **vout) {
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "sort: too many elements (>= 2^30)");
  const int db = sort_digit_bits(key_bits, int(sizeof(K)));
  int passes = (key_bits + db - 1) / db;
  if (passes < 1) passes = 1;
  if (db == 8 && passes > int(sizeof(K))) passes = int(sizeof(K));
  if (n == 0) {
    *kout = ka;
    *vout = va;
    return;
  }
  // never write pass 0 over its own input
  const bool alias_a = (const void *)keys_in == (const void *)ka ||
                       (vals_in && (const void *)vals_in == (const void *)va);
  const bool iota = vals_in == nullptr;
#define FH_SORT_RUN(DBV)                                                                         \
  if (iota)                                                                                     \
    sort_passes<K, VT, DBV, ArraySrc<K, VT, true>>(ArraySrc<K, VT, true>{keys_in, nullptr},     \
                                                   false, ka, va, kb, vb, alias_a, n, passes,  \
                                                   db, ws, s, kout, vout);                      \
  else                                                                                          \
    sort_passes<K, VT, DBV, ArraySrc<K, VT, false>>(ArraySrc<K, VT, false>{keys_in, vals_in},   \
                                                    true, ka, va, kb, vb, alias_a, n, passes,  \
                                                    db, ws, s, kout, vout);
  if (db == 6) {
    FH_SORT_RUN(6)
  } else if (db == 7) {
    FH_SORT_RUN(7)
  } else {
    FH_SORT_RUN(8)
  }
#undef FH_SORT_RUN
}

template void sort_pairs<uint32_t, uint32_t>(const uint32_t *, const uint32_t *, uint32_t *,
                                             uint32_t *, uint32_t *, uint32_t *, size_t, int,
                                             SortWorkspace &, hipStream_t, uint32_t **,
                                             uint32_t **);
template void sort_pairs<uint64_t, uint32_t>(const uint64_t *, const uint32_t *, uint64_t *,
                                             uint32_t *, uint64_t *, uint32_t *, size_t, int,
                                             SortWorkspace &, hipStream_t, uint64_t **,
                                             uint32_t **);
template void sort_pairs<uint32_t, uint64_t>(const uint32_t *, const uint64_t *, uint32_t *,
                                             uint64_t *, uint32_t *, uint64_t *, size_t, int,
                                             SortWorkspace &, hipStream_t, uint32_t **,
                                             uint64_t **);

}  // namespace fh
