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

namespace {
template <int DB>
void unpack_passes(const uint32_t *keys_in, const uint32_t *vals_in, uint32_t *ka, uint32_t *va,
                   uint32_t *kb, uint32_t *vb, size_t n, int passes, int db, int sb,
                   uint64_t *dout, SortWorkspace &ws, hipStream_t s, uint32_t **kout) {
  using Src = ArraySrc<uint32_t, uint32_t, false>;
  const uint32_t tiles = uint32_t((n + kTile - 1) / kTile);
  const uint32_t groups = (tiles + kGroup - 1) / kGroup;
  ws.prepare(tiles, passes, s);
  const uint32_t R = 1u << db;
  uint32_t *counts = ws.meta.get();
  uint32_t *gsum = counts + size_t(tiles) * R;
  uint32_t *dbase = gsum + size_t(std::max<uint32_t>(groups, 4)) * R;
  const uint32_t *ki = keys_in, *vi = vals_in;
  for (int p = 0; p + 1 < passes; p++) {
    // never write a pass over its own input
    const bool to_b = ki == ka || vi == va;
    uint32_t *kn = to_b ? kb : ka, *vn = to_b ? vb : va;
    sort_pass<uint32_t, uint32_t, DB, Src>(Src{ki, vi}, kn, StoreVal<uint32_t>{vn}, n, db * p,
                                           tiles, groups, counts, gsum, dbase, s, true);
    ki = kn;
    vi = vn;
  }
  uint32_t *kn = ki == ka ? kb : ka;
  sort_pass<uint32_t, uint32_t, DB, Src, StoreUnpackDot>(Src{ki, vi}, kn, StoreUnpackDot{dout, sb},
                                                         n, db * (passes - 1), tiles, groups,
                                                         counts, gsum, dbase, s, true);
  *kout = kn;
}
}  // namespace

void sort_pairs_unpack_dots(const uint32_t *keys_in, const uint32_t *vals_in, uint32_t *ka,
                            uint32_t *va, uint32_t *kb, uint32_t *vb, size_t n, int key_bits,
                            int sb, uint64_t *dout, SortWorkspace &ws, hipStream_t s,
                            uint32_t **kout) {
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "sort: too many elements (>= 2^30)");
  FH_CHECK(vals_in != nullptr && sb >= 1 && sb <= 31, FH_EINVAL, "sort: packed dots expected");
  const int db = sort_digit_bits(key_bits, 4);
  int passes = (key_bits + db - 1) / db;
  if (passes < 1) passes = 1;
  if (db == 8 && passes > 4) passes = 4;
  if (n == 0) {
    *kout = ka;
    return;
  }
  if (db == 6)
    unpack_passes<6>(keys_in, vals_in, ka, va, kb, vb, n, passes, db, sb, dout, ws, s, kout);
  else if (db == 7)
    unpack_passes<7>(keys_in, vals_in, ka, va, kb, vb, n, passes, db, sb, dout, ws, s, kout);
  else
    unpack_passes<8>(keys_in, vals_in, ka, va, kb, vb, n, passes, db, sb, dout, ws, s, kout);
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
