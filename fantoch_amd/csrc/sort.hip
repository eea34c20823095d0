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

namespace fh {
namespace {

constexpr int kThreads = kSortThreads;  // 256
constexpr int kItems = kSortItems;      // 16
constexpr int kTile = kSortTile;        // 4096
constexpr int kWaves = kThreads / 64;
constexpr int kGroup = 64;              // tiles per scan group

__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
  uint64_t peers = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; b++) {
    const bool bit = (d >> b) & 1;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  return peers;
}

// Exclusive scan of one value per thread over the 256-thread block.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_tmp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  uint32_t pre = 0;
#pragma unroll
  for (int i = 0; i < kWaves; i++)
    if (i < w) pre += s_tmp[i];
  __syncthreads();
  return pre + x - v;
}

// Tile element mapping (coalesced): wave w owns a contiguous sub-tile of
// 64*kItems elements, item i of lane l is element w*64*kItems + i*64 + l.
// Tile order == (wave, item, lane) lexicographic == input order.
__device__ __forceinline__ uint32_t elem_index(uint32_t base, int w, int i, int lane) {
  return base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + uint32_t(lane);
}

template <class K>
__global__ void __launch_bounds__(kThreads)
    k_up(const K *__restrict__ keys, uint32_t n, int shift, uint32_t *__restrict__ counts) {
  __shared__ uint32_t s_h[kWaves][256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < kWaves * 256; i += kThreads) (&s_h[0][0])[i] = 0;
  const uint32_t base = blockIdx.x * kTile;
  K key[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = elem_index(base, w, i, lane);
    key[i] = idx < n ? keys[idx] : K(0);
  }
  __syncthreads();
  const uint64_t lt = (uint64_t(1) << lane) - 1;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = elem_index(base, w, i, lane);
    const bool valid = idx < n;
    const uint32_t d = uint32_t((key[i] >> shift) & 255);
    const uint64_t peers = match_digit(d, valid);
    if (valid && (peers & lt) == 0) s_h[w][d] += uint32_t(__popcll(peers));  // wave-private
  }
  __syncthreads();
  uint32_t c = 0;
#pragma unroll
  for (int ww = 0; ww < kWaves; ww++) c += s_h[ww][tid];
  counts[size_t(blockIdx.x) * 256 + tid] = c;
}

// Group g of kGroup tiles: counts[t][d] <- exclusive prefix within the group,
// gsum[g][d] <- group total.
__global__ void __launch_bounds__(256)
    k_scan_a(uint32_t *__restrict__ counts, uint32_t tiles, uint32_t *__restrict__ gsum) {
  const uint32_t g = blockIdx.x, d = threadIdx.x;
  const uint32_t t0 = g * kGroup, t1 = min(tiles, t0 + kGroup);
  uint32_t v[kGroup];
#pragma unroll
  for (int i = 0; i < kGroup; i++) v[i] = (t0 + i < t1) ? counts[size_t(t0 + i) * 256 + d] : 0u;
  uint32_t run = 0;
#pragma unroll
  for (int i = 0; i < kGroup; i++) {
    if (t0 + i < t1) counts[size_t(t0 + i) * 256 + d] = run;
    run += v[i];
  }
  gsum[size_t(g) * 256 + d] = run;
}

// One workgroup: gsum[g][d] <- exclusive prefix over groups, dbase[d] <-
// exclusive prefix of the digit totals.
__global__ void __launch_bounds__(256)
    k_scan_b(uint32_t *__restrict__ gsum, uint32_t groups, uint32_t *__restrict__ dbase) {
  __shared__ uint32_t s_tmp[kWaves];
  const uint32_t d = threadIdx.x;
  uint32_t run = 0;
  for (uint32_t g0 = 0; g0 < groups; g0 += 16) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = (g0 + i < groups) ? gsum[size_t(g0 + i) * 256 + d] : 0u;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      if (g0 + i < groups) gsum[size_t(g0 + i) * 256 + d] = run;
      run += v[i];
    }
  }
  dbase[d] = block_excl_scan(run, s_tmp);
}

// Small sorts (tiles <= kFusedMaxTiles): one 1024-thread workgroup does both
// scan levels -- 4 threads per digit, each over a contiguous quarter of the
// tiles (gsum[q][d] <- quarter prefix, dbase[d] <- digit base).
constexpr int kFusedMaxTiles = 1024;
__global__ void __launch_bounds__(1024)
    k_scan_fused(uint32_t *__restrict__ counts, uint32_t tiles, uint32_t per,
                 uint32_t *__restrict__ gsum, uint32_t *__restrict__ dbase) {
  __shared__ uint32_t s_part[4][256];
  __shared__ uint32_t s_tmp[4];
  const uint32_t d = threadIdx.x & 255, q = threadIdx.x >> 8;
  const uint32_t t0 = q * per, t1 = min(tiles, t0 + per);
  uint32_t run = 0;
  for (uint32_t t = t0; t < t1; t += 16) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = (t + i < t1) ? counts[size_t(t + i) * 256 + d] : 0u;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      if (t + i < t1) counts[size_t(t + i) * 256 + d] = run;
      run += v[i];
    }
  }
  s_part[q][d] = run;
  __syncthreads();
  uint32_t qpre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (uint32_t(i) < q) qpre += s_part[i][d];
    tot += s_part[i][d];
  }
  gsum[q * 256 + d] = qpre;
  // exclusive scan of the digit totals (waves 0..3 hold digits 0..255; every
  // thread reaches the barrier)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (q == 0 && lane == 63) s_tmp[w] = x;
  __syncthreads();
  if (q == 0) {
    uint32_t pre = 0;
    for (int i = 0; i < w; i++) pre += s_tmp[i];
    dbase[d] = pre + x - tot;
  }
}

template <class K, class VT, bool IOTA>
__global__ void __launch_bounds__(kThreads)
    k_down(const K *__restrict__ kin, const VT *__restrict__ vin, K *__restrict__ kout,
           VT *__restrict__ vout, uint32_t n, int shift,
           const uint32_t *__restrict__ counts, const uint32_t *__restrict__ gsum,
           uint32_t gsize, const uint32_t *__restrict__ dbase) {
  __shared__ K s_k[kTile];
  __shared__ VT s_v[kTile];
  __shared__ uint32_t s_wh[kWaves][256];
  __shared__ uint32_t s_dex[256];
  __shared__ uint32_t s_gb[256];
  __shared__ uint32_t s_tmp[kWaves];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t tile = blockIdx.x;
  const uint32_t base = tile * kTile;
  for (int i = tid; i < kWaves * 256; i += kThreads) (&s_wh[0][0])[i] = 0;
  // global offset of this tile's digit runs (independent of the items)
  const uint32_t gofs =
      dbase[tid] + gsum[size_t(tile / gsize) * 256 + tid] + counts[size_t(tile) * 256 + tid];
  K key[kItems];
  VT val[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = elem_index(base, w, i, lane);
    const bool valid = idx < n;
    key[i] = valid ? kin[idx] : K(0);
    val[i] = IOTA ? VT(idx) : (valid ? vin[idx] : VT(0));
  }
  __syncthreads();
  const uint64_t lt = (uint64_t(1) << lane) - 1;
  uint32_t rank[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = elem_index(base, w, i, lane);
    const bool valid = idx < n;
    const uint32_t d = uint32_t((key[i] >> shift) & 255);
    const uint64_t peers = match_digit(d, valid);
    uint32_t b0 = 0;
    if (valid) b0 = s_wh[w][d];
    if (valid && (peers & lt) == 0) s_wh[w][d] = b0 + uint32_t(__popcll(peers));
    rank[i] = b0 + uint32_t(__popcll(peers & lt));
  }
  __syncthreads();
  uint32_t cnt = 0;
#pragma unroll
  for (int ww = 0; ww < kWaves; ww++) {
    const uint32_t c = s_wh[ww][tid];
    s_wh[ww][tid] = cnt;
    cnt += c;
  }
  const uint32_t lpre = block_excl_scan(cnt, s_tmp);
  s_dex[tid] = lpre;
  s_gb[tid] = gofs;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = elem_index(base, w, i, lane);
    if (idx < n) {
      const uint32_t d = uint32_t((key[i] >> shift) & 255);
      const uint32_t pos = s_dex[d] + s_wh[w][d] + rank[i];
      s_k[pos] = key[i];
      s_v[pos] = val[i];
    }
  }
  __syncthreads();
  const uint32_t tile_n = min(uint32_t(kTile), n - base);
#pragma unroll 4
  for (uint32_t j = tid; j < tile_n; j += kThreads) {
    const K k = s_k[j];
    const uint32_t d = uint32_t((k >> shift) & 255);
    const uint32_t o = s_gb[d] + (j - s_dex[d]);
    kout[o] = k;
    vout[o] = s_v[j];
  }
}

}  // namespace

size_t SortWorkspace::meta_words(size_t n, int) const {
  const size_t tiles = (n + kTile - 1) / kTile;
  const size_t groups = (tiles + kGroup - 1) / kGroup;
  return (tiles + groups) * 256;
}

void SortWorkspace::prepare(size_t tiles, int, hipStream_t) {
  const size_t groups = std::max<size_t>((tiles + kGroup - 1) / kGroup, 4);
  meta.ensure((tiles + groups + 1) * 256);
}

template <class K, class VT>
void sort_pairs(const K *keys_in, const VT *vals_in, K *ka, VT *va, K *kb, VT *vb, size_t n,
                int key_bits, SortWorkspace &ws, hipStream_t s, K **kout, VT **vout) {
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "sort: too many elements (>= 2^30)");
  int passes = (key_bits + 7) / 8;
  if (passes < 1) passes = 1;
  if (passes > int(sizeof(K))) passes = int(sizeof(K));
  if (n == 0) {
    *kout = ka;
    *vout = va;
    return;
  }
  const uint32_t tiles = uint32_t((n + kTile - 1) / kTile);
  const uint32_t groups = (tiles + kGroup - 1) / kGroup;
  ws.prepare(tiles, passes, s);
  uint32_t *counts = ws.meta.get();
  uint32_t *gsum = counts + size_t(tiles) * 256;
  uint32_t *dbase = gsum + size_t(std::max<uint32_t>(groups, 4)) * 256;
  const K *ki = keys_in;
  const VT *vi = vals_in;
  // never write pass 0 over its own input
  const bool alias_a = (const void *)keys_in == (const void *)ka ||
                       (vals_in && (const void *)vals_in == (const void *)va);
  K *ko = alias_a ? kb : ka;
  VT *vo = alias_a ? vb : va;
  for (int p = 0; p < passes; p++) {
    const int shift = 8 * p;
    k_up<K><<<tiles, kThreads, 0, s>>>(ki, uint32_t(n), shift, counts);
    uint32_t gsize = kGroup;
    if (tiles <= kFusedMaxTiles) {
      gsize = (tiles + 3) / 4;
      k_scan_fused<<<1, 1024, 0, s>>>(counts, tiles, gsize, gsum, dbase);
    } else {
      k_scan_a<<<groups, 256, 0, s>>>(counts, tiles, gsum);
      k_scan_b<<<1, 256, 0, s>>>(gsum, groups, dbase);
    }
    if (p == 0 && vals_in == nullptr) {
      k_down<K, VT, true><<<tiles, kThreads, 0, s>>>(ki, nullptr, ko, vo, uint32_t(n), shift,
                                                      counts, gsum, gsize, dbase);
    } else {
      // algorithmic traffic of a key+value scatter pass: read and write every
      // pair once
      probed_launch("sort_scatter", double(n) * 2.0 * (sizeof(K) + sizeof(VT)),
                    k_down<K, VT, false>, dim3(tiles), dim3(kThreads), s, ki, vi, ko, vo,
                    uint32_t(n), shift, (const uint32_t *)counts, (const uint32_t *)gsum, gsize,
                    (const uint32_t *)dbase);
    }
    ki = ko;
    vi = vo;
    if (ko == ka) {
      ko = kb;
      vo = vb;
    } else {
      ko = ka;
      vo = va;
    }
  }
  *kout = const_cast<K *>(ki);
  *vout = const_cast<VT *>(vi);
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
