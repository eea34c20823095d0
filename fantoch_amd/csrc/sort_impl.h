// sort_impl.h -- the radix sort kernels and pass driver (sort.hip), shared
// with callers that feed pass 0 from their own source (sort_pairs_src).
#pragma once

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

template <int DB>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
  uint64_t peers = __ballot(valid);
#pragma unroll
  for (int b = 0; b < DB; b++) {
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

// Tile digit counts.  Runs of equal digits in adjacent lanes (passes after
// the first see each key's elements contiguous: a hot key fills whole waves)
// add their length with one LDS atomic from the run's first lane.  (Tried:
// one atomic per item, 35 against 16 us per pass on a C4 chunk; wave64
// ballot matching, slower on Zipf streams than either.)
template <class K, class VT, int DB, class Src>
__global__ void __launch_bounds__(kThreads)
    k_up(Src src, uint32_t n, int shift, uint32_t *__restrict__ counts) {
  constexpr int R = 1 << DB;
  __shared__ uint32_t s_h[kWaves][R];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < kWaves * R; i += kThreads) (&s_h[0][0])[i] = 0;
  const uint32_t base = blockIdx.x * kTile;
  K key[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = elem_index(base, w, i, lane);
    key[i] = K(0);
    if (idx < n) {
      VT unused;
      src.get(idx, key[i], unused);
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = elem_index(base, w, i, lane);
    const uint32_t d = idx < n ? uint32_t((key[i] >> shift) & (R - 1)) : ~0u;
    const uint32_t dp = __shfl_up(d, 1, 64);
    const bool head = lane == 0 || d != dp;
    const uint64_t heads = __ballot(head);
    if (head && d != ~0u) {
      const uint64_t after = lane == 63 ? 0ull : heads >> (lane + 1);
      const uint32_t len = after ? uint32_t(__builtin_ctzll(after)) + 1u : uint32_t(64 - lane);
      atomicAdd(&s_h[w][d], len);
    }
  }
  __syncthreads();
  for (int d = tid; d < R; d += kThreads) {
    uint32_t c = 0;
#pragma unroll
    for (int ww = 0; ww < kWaves; ww++) c += s_h[ww][d];
    counts[size_t(blockIdx.x) * R + d] = c;
  }
}

// Group g of kGroup tiles: counts[t][d] <- exclusive prefix within the group,
// gsum[g][d] <- group total.
template <int DB>
__global__ void __launch_bounds__(256)
    k_scan_a(uint32_t *__restrict__ counts, uint32_t tiles, uint32_t *__restrict__ gsum) {
  constexpr int R = 1 << DB;
  const uint32_t g = blockIdx.x;
  const uint32_t t0 = g * kGroup, t1 = min(tiles, t0 + kGroup);
  // blockIdx.y: a 256-digit slice (grid y = R / 256), else the block loops
  for (uint32_t d = blockIdx.y * 256 + threadIdx.x; d < uint32_t(R); d += 256 * gridDim.y) {
    uint32_t v[kGroup];
#pragma unroll
    for (int i = 0; i < kGroup; i++) v[i] = (t0 + i < t1) ? counts[size_t(t0 + i) * R + d] : 0u;
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < kGroup; i++) {
      if (t0 + i < t1) counts[size_t(t0 + i) * R + d] = run;
      run += v[i];
    }
    gsum[size_t(g) * R + d] = run;
  }
}

// One workgroup: gsum[g][d] <- exclusive prefix over groups, dbase[d] <-
// exclusive prefix of the digit totals.  Thread t owns the Q = R/256
// consecutive digits [t·Q, (t+1)·Q).
template <int DB>
__global__ void __launch_bounds__(256)
    k_scan_b(uint32_t *__restrict__ gsum, uint32_t groups, uint32_t *__restrict__ dbase) {
  constexpr int R = 1 << DB, Q = R / 256;
  __shared__ uint32_t s_tmp[kWaves];
  uint32_t tot[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const uint32_t d = threadIdx.x * Q + q;
    uint32_t run = 0;
    for (uint32_t g0 = 0; g0 < groups; g0 += 16) {
      uint32_t v[16];
#pragma unroll
      for (int i = 0; i < 16; i++) v[i] = (g0 + i < groups) ? gsum[size_t(g0 + i) * R + d] : 0u;
#pragma unroll
      for (int i = 0; i < 16; i++) {
        if (g0 + i < groups) gsum[size_t(g0 + i) * R + d] = run;
        run += v[i];
      }
    }
    tot[q] = run;
  }
  uint32_t mine = 0;
#pragma unroll
  for (int q = 0; q < Q; q++) mine += tot[q];
  uint32_t pre = block_excl_scan(mine, s_tmp);
#pragma unroll
  for (int q = 0; q < Q; q++) {
    dbase[threadIdx.x * Q + q] = pre;
    pre += tot[q];
  }
}

// k_scan_b over 1024 threads: P = 1024 / R threads per digit, each over a
// contiguous slice of the groups (a first pass sums the slice, a second
// writes its exclusive prefixes from the slice's base): two dependent load
// rounds instead of one per 16 groups.
template <int DB>
__global__ void __launch_bounds__(1024)
    k_scan_b_wide(uint32_t *__restrict__ gsum, uint32_t groups, uint32_t *__restrict__ dbase) {
  constexpr int R = 1 << DB, P = 1024 / R;
  static_assert(P >= 1 && 1024 % R == 0, "k_scan_b_wide: at most 1024 digits");
  __shared__ uint32_t s_part[P][R];
  __shared__ uint32_t s_tmp[16];
  const uint32_t d = threadIdx.x % R, q = threadIdx.x / R;
  const uint32_t per = (groups + P - 1) / P;
  const uint32_t g0 = min(groups, q * per), g1 = min(groups, g0 + per);
  uint32_t sum = 0;
  for (uint32_t g = g0; g < g1; g += 16) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = (g + i < g1) ? gsum[size_t(g + i) * R + d] : 0u;
#pragma unroll
    for (int i = 0; i < 16; i++) sum += v[i];
  }
  s_part[q][d] = sum;
  __syncthreads();
  uint32_t run = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < P; i++) {
    if (uint32_t(i) < q) run += s_part[i][d];
    tot += s_part[i][d];
  }
  for (uint32_t g = g0; g < g1; g += 16) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = (g + i < g1) ? gsum[size_t(g + i) * R + d] : 0u;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      if (g + i < g1) gsum[size_t(g + i) * R + d] = run;
      run += v[i];
    }
  }
  // dbase: exclusive scan of the digit totals over threads q == 0 (tid = d)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = q == 0 ? tot : 0u;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  if (q == 0 && d < R) {
    uint32_t pre = 0;
    for (int i = 0; i < w; i++) pre += s_tmp[i];
    dbase[d] = pre + x - tot;
  }
}

// the second scan level: k_scan_b_wide up to 1024 digits (the 256-thread
// k_scan_b took 5.9 against 5.0 us for 8-bit digits, 9.5 against 6.3 for 9)
template <int DB>
inline void scan_b(uint32_t *gsum, uint32_t groups, uint32_t *dbase, hipStream_t s) {
  if constexpr (DB <= 10)
    k_scan_b_wide<DB><<<1, 1024, 0, s>>>(gsum, groups, dbase);
  else
    k_scan_b<DB><<<1, 256, 0, s>>>(gsum, groups, dbase);
}

// Small sorts (tiles <= kFusedMaxTiles): one 1024-thread workgroup does both
// scan levels -- 4 threads per digit, each over a contiguous quarter of the
// tiles (gsum[q][d] <- quarter prefix, dbase[d] <- digit base).
constexpr int kFusedMaxTiles = 1024;
template <int DB>
__global__ void __launch_bounds__(1024)
    k_scan_fused(uint32_t *__restrict__ counts, uint32_t tiles, uint32_t per,
                 uint32_t *__restrict__ gsum, uint32_t *__restrict__ dbase) {
  constexpr uint32_t R = 1u << DB;  // <= 256: threads d >= R only join the barriers
  __shared__ uint32_t s_part[4][256];
  __shared__ uint32_t s_tmp[4];
  const uint32_t d = threadIdx.x & 255, q = threadIdx.x >> 8;
  const uint32_t t0 = q * per, t1 = d < R ? min(tiles, t0 + per) : t0;
  uint32_t run = 0;
  for (uint32_t t = t0; t < t1; t += 16) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = (t + i < t1) ? counts[size_t(t + i) * R + d] : 0u;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      if (t + i < t1) counts[size_t(t + i) * R + d] = run;
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
  if (d < R) gsum[q * R + d] = qpre;
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
  if (q == 0 && d < R) {
    uint32_t pre = 0;
    for (int i = 0; i < w; i++) pre += s_tmp[i];
    dbase[d] = pre + x - tot;
  }
}

// Exclusive scan of one value per thread over a TH-thread block.
template <int TH>
__device__ __forceinline__ uint32_t block_excl_scan_t(uint32_t v, uint32_t *s_tmp) {
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
  for (int i = 0; i < TH / 64; i++)
    if (i < w) pre += s_tmp[i];
  __syncthreads();
  return pre + x - v;
}

// Value stores of the scatter: as they are, or (the per-key sequences) a
// packed 32-bit dot src << sb | seq widened to the u64 dot src << 56 | seq
template <class VT>
struct StoreVal {
  static constexpr int kBytes = sizeof(VT);
  VT *p;
  __device__ __forceinline__ void operator()(uint32_t o, VT v) const { p[o] = v; }
};
struct StoreUnpackDot {
  static constexpr int kBytes = 8;
  uint64_t *p;
  int sb;
  __device__ __forceinline__ void operator()(uint32_t o, uint32_t v) const {
    p[o] = (uint64_t(v >> sb) << 56) | (v & ((1u << sb) - 1));
  }
};

// The scatter of one pass over a tile of kTile elements, TH threads of kTile /
// TH items (512 by default: twice the waves per tile for the same LDS, so a
// CU holds 24 instead of 12 waves of the u64-value scatter).  Wave
// w owns the contiguous sub-tile [w·64·IT, (w+1)·64·IT), so (wave, item,
// lane) order is input order and the scatter stays stable; the tile digit
// counts (k_up) do not depend on TH.
template <class K, class VT, int DB, class Src, int TH = kThreads, class St = StoreVal<VT>>
__global__ void __launch_bounds__(TH)
    k_down(Src src, K *__restrict__ kout, St vout, uint32_t n, int shift,
           const uint32_t *__restrict__ counts, const uint32_t *__restrict__ gsum,
           uint32_t gsize, const uint32_t *__restrict__ dbase) {
  // digits per thread in the tile-wide scan: Q = R / TH, or one digit for
  // the first R threads when R < TH
  constexpr int R = 1 << DB, Q = R >= TH ? R / TH : 1;
  constexpr int IT = kTile / TH, WV = TH / 64;
  __shared__ K s_k[kTile];
  __shared__ VT s_v[kTile];
  __shared__ uint32_t s_wh[WV][R];
  __shared__ uint32_t s_dex[R];
  __shared__ uint32_t s_gb[R];
  __shared__ uint32_t s_tmp[WV];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t tile = blockIdx.x;
  const uint32_t base = tile * kTile;
  auto eidx = [&](int i) {
    return base + uint32_t(w) * 64 * IT + uint32_t(i) * 64 + uint32_t(lane);
  };
  for (int i = tid; i < WV * R; i += TH) (&s_wh[0][0])[i] = 0;
  // global offset of this tile's digit runs (independent of the items)
  for (int d = tid; d < R; d += TH)
    s_gb[d] = dbase[d] + gsum[size_t(tile / gsize) * R + d] + counts[size_t(tile) * R + d];
  K key[IT];
  VT val[IT];
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const uint32_t idx = eidx(i);
    const bool valid = idx < n;
    key[i] = K(0);
    val[i] = VT(0);
    if (valid) src.get(idx, key[i], val[i]);
  }
  __syncthreads();
  const uint64_t lt = (uint64_t(1) << lane) - 1;
  uint32_t rank[IT];
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const uint32_t idx = eidx(i);
    const bool valid = idx < n;
    const uint32_t d = uint32_t((key[i] >> shift) & (R - 1));
    const uint64_t peers = match_digit<DB>(d, valid);
    uint32_t b0 = 0;
    if (valid) b0 = s_wh[w][d];
    if (valid && (peers & lt) == 0) s_wh[w][d] = b0 + uint32_t(__popcll(peers));
    rank[i] = b0 + uint32_t(__popcll(peers & lt));
  }
  __syncthreads();
  // per digit: the waves' exclusive prefix (stability: wave order = input
  // order), then the tile-wide exclusive prefix over digits; thread t owns
  // the Q consecutive digits [t·Q, (t+1)·Q)
  uint32_t cnt[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const int d = tid * Q + q;
    uint32_t c0 = 0;
    if (d < R) {
#pragma unroll
      for (int ww = 0; ww < WV; ww++) {
        const uint32_t c = s_wh[ww][d];
        s_wh[ww][d] = c0;
        c0 += c;
      }
    }
    cnt[q] = c0;
  }
  uint32_t mine = 0;
#pragma unroll
  for (int q = 0; q < Q; q++) mine += cnt[q];
  uint32_t lpre = block_excl_scan_t<TH>(mine, s_tmp);
#pragma unroll
  for (int q = 0; q < Q; q++) {
    if (tid * Q + q < R) s_dex[tid * Q + q] = lpre;
    lpre += cnt[q];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const uint32_t idx = eidx(i);
    if (idx < n) {
      const uint32_t d = uint32_t((key[i] >> shift) & (R - 1));
      const uint32_t pos = s_dex[d] + s_wh[w][d] + rank[i];
      s_k[pos] = key[i];
      s_v[pos] = val[i];
    }
  }
  __syncthreads();
  const uint32_t tile_n = min(uint32_t(kTile), n - base);
#pragma unroll 4
  for (uint32_t j = tid; j < tile_n; j += TH) {
    const K k = s_k[j];
    const uint32_t d = uint32_t((k >> shift) & (R - 1));
    const uint32_t o = s_gb[d] + (j - s_dex[d]);
    kout[o] = k;
    vout(o, s_v[j]);
  }
}


// Pass inputs: a source yields the (key, value) of input element idx.
// ArraySrc reads the arrays (IOTA: the value is the position); callers may
// pass their own source for pass 0 and skip materialising its input.
template <class K, class VT, bool IOTA>
struct ArraySrc {
  const K *k;
  const VT *v;
  __device__ __forceinline__ void get(uint32_t idx, K &key, VT &val) const {
    key = k[idx];
    val = IOTA ? VT(idx) : v[idx];
  }
};

// one LSD pass over DB bits at `shift`, input from `src`
template <class K, class VT, int DB, class Src, class St = StoreVal<VT>>
void sort_pass(const Src &src, K *ko, St vo, size_t n, int shift, uint32_t tiles,
               uint32_t groups, uint32_t *counts, uint32_t *gsum, uint32_t *dbase, hipStream_t s,
               bool probe, bool have_counts = false) {
  if (!have_counts)  // (else the producer of the input wrote the tile counts)
    k_up<K, VT, DB, Src><<<tiles, kThreads, 0, s>>>(src, uint32_t(n), shift, counts);
  uint32_t gsize = kGroup;
  if (DB <= 8 && tiles <= kFusedMaxTiles) {
    gsize = (tiles + 3) / 4;
    k_scan_fused<DB><<<1, 1024, 0, s>>>(counts, tiles, gsize, gsum, dbase);
  } else {
    k_scan_a<DB><<<groups, 256, 0, s>>>(counts, tiles, gsum);
    scan_b<DB>(gsum, groups, dbase, s);
  }
  // the 512-thread scatter (k_down).  Measured on C4, u64 values: 613 -> 592
  // us per 100M-element pass against 256 threads.  (Tried for the key-order
  // path's 12-B values: 1024 threads, 32 waves per CU instead of 16 -- KeyDeps
  // views 6.07 against 6.09 ms, no different, r05st.)
  constexpr int down_th = 512;
  auto down = [&](auto kern, int th) {
    if (!probe) {
      kern<<<tiles, th, 0, s>>>(src, ko, vo, uint32_t(n), shift, counts, gsum, gsize, dbase);
    } else {
      // algorithmic traffic of a key+value scatter pass: read and write every
      // pair once
      // one probe name per kernel instantiation, as rocprof reports them
      const char *name = sizeof(K) == 8 ? "sort_scatter_u64"
                         : sizeof(VT) == 8 ? "sort_scatter_dots"
                         : sizeof(VT) == 12 ? "sort_scatter_v3" : "sort_scatter";
      probed_launch(name, double(n) * (2.0 * sizeof(K) + sizeof(VT) + St::kBytes), kern, dim3(tiles),
                    dim3(th), s, src, ko, vo, uint32_t(n), shift, (const uint32_t *)counts,
                    (const uint32_t *)gsum, gsize, (const uint32_t *)dbase);
    }
  };
  if (down_th == 512)
    down(k_down<K, VT, DB, Src, 512, St>, 512);
  else
    down(k_down<K, VT, DB, Src, kThreads, St>, kThreads);
}

template <class K, class VT, int DB, class Src0>
void sort_passes(const Src0 &src0, bool probe0, K *ka, VT *va, K *kb, VT *vb, bool alias_a,
                 size_t n, int passes, int db, SortWorkspace &ws, hipStream_t s, K **kout,
                 VT **vout, bool counts0 = false) {
  const uint32_t tiles = uint32_t((n + kTile - 1) / kTile);
  const uint32_t groups = (tiles + kGroup - 1) / kGroup;
  ws.prepare(tiles, passes, s);
  const uint32_t R = 1u << db;
  uint32_t *counts = ws.meta.get();
  uint32_t *gsum = counts + size_t(tiles) * R;
  uint32_t *dbase = gsum + size_t(std::max<uint32_t>(groups, 4)) * R;
  K *ko = alias_a ? kb : ka;
  VT *vo = alias_a ? vb : va;
  sort_pass<K, VT, DB, Src0>(src0, ko, StoreVal<VT>{vo}, n, 0, tiles, groups, counts, gsum, dbase,
                            s, probe0, counts0);
  const K *ki = ko;
  const VT *vi = vo;
  for (int p = 1; p < passes; p++) {
    K *kn = ko == ka ? kb : ka;
    VT *vn = ko == ka ? vb : va;
    sort_pass<K, VT, DB, ArraySrc<K, VT, false>>(ArraySrc<K, VT, false>{ki, vi}, kn,
                                                 StoreVal<VT>{vn}, n, db * p, tiles, groups,
                                                 counts, gsum, dbase, s, true);
    ko = kn;
    vo = vn;
    ki = ko;
    vi = vo;
  }
  *kout = const_cast<K *>(ki);
  *vout = const_cast<VT *>(vi);
}

// sort_pairs with pass 0 reading `src` (n elements); result in (ka, va) or
// (kb, vb).  Digit plan as sort_pairs.
template <class K, class VT, class Src>
void sort_pairs_src(const Src &src, K *ka, VT *va, K *kb, VT *vb, size_t n, int key_bits,
                    SortWorkspace &ws, hipStream_t s, K **kout, VT **vout) {
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "sort: too many elements (>= 2^30)");
  int db = 8;
  int passes = std::max(1, (key_bits + db - 1) / db);
  if (passes > int(sizeof(K))) passes = int(sizeof(K));
  if (n == 0) {
    *kout = ka;
    *vout = va;
    return;
  }
  sort_passes<K, VT, 8, Src>(src, true, ka, va, kb, vb, false, n, passes, db, ws, s, kout, vout);
}

// sort_pairs of (ka, va) whose pass-0 tile digit counts (8-bit digits at
// shift 0, tiles of kTile consecutive elements, counts[tile][256] in
// ws.meta after ws.prepare(tiles)) were written by the kernel that produced
// the input; result in (ka, va) or (kb, vb).
// The digit plan: the fewest passes of at most 8 bits, the bits spread evenly
// over them (20-bit keys: 7 + 7 + 6 instead of 8 + 8 + 4).  A narrower digit
// means fewer ballots per item in k_down and longer same-digit runs per tile
// (32 instead of 16 elements on average at 7 bits: 128-B writes instead of
// 64-B ones).
inline int sort_digit_bits(int key_bits, int key_bytes) {
  int passes = std::max(1, (key_bits + 7) / 8);
  if (passes > key_bytes) passes = key_bytes;
  const int db = (key_bits + passes - 1) / passes;
  return db >= 8 ? 8 : db <= 6 ? 6 : 7;
}

template <class K, class VT>
void sort_pairs_counted(K *ka, VT *va, K *kb, VT *vb, size_t n, int key_bits, SortWorkspace &ws,
                        hipStream_t s, K **kout, VT **vout, int db) {
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "sort: too many elements (>= 2^30)");
  const int passes = std::max(1, (key_bits + db - 1) / db);
  if (n == 0) {
    *kout = ka;
    *vout = va;
    return;
  }
  using Src = ArraySrc<K, VT, false>;
  if (db == 6)
    sort_passes<K, VT, 6, Src>(Src{ka, va}, true, ka, va, kb, vb, true, n, passes, 6, ws, s, kout,
                               vout, true);
  else if (db == 7)
    sort_passes<K, VT, 7, Src>(Src{ka, va}, true, ka, va, kb, vb, true, n, passes, 7, ws, s, kout,
                               vout, true);
  else
    sort_passes<K, VT, 8, Src>(Src{ka, va}, true, ka, va, kb, vb, true, n, passes, 8, ws, s, kout,
                               vout, true);
}

// sort_pairs_counted with pass 0 reading `src` (whose tile digit counts the
// caller wrote, as for sort_pairs_counted): the producer of the sort input is
// folded into the first scatter; result in (ka, va) or (kb, vb).
template <class K, class VT, class Src>
void sort_pairs_counted_src(const Src &src, K *ka, VT *va, K *kb, VT *vb, size_t n, int key_bits,
                            SortWorkspace &ws, hipStream_t s, K **kout, VT **vout, int db) {
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "sort: too many elements (>= 2^30)");
  const int passes = std::max(1, (key_bits + db - 1) / db);
  if (n == 0) {
    *kout = ka;
    *vout = va;
    return;
  }
  if (db == 6)
    sort_passes<K, VT, 6, Src>(src, true, ka, va, kb, vb, false, n, passes, 6, ws, s, kout, vout,
                               true);
  else if (db == 7)
    sort_passes<K, VT, 7, Src>(src, true, ka, va, kb, vb, false, n, passes, 7, ws, s, kout, vout,
                               true);
  else
    sort_passes<K, VT, 8, Src>(src, true, ka, va, kb, vb, false, n, passes, 8, ws, s, kout, vout,
                               true);
}

}  // namespace
}  // namespace fh
