// sort.hip -- onesweep LSD radix sort for gfx950 (see sort.h).
#include "sort.h"

namespace fh {
namespace {

constexpr int kWaves = kSortThreads / 64;
constexpr uint32_t kAgg = 1u << 30;
constexpr uint32_t kInc = 2u << 30;
constexpr uint32_t kCnt = (1u << 30) - 1;
constexpr int kHistWords = 8 * 256;
constexpr int kCtrWords = 16;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive scan of one value per thread over a 256-thread block.
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

template <class K>
__global__ void __launch_bounds__(256) k_hist(const K *__restrict__ keys, uint32_t n,
                                              int passes, uint32_t *__restrict__ ghist) {
  __shared__ uint32_t h[kHistWords];
  for (int i = threadIdx.x; i < passes * 256; i += 256) h[i] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    K k = keys[i];
    for (int p = 0; p < passes; p++)
      atomicAdd(&h[p * 256 + uint32_t((k >> (8 * p)) & 255)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < passes * 256; i += 256)
    if (h[i]) atomicAdd(&ghist[i], h[i]);
}

template <class K, bool IOTA>
__global__ void __launch_bounds__(256)
    k_onesweep(const K *__restrict__ kin, const uint32_t *__restrict__ vin,
               K *__restrict__ kout, uint32_t *__restrict__ vout, uint32_t n, int shift,
               const uint32_t *__restrict__ ghist, uint32_t *status, uint32_t *ctr) {
  __shared__ K s_k[kSortTile];
  __shared__ uint32_t s_v[kSortTile];
  __shared__ uint32_t s_wh[kWaves][256];
  __shared__ uint32_t s_dex[256];
  __shared__ uint32_t s_gb[256];
  __shared__ uint32_t s_tmp[kWaves];
  __shared__ uint32_t s_tile;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(&ctr[0], 1u);
  for (int i = tid; i < kWaves * 256; i += 256) (&s_wh[0][0])[i] = 0;
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t base = tile * kSortTile;
  const uint64_t lt = (uint64_t(1) << lane) - 1;

  K key[kSortItems];
  uint32_t val[kSortItems];
  uint32_t dig[kSortItems];
  uint32_t rank[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kSortItems + i * 64 + lane;
    const bool valid = idx < n;
    key[i] = valid ? kin[idx] : K(0);
    val[i] = IOTA ? idx : (valid ? vin[idx] : 0u);
    dig[i] = valid ? uint32_t((key[i] >> shift) & 255) : 256u;
  }
  // Stable rank within the wave's sub-tile: order (item round, lane).
#pragma unroll
  for (int i = 0; i < kSortItems; i++) {
    const uint32_t d = dig[i];
    uint64_t peers = __ballot(d < 256);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const bool bit = (d >> b) & 1;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    uint32_t b0 = 0;
    if (d < 256) b0 = s_wh[w][d];
    if (d < 256 && (peers & lt) == 0) s_wh[w][d] = b0 + uint32_t(__popcll(peers));
    rank[i] = b0 + uint32_t(__popcll(peers & lt));
  }
  __syncthreads();

  // Per digit (one per thread): exclusive prefix across waves, tile count.
  const uint32_t d = tid;
  uint32_t run = 0;
#pragma unroll
  for (int ww = 0; ww < kWaves; ww++) {
    const uint32_t c = s_wh[ww][d];
    s_wh[ww][d] = run;
    run += c;
  }
  const uint32_t cnt = run;

  // Decoupled look-back over tiles for this digit.
  uint32_t excl = 0;
  uint32_t *my = status + size_t(tile) * 256 + d;
  if (tile == 0) {
    st_agent(my, kInc | cnt);
  } else {
    st_agent(my, kAgg | cnt);
    int t = int(tile) - 1;
    uint32_t spins = 0;
    while (t >= 0) {
      const uint32_t sv = ld_agent(status + size_t(t) * 256 + d);
      const uint32_t flag = sv & ~kCnt;
      if (flag == kInc) {
        excl += sv & kCnt;
        break;
      }
      if (flag == kAgg) {
        excl += sv & kCnt;
        t--;
        continue;
      }
      if (++spins > (1u << 24)) {  // bounded: report instead of hanging
        atomicOr(&ctr[8], 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    st_agent(my, kInc | (excl + cnt));
  }

  const uint32_t gpre = block_excl_scan(ghist[d], s_tmp);
  const uint32_t lpre = block_excl_scan(cnt, s_tmp);
  s_gb[d] = gpre + excl;
  s_dex[d] = lpre;
  __syncthreads();

#pragma unroll
  for (int i = 0; i < kSortItems; i++) {
    const uint32_t dd = dig[i];
    if (dd < 256) {
      const uint32_t pos = s_dex[dd] + s_wh[w][dd] + rank[i];
      s_k[pos] = key[i];
      s_v[pos] = val[i];
    }
  }
  __syncthreads();
  const uint32_t tile_n = min(uint32_t(kSortTile), n - base);
  for (uint32_t j = tid; j < tile_n; j += 256) {
    const K k = s_k[j];
    const uint32_t dd = uint32_t((k >> shift) & 255);
    const uint32_t o = s_gb[dd] + (j - s_dex[dd]);
    kout[o] = k;
    vout[o] = s_v[j];
  }
}

}  // namespace

size_t SortWorkspace::meta_words(size_t n, int passes) const {
  const size_t tiles = (n + kSortTile - 1) / kSortTile;
  return kHistWords + kCtrWords + size_t(passes) * tiles * 256;
}

template <class K>
void sort_pairs(const K *keys_in, const uint32_t *vals_in, K *ka, uint32_t *va, K *kb,
                uint32_t *vb, size_t n, int key_bits, SortWorkspace &ws, hipStream_t s,
                K **kout, uint32_t **vout) {
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "sort: too many elements (>= 2^30)");
  int passes = (key_bits + 7) / 8;
  if (passes < 1) passes = 1;
  if (passes > int(sizeof(K))) passes = int(sizeof(K));
  if (n == 0) {
    *kout = ka;
    *vout = va;
    return;
  }
  const size_t words = ws.meta_words(n, passes);
  uint32_t *meta = ws.meta.ensure(words);
  FH_HIP(hipMemsetAsync(meta, 0, words * sizeof(uint32_t), s));
  uint32_t *ghist = meta;
  uint32_t *ctr = meta + kHistWords;
  uint32_t *status = ctr + kCtrWords;
  const size_t tiles = (n + kSortTile - 1) / kSortTile;
  k_hist<K><<<grid_for(n, 256, 1024), 256, 0, s>>>(keys_in, uint32_t(n), passes, ghist);
  const K *ki = keys_in;
  const uint32_t *vi = vals_in;
  // never write pass 0 over its own input
  const bool alias_a = (const void *)keys_in == (const void *)ka ||
                       (vals_in && (const void *)vals_in == (const void *)va);
  K *ko = alias_a ? kb : ka;
  uint32_t *vo = alias_a ? vb : va;
  for (int p = 0; p < passes; p++) {
    uint32_t *st = status + size_t(p) * tiles * 256;
    // each pass gets its own ticket counter ctr[p] ... use ctr[p] via offset
    if (p == 0 && vals_in == nullptr)
      k_onesweep<K, true><<<unsigned(tiles), 256, 0, s>>>(
          ki, nullptr, ko, vo, uint32_t(n), 8 * p, ghist + 256 * p, st, ctr + 0);
    else
      k_onesweep<K, false><<<unsigned(tiles), 256, 0, s>>>(
          ki, vi, ko, vo, uint32_t(n), 8 * p, ghist + 256 * p, st, ctr + 0);
    // reset the ticket for the next pass (error word ctr[8] is kept)
    FH_HIP(hipMemsetAsync(ctr, 0, sizeof(uint32_t), s));
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
  *vout = const_cast<uint32_t *>(vi);
}

template void sort_pairs<uint32_t>(const uint32_t *, const uint32_t *, uint32_t *,
                                   uint32_t *, uint32_t *, uint32_t *, size_t, int,
                                   SortWorkspace &, hipStream_t, uint32_t **, uint32_t **);
template void sort_pairs<uint64_t>(const uint64_t *, const uint32_t *, uint64_t *,
                                   uint32_t *, uint64_t *, uint32_t *, size_t, int,
                                   SortWorkspace &, hipStream_t, uint64_t **, uint32_t **);

}  // namespace fh
