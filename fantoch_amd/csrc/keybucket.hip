// keybucket.hip -- the two-launch single-view KeyDeps path (see keybucket.h).
//
// Why two launches and no radix passes: a 1M-command batch is latency bound on
// a 256-CU part, so the path is cut at the one exchange it needs (commands of
// one key meet in one workgroup).  k_kb_partition streams the batch once
// (16 B/command) and leaves every tile partitioned by bucket in place, with
// coalesced writes; k_kb_order gathers a bucket's runs from all tiles (tile
// order = arrival order, so no stable global sort is needed), orders them by
// slot in LDS and writes the per-key sequence and the dependencies.
#include <algorithm>
#include <cmath>

#include "keybucket.h"

namespace fh {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kItems = 8;
constexpr int kTile = kThreads * kItems;  // commands per partition tile
constexpr int kChunk = 2048;              // bucket elements staged in LDS at once
constexpr int kMaxTiles = 512;   // batches up to 2^20 commands
constexpr int kSlotBits = 10;             // at most 1024 keys per bucket

// Lanes whose `bits`-bit value equals this lane's (valid lanes only).
__device__ __forceinline__ uint64_t match_bits(uint32_t d, bool valid, int bits) {
  uint64_t peers = __ballot(valid);
  for (int b = 0; b < bits; b++) {
    const bool bit = (d >> b) & 1u;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  return peers;
}

// Exclusive scan of one value per thread over the block; *total = block sum.
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t *s_tmp, uint32_t *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kWaves; i++) {
    const uint32_t s = s_tmp[i];
    pre += i < w ? s : 0u;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// ---------------------------------------------------------------- partition
// One 4096-command tile per workgroup.  Item i of lane l in wave w is command
// base + w*1024 + i*64 + l, so (w, i, l) order is arrival order and the
// ballot-matched ranks give a stable partition.
template <int BB>
__global__ void __launch_bounds__(kThreads)
    k_kb_partition(uint32_t n, int bb, int hb, int vb, uint32_t kmul, uint32_t kmask,
                   const uint32_t *__restrict__ key32, const uint64_t *__restrict__ dot,
                   uint32_t *__restrict__ part, uint16_t *__restrict__ toff,
                   unsigned long long *__restrict__ frontier,
                   unsigned long long *__restrict__ excount) {
  constexpr int BMAX = 1 << BB;
  constexpr int RB = BMAX / kThreads;  // buckets per thread in the scan
  __shared__ uint32_t s_wh[kWaves][BMAX];
  __shared__ uint32_t s_dex[BMAX];
  __shared__ uint32_t s_out[kTile];
  __shared__ unsigned long long s_mx[256];
  __shared__ uint32_t s_nc[256];
  __shared__ uint32_t s_tmp[kWaves];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t B = 1u << bb;
  for (int i = tid; i < kWaves * BMAX; i += kThreads) (&s_wh[0][0])[i] = 0;
  s_mx[tid] = 0;
  s_nc[tid] = 0;
  const uint32_t base = blockIdx.x * kTile;
  const uint32_t tile_n = min(uint32_t(kTile), n - base);
  uint32_t pk[kItems], bkt[kItems], rank[kItems];
  uint64_t d[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + lane;
    pk[i] = idx < n ? key32[idx] : 0u;
    d[i] = idx < n ? dot[idx] : 0ull;
  }
  __syncthreads();
  const uint64_t lt = (uint64_t(1) << lane) - 1;
  const uint32_t smask = (1u << hb) - 1;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + lane;
    const bool valid = idx < n;
    if (valid) {
      // executed clock (AEClock::add for every executed dot, tarjan.rs:296)
      atomicMax(&s_mx[d[i] >> 56], (unsigned long long)(d[i] & 0x00FFFFFFFFFFFFFFull));
      atomicAdd(&s_nc[d[i] >> 56], 1u);
    }
    const uint32_t p = (pk[i] * kmul) & kmask;
    const uint32_t bk = p >> hb;
    const uint64_t peers = match_bits(bk, valid, bb);
    const uint32_t b0 = valid ? s_wh[w][bk] : 0u;
    if (valid && (peers & lt) == 0) s_wh[w][bk] = b0 + uint32_t(__popcll(peers));
    rank[i] = b0 + uint32_t(__popcll(peers & lt));
    bkt[i] = bk;
    pk[i] = ((p & smask) << vb) | idx;
  }
  __syncthreads();
  // per-bucket tile counts -> per-wave exclusive offsets and bucket starts
  uint32_t loc[RB];
  uint32_t sum = 0;
#pragma unroll
  for (int r = 0; r < RB; r++) {
    const uint32_t bk = uint32_t(tid) * RB + r;
    uint32_t c = 0;
    if (bk < B) {
#pragma unroll
      for (int ww = 0; ww < kWaves; ww++) {
        const uint32_t cw = s_wh[ww][bk];
        s_wh[ww][bk] = c;
        c += cw;
      }
    }
    loc[r] = c;
    sum += c;
  }
  uint32_t tot;
  uint32_t pre = block_scan(sum, s_tmp, &tot);
  uint16_t *row = toff + size_t(blockIdx.x) * (B + 1);
#pragma unroll
  for (int r = 0; r < RB; r++) {
    const uint32_t bk = uint32_t(tid) * RB + r;
    if (bk < B) {
      s_dex[bk] = pre;
      row[bk] = uint16_t(pre);
    }
    pre += loc[r];
  }
  if (tid == 0) row[B] = uint16_t(tile_n);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + lane;
    if (idx < n) s_out[s_dex[bkt[i]] + s_wh[w][bkt[i]] + rank[i]] = pk[i];
  }
  __syncthreads();
  if (tile_n == uint32_t(kTile)) {
    uint4 *dst = reinterpret_cast<uint4 *>(part + base);
    const uint4 *src = reinterpret_cast<const uint4 *>(s_out);
#pragma unroll
    for (int j = tid; j < kTile / 4; j += kThreads) dst[j] = src[j];
  } else {
    for (uint32_t j = tid; j < tile_n; j += kThreads) part[base + j] = s_out[j];
  }
  if (s_nc[tid]) {
    atomicMax(&frontier[tid], s_mx[tid]);
    atomicAdd(&excount[tid], (unsigned long long)s_nc[tid]);
  }
}

// ---------------------------------------------------------------- order
// Helpers of k_kb_order (all inlined; LDS arrays passed explicitly).

// first tile run holding bucket element q: s_rs[t] <= q < s_rs[t + 1]
__device__ __forceinline__ uint32_t run_of(const uint32_t *s_rs, uint32_t tiles, uint32_t q) {
  uint32_t tl = 0, th = tiles;
  while (th - tl > 1) {
    const uint32_t mid = (tl + th) >> 1;
    if (s_rs[mid] <= q) tl = mid;
    else th = mid;
  }
  return tl;
}

// bucket elements [c0, c1) -> dst[0, c1 - c0), G consecutive ones per thread
template <int G>
__device__ __forceinline__ void gather_runs(const uint32_t *__restrict__ part,
                                            const uint32_t *s_rs, const uint32_t *s_src,
                                            uint32_t tiles, uint32_t c0, uint32_t c1,
                                            uint32_t *dst) {
  const uint32_t q0 = c0 + threadIdx.x * G;
  if (q0 >= c1) return;
  uint32_t t = run_of(s_rs, tiles, q0);
  uint32_t v[G];
#pragma unroll
  for (int g = 0; g < G; g++) {
    const uint32_t q = q0 + g;
    v[g] = 0;
    if (q < c1) {
      while (s_rs[t + 1] <= q) t++;
      v[g] = part[s_src[t] + (q - s_rs[t])];
    }
  }
#pragma unroll
  for (int g = 0; g < G; g++)
    if (q0 + g < c1) dst[q0 + g - c0] = v[g];
}

// One stable LDS pass over src[0, c) by slot bits [shift, shift + nbits).
// Element q is item (q / 64) % G of lane q % 64 in wave q / (64 G), so
// (wave, item, lane) order is element order and ballot ranks keep it stable.
template <int G, int ND>
__device__ __forceinline__ void slot_sort_pass(const uint32_t *src, uint32_t *dst, uint32_t c,
                                               int vb, int shift, int nbits,
                                               uint32_t (*s_h)[ND], uint32_t *s_db) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t lt = (uint64_t(1) << lane) - 1;
  for (int i = tid; i < kWaves * ND; i += kThreads) (&s_h[0][0])[i] = 0;
  __syncthreads();
  uint32_t e[G], rk[G];
  const uint32_t dm = (1u << nbits) - 1;
#pragma unroll
  for (int i = 0; i < G; i++) {
    const uint32_t q = uint32_t(w) * 64 * G + uint32_t(i) * 64 + lane;
    const bool valid = q < c;
    e[i] = valid ? src[q] : 0u;
    const uint32_t d = ((e[i] >> vb) >> shift) & dm;
    const uint64_t peers = match_bits(d, valid, nbits);
    const uint32_t b0 = valid ? s_h[w][d] : 0u;
    if (valid && (peers & lt) == 0) s_h[w][d] = b0 + uint32_t(__popcll(peers));
    rk[i] = b0 + uint32_t(__popcll(peers & lt));
  }
  __syncthreads();
  if (w == 0) {
    uint32_t tot = 0;
    if (lane < ND) {
#pragma unroll
      for (int ww = 0; ww < kWaves; ww++) {
        const uint32_t t = s_h[ww][lane];
        s_h[ww][lane] = tot;
        tot += t;
      }
    }
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < ND; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane < ND) s_db[lane] = x - tot;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < G; i++) {
    const uint32_t q = uint32_t(w) * 64 * G + uint32_t(i) * 64 + lane;
    if (q < c) {
      const uint32_t d = ((e[i] >> vb) >> shift) & dm;
      dst[s_db[d] + s_h[w][d] + rk[i]] = e[i];
    }
  }
  __syncthreads();
}

// One bucket per workgroup.  The bucket's commands are the concatenation of
// its run in every tile, in tile order: that is arrival order.  Chunks of
// kChunk are staged in LDS and stably sorted by slot (key) with two 5-bit
// passes (wave64 ballot ranks), which puts each key's commands together in
// arrival order: the predecessor of a command is its left neighbour, or, for
// the first one of a key, latest[key] (sequential.rs:83-87); the key's last
// command then becomes latest[key] (:88-95).  A bucket that fits one chunk
// writes its sorted chunk as is (the output is contiguous); larger buckets
// first count every slot, then place each chunk's runs behind the earlier
// chunks' runs of the same slot.
template <int HB>
__global__ void __launch_bounds__(kThreads)
    k_kb_order(uint32_t tiles, int bb, int hb, int vb, uint32_t kinv, uint32_t kmask,
               const uint32_t *__restrict__ part, const uint16_t *__restrict__ toff,
               const uint64_t *__restrict__ dot, uint64_t *__restrict__ latest,
               uint32_t *__restrict__ sk, uint32_t *__restrict__ sv,
               uint64_t *__restrict__ dep_sorted) {
  constexpr int HMAX = 1 << HB;
  constexpr int RS = (HMAX + kThreads - 1) / kThreads;  // slots per thread in scans
  constexpr int G = kChunk / kThreads;                  // elements per thread per chunk
  constexpr int DB = 5;                                 // LDS sort digit bits
  constexpr int ND = 1 << DB;
  constexpr int PC = 16;                                // elements per thread, slot count
  __shared__ uint32_t s_a[kChunk], s_b[kChunk];
  __shared__ uint32_t s_h[kWaves][ND];
  __shared__ uint32_t s_db[ND];
  __shared__ uint32_t s_rs[kMaxTiles + 1];  // run start (bucket order) per tile
  __shared__ uint32_t s_src[kMaxTiles];     // run start in part[] per tile
  // buckets larger than one chunk only
  __shared__ uint32_t s_kbase[HMAX], s_ccnt[HMAX], s_clast[HMAX], s_hpos[HMAX];
  __shared__ uint32_t s_tmp[kWaves];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t b = blockIdx.x, B = 1u << bb, H = 1u << hb;
  const uint32_t vmask = (1u << vb) - 1;
  const uint64_t lt = (uint64_t(1) << lane) - 1;

  // this bucket's run in every tile
  const uint32_t RT = (tiles + kThreads - 1) / kThreads;  // <= 2
  uint32_t lo[2], cn[2], csum = 0, lsum = 0;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const uint32_t t = uint32_t(tid) * RT + r;
    lo[r] = 0;
    cn[r] = 0;
    if (uint32_t(r) < RT && t < tiles) {
      const uint16_t *row = toff + size_t(t) * (B + 1);
      lo[r] = row[b];
      cn[r] = uint32_t(row[b + 1]) - lo[r];
    }
    csum += cn[r];
    lsum += lo[r];
  }
  uint32_t Nb, gbase;
  uint32_t pre = block_scan(csum, s_tmp, &Nb);
  (void)block_scan(lsum, s_tmp, &gbase);  // commands of all lower buckets
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const uint32_t t = uint32_t(tid) * RT + r;
    if (uint32_t(r) < RT && t < tiles) {
      s_rs[t] = pre;
      s_src[t] = t * uint32_t(kTile) + lo[r];
    }
    pre += cn[r];
  }
  if (tid == 0) s_rs[tiles] = Nb;
  if (Nb == 0) return;  // uniform
  __syncthreads();

  // sorts s_a[0, c) by slot; returns the buffer holding the result
#define FH_GATHER(c0, c1) gather_runs<G>(part, s_rs, s_src, tiles, (c0), (c1), s_a)
#define FH_SORT_CHUNK(c)                                                       \
  (hb == 0 ? (const uint32_t *)s_a                                             \
   : hb <= DB ? (slot_sort_pass<G, ND>(s_a, s_b, (c), vb, 0, hb, s_h, s_db),   \
                (const uint32_t *)s_b)                                         \
              : (slot_sort_pass<G, ND>(s_a, s_b, (c), vb, 0, DB, s_h, s_db),   \
                 slot_sort_pass<G, ND>(s_b, s_a, (c), vb, DB, hb - DB, s_h, s_db), \
                 (const uint32_t *)s_a))

  if (Nb <= uint32_t(kChunk)) {
    // the whole bucket in one chunk: the sorted chunk is the output
    FH_GATHER(0, Nb);
    __syncthreads();
    const uint32_t *S = FH_SORT_CHUNK(Nb);
    for (uint32_t j = tid; j < Nb; j += kThreads) {
      const uint32_t e = S[j], slot = e >> vb, vid = e & vmask;
      const uint32_t mk = (b << hb) | slot;  // mapped key
      const bool head = j == 0 || (S[j - 1] >> vb) != slot;
      const uint32_t pos = gbase + j;
      sk[pos] = (mk * kinv) & kmask;
      sv[pos] = vid;
      dep_sorted[pos] = head ? latest[mk] : uint64_t(S[j - 1] & vmask) + 1;
    }
    __syncthreads();  // every head has read latest
    for (uint32_t j = tid; j < Nb; j += kThreads) {
      const uint32_t e = S[j], slot = e >> vb;
      if (j + 1 == Nb || (S[j + 1] >> vb) != slot) latest[(b << hb) | slot] = dot[e & vmask];
    }
    return;
  }

  // ---- larger buckets: slot totals first (one pass over the bucket)
  for (uint32_t k = tid; k < H; k += kThreads) {
    s_kbase[k] = 0;
    s_ccnt[k] = 0;
  }
  __syncthreads();
  for (uint32_t r0 = 0; r0 < Nb; r0 += uint32_t(kThreads) * PC) {
    const uint32_t q0 = r0 + uint32_t(tid) * PC;
    uint32_t v[PC];
    uint32_t t = q0 < Nb ? run_of(s_rs, tiles, q0) : 0u;
#pragma unroll
    for (int g = 0; g < PC; g++) {
      const uint32_t q = q0 + g;
      v[g] = 0;
      if (q < Nb) {
        while (s_rs[t + 1] <= q) t++;
        v[g] = part[s_src[t] + (q - s_rs[t])];
      }
    }
#pragma unroll
    for (int g = 0; g < PC; g++) {
      const bool valid = q0 + g < Nb;
      const uint32_t slot = valid ? (v[g] >> vb) : 0u;
      const uint64_t peers = match_bits(slot, valid, hb);
      if (valid && (peers & lt) == 0) atomicAdd(&s_kbase[slot], uint32_t(__popcll(peers)));
    }
  }
  __syncthreads();
  {
    uint32_t tl[RS], sum = 0;
#pragma unroll
    for (int r = 0; r < RS; r++) {
      const uint32_t k = uint32_t(tid) * RS + r;
      tl[r] = k < H ? s_kbase[k] : 0u;
      sum += tl[r];
    }
    uint32_t tot;
    uint32_t p2 = block_scan(sum, s_tmp, &tot);
#pragma unroll
    for (int r = 0; r < RS; r++) {
      const uint32_t k = uint32_t(tid) * RS + r;
      if (k < H) s_kbase[k] = p2;
      p2 += tl[r];
    }
  }
  __syncthreads();
  for (uint32_t c0 = 0; c0 < Nb; c0 += kChunk) {
    const uint32_t c = min(Nb - c0, uint32_t(kChunk));
    FH_GATHER(c0, c0 + c);
    __syncthreads();
    const uint32_t *S = FH_SORT_CHUNK(c);
    for (uint32_t j = tid; j < c; j += kThreads) {
      const uint32_t slot = S[j] >> vb;
      if (j == 0 || (S[j - 1] >> vb) != slot) s_hpos[slot] = j;
    }
    __syncthreads();
    for (uint32_t j = tid; j < c; j += kThreads) {
      const uint32_t e = S[j], slot = e >> vb, vid = e & vmask;
      const uint32_t mk = (b << hb) | slot;
      const uint32_t hp = s_hpos[slot], cc = s_ccnt[slot];
      const uint32_t pos = gbase + s_kbase[slot] + cc + (j - hp);
      uint64_t dep;
      if (j != hp) dep = uint64_t(S[j - 1] & vmask) + 1;
      else dep = cc ? uint64_t(s_clast[slot]) + 1 : latest[mk];
      sk[pos] = (mk * kinv) & kmask;
      sv[pos] = vid;
      dep_sorted[pos] = dep;
    }
    __syncthreads();
    for (uint32_t j = tid; j < c; j += kThreads) {
      const uint32_t e = S[j], slot = e >> vb;
      if (j + 1 == c || (S[j + 1] >> vb) != slot) {
        s_ccnt[slot] += j - s_hpos[slot] + 1;
        s_clast[slot] = e & vmask;
      }
    }
    __syncthreads();
  }
  // the key's last command becomes latest (after every head read above)
#pragma unroll
  for (int r = 0; r < RS; r++) {
    const uint32_t k = uint32_t(tid) * RS + r;
    if (k < H && s_ccnt[k]) latest[(b << hb) | k] = dot[s_clast[k]];
  }
#undef FH_GATHER
#undef FH_SORT_CHUNK
}

}  // namespace

void keybucket_map(int kb, uint32_t *kmul, uint32_t *kinv, uint32_t *kmask) {
  const uint32_t mask = kb >= 32 ? 0xFFFFFFFFu : ((1u << kb) - 1u);
  // Fibonacci hashing on the kb-bit space: odd multiplier ~ 0.618 * 2^kb
  uint32_t a = (uint32_t(std::ldexp(0.6180339887498949, kb)) | 1u) & mask;
  a |= 1u;
  uint32_t x = a;  // inverse mod 2^32 by Newton's iteration
  for (int i = 0; i < 5; i++) x *= 2u - a * x;
  *kmul = a;
  *kinv = x & mask;
  *kmask = mask;
}

KeyBucketPlan keybucket_plan(size_t n, int kb) {
  KeyBucketPlan p;
  p.kb = kb;
  p.bb = std::min(kb, 10);
  p.hb = kb - p.bb;
  if (p.hb > kSlotBits) {
    p.hb = kSlotBits;
    p.bb = kb - kSlotBits;
  }
  p.vb = bits_for(n ? n : 1);
  p.tiles = uint32_t((n + kTile - 1) / kTile);
  keybucket_map(kb, &p.kmul, &p.kinv, &p.kmask);
  p.ok = n >= 1 && n < (size_t(1) << 30) && kb >= 1 && kb <= 22 && p.bb <= 12 &&
         p.hb + p.vb <= 32 && p.tiles <= uint32_t(kMaxTiles);
  return p;
}

void keybucket_run(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32, const uint64_t *dot,
                   uint64_t *latest, unsigned long long *frontier, unsigned long long *excount,
                   KeyBucketWorkspace &ws, uint32_t *sk, uint32_t *sv, uint64_t *dep_sorted,
                   hipStream_t s) {
  FH_CHECK(p.ok, FH_EINVARIANT, "keybucket_run: batch does not fit the bucket plan");
  if (n == 0) return;
  const uint32_t B = 1u << p.bb;
  uint32_t *part = ws.part.ensure(size_t(n) + 1);
  uint16_t *toff = ws.toff.ensure(size_t(p.tiles) * (B + 1) + 1);
  auto k1 = p.bb <= 10 ? k_kb_partition<10> : k_kb_partition<12>;
  // read key (4) + dot (8), write the packed element (4)
  probed_launch("kb_partition", double(n) * 16.0, k1, dim3(p.tiles), dim3(kThreads), s, n, p.bb,
                p.hb, p.vb, p.kmul, p.kmask, key32, dot, part, toff, frontier, excount);
  // read the packed element (4), write key + command index + dependency (16)
  probed_launch("kb_order", double(n) * 20.0, k_kb_order<kSlotBits>, dim3(B), dim3(kThreads), s,
                p.tiles, p.bb, p.hb, p.vb, p.kinv, p.kmask, (const uint32_t *)part,
                (const uint16_t *)toff, dot, latest, sk, sv, dep_sorted);
}

}  // namespace fh
