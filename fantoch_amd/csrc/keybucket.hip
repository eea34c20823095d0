// keybucket.hip -- the two-launch single-view KeyDeps path (see keybucket.h).
//
// Why two launches and no global radix passes: a 1M-command batch is latency
// bound on a 256-CU part, so the path is cut at the one exchange it needs
// (commands of one key meet in one workgroup).  k_kb_partition streams the
// batch once and leaves every 2048-command tile partitioned by bucket in
// place (coalesced writes); k_kb_order gathers a bucket's runs from all tiles
// (tile order = arrival order, so no global stable sort is needed), sorts
// them by slot in LDS and writes the per-key sequence and the dependencies.
// 256 buckets keep the runs 8 commands long on average, so the gather reads
// whole sectors rather than one line per command (the first 1024-bucket
// design was bound by MALL line fetches: 1M requests for 4 MB of data).
#include <algorithm>
#include <cmath>

#include "keybucket.h"


namespace fh {
namespace {

// partition (same 1024-thread workgroups as the order role, so both roles
// can share one launch)
constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kItems = 4;
constexpr int kTile = kThreads * kItems;  // 4096 commands per partition tile
constexpr int kMaxTiles = 1024;           // batches up to 4M commands
// order
constexpr int kOThreads = 1024;
constexpr int kOWaves = kOThreads / 64;
constexpr int kChunk = kOThreads * 8;     // bucket commands staged in LDS at once
                                          // (2 order workgroups fit one CU)
constexpr int kSlotBits = 12;             // at most 4096 keys per bucket
constexpr int kDigit = 6;                 // LDS sort digit bits
constexpr int kHot = 16;                  // hot-key buckets (after the B regular ones)
constexpr int kCand = 64;                 // hot-key candidates per schedule refresh
// hot table words: [kHot] mapped keys, [1] candidate count, [kCand][2] (count, key)
constexpr int kHotWords = kHot + 1 + 2 * kCand;
constexpr int kMatchBlock = 4;           // items whose ballot matches are interleaved

// Peer masks of N independent items at once: peers[i] = lanes whose BITS-bit
// value d[i] equals this lane's (valid lanes only).  The bits loop is
// unrolled and the items interleaved, so the N ballot chains overlap; the
// select `bit ? m : ~m` is m ^ (bit - 1) on both halves (VALU only).
template <int BITS, int N>
__device__ __forceinline__ void match_many(const uint32_t (&d)[N], const bool (&valid)[N],
                                           uint64_t (&peers)[N]) {
#pragma unroll
  for (int i = 0; i < N; i++) peers[i] = __ballot(valid[i]);
#pragma unroll
  for (int b = 0; b < BITS; b++) {
#pragma unroll
    for (int i = 0; i < N; i++) {
      // m = lanes with bit b set; mk = all ones where this lane's bit is set;
      // keep the lanes whose bit equals ours: ~(m ^ mk) on both halves
      const uint64_t m = __builtin_amdgcn_ballot_w64(__builtin_amdgcn_ubfe(d[i], b, 1) != 0u);
      const uint32_t mk = uint32_t(__builtin_amdgcn_sbfe(int(d[i]), b, 1));
      const uint32_t lo = ~(uint32_t(m) ^ mk), hi = ~(uint32_t(m >> 32) ^ mk);
      peers[i] &= (uint64_t(hi) << 32) | lo;
    }
  }
}

// match_many with a runtime width (0..12)
template <int N>
__device__ __forceinline__ void match_n(int bits, const uint32_t (&d)[N], const bool (&valid)[N],
                                        uint64_t (&peers)[N]) {
  switch (bits) {
#define FH_MATCH_CASE(K)               \
  case K:                              \
    match_many<K, N>(d, valid, peers); \
    break;
    FH_MATCH_CASE(1) FH_MATCH_CASE(2) FH_MATCH_CASE(3) FH_MATCH_CASE(4) FH_MATCH_CASE(5)
    FH_MATCH_CASE(6) FH_MATCH_CASE(7) FH_MATCH_CASE(8) FH_MATCH_CASE(9) FH_MATCH_CASE(10)
    FH_MATCH_CASE(11) FH_MATCH_CASE(12)
#undef FH_MATCH_CASE
    default:
#pragma unroll
      for (int i = 0; i < N; i++) peers[i] = __ballot(valid[i]);
  }
}

// Exclusive scan of two values per thread over a block of NW waves (one set
// of barriers); t0 / t1 = block sums.  s_tmp holds 2 NW words.
template <int NW>
__device__ __forceinline__ void block_scan2(uint32_t v0, uint32_t v1, uint32_t *s_tmp,
                                            uint32_t *p0, uint32_t *p1, uint32_t *t0,
                                            uint32_t *t1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x0 = v0, x1 = v1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a0 = __shfl_up(x0, o, 64), a1 = __shfl_up(x1, o, 64);
    if (lane >= o) {
      x0 += a0;
      x1 += a1;
    }
  }
  if (lane == 63) {
    s_tmp[w] = x0;
    s_tmp[NW + w] = x1;
  }
  __syncthreads();
  uint32_t q0 = 0, q1 = 0, s0 = 0, s1 = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    const uint32_t a0 = s_tmp[i], a1 = s_tmp[NW + i];
    q0 += i < w ? a0 : 0u;
    q1 += i < w ? a1 : 0u;
    s0 += a0;
    s1 += a1;
  }
  __syncthreads();
  *p0 = q0 + x0 - v0;
  *p1 = q1 + x1 - v1;
  *t0 = s0;
  *t1 = s1;
}

template <int NW>
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t *s_tmp, uint32_t *total) {
  uint32_t p, q, t;
  block_scan2<NW>(v, 0u, s_tmp, &p, &q, total, &t);
  return p;
}

// ---------------------------------------------------------------- partition
// One 4096-command tile per workgroup.  Item i of lane l in wave w is command
// base + w*512 + i*64 + l, so (w, i, l) order is arrival order and the
// ballot-matched ranks give a stable partition.  The executed clock
// (AEClock::add for every executed dot, tarjan.rs:296) is reduced in LDS and
// added to one of 8 shards (one per XCD under round-robin placement) so the
// workgroups do not serialise on one address.
template <int BB>
struct PartSmem {
  static constexpr int BMAX = 1 << BB;
  static constexpr size_t wh = 0;                                   // u32 [kWaves][BMAX]
  static constexpr size_t dex = wh + size_t(kWaves) * BMAX * 4;     // u32 [BMAX]
  static constexpr size_t out = dex + size_t(BMAX) * 4;             // u32 [kTile]
  static constexpr size_t mx = out + size_t(kTile) * 4;             // u64 [256]
  static constexpr size_t nc = mx + 256 * 8;                        // u32 [256]
  static constexpr size_t tmp = nc + 256 * 4;                       // u32 [2 kWaves]
  static constexpr size_t bytes = tmp + 2 * kWaves * 4;
};

// A tile's inputs, loaded into registers (item i of lane l in wave w is
// command base + w 64 kItems + i 64 + l).  The fused step issues these loads
// before ordering a bucket, so they land while the bucket is sorted.
struct TileLoad {
  uint32_t key[kItems];
  uint64_t dot[kItems];
};

__device__ __forceinline__ void tile_load(uint32_t bid, uint32_t n,
                                          const uint32_t *__restrict__ key32,
                                          const uint64_t *__restrict__ dot, TileLoad &tl) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t base = bid * kTile;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + lane;
    tl.key[i] = idx < n ? key32[idx] : 0u;
    tl.dot[i] = idx < n ? dot[idx] : 0ull;
  }
}

// Bucket ids: 0..B-1 by the high bits of the mapped key, B + h for hot key
// h of the hot table (its commands need no sort: one key).
template <int BB>
__device__ __forceinline__ void partition_tile(uint32_t bid, uint32_t n, int bb, int hb, int vb,
                                               uint32_t kmul, uint32_t kmask,
                                               const TileLoad &tl,
                                               uint32_t *__restrict__ part,
                                               uint32_t *__restrict__ toff,
                                               unsigned long long *__restrict__ clk,
                                               const uint32_t *__restrict__ hot,
                                               uint32_t *__restrict__ hot_snap,
                                               unsigned char *smem) {
  using L = PartSmem<BB>;
  constexpr int BMAX = L::BMAX;
  constexpr int RB = (BMAX + kThreads - 1) / kThreads;  // buckets per thread in the scan
  uint32_t(*s_wh)[BMAX] = reinterpret_cast<uint32_t(*)[BMAX]>(smem + L::wh);
  uint32_t *s_dex = reinterpret_cast<uint32_t *>(smem + L::dex);
  uint32_t *s_out = reinterpret_cast<uint32_t *>(smem + L::out);
  unsigned long long *s_mx = reinterpret_cast<unsigned long long *>(smem + L::mx);
  uint32_t *s_nc = reinterpret_cast<uint32_t *>(smem + L::nc);
  uint32_t *s_tmp = reinterpret_cast<uint32_t *>(smem + L::tmp);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t B = 1u << bb, BT = B + kHot;
  const int mb = 32 - __builtin_clz(BT - 1);  // bucket-id bits
  for (int i = tid; i < kWaves * BMAX; i += kThreads) (&s_wh[0][0])[i] = 0;
  uint32_t hv[kHot];  // hot mapped keys (~0: empty), wave-uniform
#pragma unroll
  for (int j = 0; j < kHot; j++) hv[j] = hot ? hot[j] : ~0u;
  if (bid == 0 && tid < kHot) hot_snap[tid] = hot ? hot[tid] : ~0u;
  if (tid < 256) {
    s_mx[tid] = 0;
    s_nc[tid] = 0;
  }
  const uint32_t base = bid * kTile;
  const uint32_t tile_n = min(uint32_t(kTile), n - base);
  uint32_t pk[kItems], bkt[kItems], rank[kItems];
  uint64_t peers[kItems];
  uint64_t d[kItems];
  bool vld[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + lane;
    vld[i] = idx < n;
    pk[i] = tl.key[i];
    d[i] = tl.dot[i];
  }
  __syncthreads();
  const uint64_t lt = (uint64_t(1) << lane) - 1;
  const uint32_t smask = (1u << hb) - 1;
  // matches first (independent across items), then the ordered LDS counts
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + lane;
    const uint32_t p = (pk[i] * kmul) & kmask;
    uint32_t h = ~0u;
#pragma unroll
    for (int j = 0; j < kHot; j++) h = hv[j] == p ? uint32_t(j) : h;
    bkt[i] = h == ~0u ? p >> hb : B + h;
    pk[i] = (h == ~0u ? (p & smask) << vb : 0u) | idx;
  }
  match_n<kItems>(mb, bkt, vld, peers);
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    if (vld[i]) {
      atomicMax(&s_mx[d[i] >> 56], (unsigned long long)(d[i] & 0x00FFFFFFFFFFFFFFull));
      atomicAdd(&s_nc[d[i] >> 56], 1u);
    }
    const uint32_t b0 = vld[i] ? s_wh[w][bkt[i]] : 0u;
    if (vld[i] && (peers[i] & lt) == 0) s_wh[w][bkt[i]] = b0 + uint32_t(__popcll(peers[i]));
    rank[i] = b0 + uint32_t(__popcll(peers[i] & lt));
  }
  __syncthreads();
  // per-bucket tile counts -> per-wave exclusive offsets and bucket starts
  uint32_t loc[RB];
  uint32_t sum = 0;
#pragma unroll
  for (int r = 0; r < RB; r++) {
    const uint32_t bk = uint32_t(tid) * RB + r;
    uint32_t c = 0;
    if (bk < BT) {
      uint32_t cw[kWaves];
#pragma unroll
      for (int ww = 0; ww < kWaves; ww++) cw[ww] = s_wh[ww][bk];
#pragma unroll
      for (int ww = 0; ww < kWaves; ww++) {
        s_wh[ww][bk] = c;
        c += cw[ww];
      }
    }
    loc[r] = c;
    sum += c;
  }
  uint32_t tot;
  uint32_t pre = block_scan<kWaves>(sum, s_tmp, &tot);
  // bucket-major: the order role reads its bucket's row of all tiles at once
  const uint32_t tiles = (n + kTile - 1) / kTile;
#pragma unroll
  for (int r = 0; r < RB; r++) {
    const uint32_t bk = uint32_t(tid) * RB + r;
    if (bk < BT) {
      s_dex[bk] = pre;
      toff[size_t(bk) * tiles + bid] = pre | (loc[r] << 16);
    }
    pre += loc[r];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kItems; i++)
    if (vld[i]) s_out[s_dex[bkt[i]] + s_wh[w][bkt[i]] + rank[i]] = pk[i];
  __syncthreads();
  if (tile_n == uint32_t(kTile)) {
    uint4 *dst = reinterpret_cast<uint4 *>(part + base);
    const uint4 *src = reinterpret_cast<const uint4 *>(s_out);
#pragma unroll
    for (int j = tid; j < kTile / 4; j += kThreads) dst[j] = src[j];
  } else {
    for (uint32_t j = tid; j < tile_n; j += kThreads) part[base + j] = s_out[j];
  }
  if (tid < 256 && s_nc[tid]) {
    unsigned long long *shard = clk + size_t(blockIdx.x & 7) * 512;  // XCD of this launch
    atomicMax(&shard[tid], s_mx[tid]);
    atomicAdd(&shard[256 + tid], (unsigned long long)s_nc[tid]);
  }
}

// ---------------------------------------------------------------- order
// Helpers of k_kb_order (all inlined; LDS arrays passed explicitly).

// tile run holding bucket element q: the last t < tiles with s_rs[t] <= q
// (fixed-step search, so several searches interleave)
__device__ __forceinline__ uint32_t run_of(const uint32_t *s_rs, uint32_t tiles, uint32_t q) {
  uint32_t t = 0;
#pragma unroll
  for (uint32_t st = kMaxTiles / 2; st >= 1; st >>= 1) {
    const uint32_t v = s_rs[min(t + st, tiles)];
    t = (t + st < tiles && v <= q) ? t + st : t;
  }
  return t;
}

// Bucket elements [c0, c0 + c) into registers: element c0 + q with
// q = w 64 IT + i 64 + lane is item i of this thread (the layout of the sort
// passes).  The IT run searches interleave and every load is in flight at once.
template <int IT>
__device__ __forceinline__ void gather_items(const uint32_t *__restrict__ part,
                                             const uint32_t *s_rs, const uint32_t *s_src,
                                             uint32_t tiles, uint32_t c0, uint32_t c,
                                             uint32_t (&xe)[IT]) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t g[IT], t[IT];
#pragma unroll
  for (int i = 0; i < IT; i++) {
    g[i] = c0 + min(w * 64 * IT + uint32_t(i) * 64 + lane, c - 1);
    t[i] = 0;
  }
  // branch-free steps: every search reads its probe (clamped to the
  // s_rs[tiles] sentinel) so the IT reads of a step issue back to back
#pragma unroll
  for (uint32_t st = kMaxTiles / 2; st >= 1; st >>= 1) {
    uint32_t v[IT];
#pragma unroll
    for (int i = 0; i < IT; i++) v[i] = s_rs[min(t[i] + st, tiles)];
#pragma unroll
    for (int i = 0; i < IT; i++) t[i] = (t[i] + st < tiles && v[i] <= g[i]) ? t[i] + st : t[i];
  }
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const uint32_t q = w * 64 * IT + uint32_t(i) * 64 + lane;
    xe[i] = q < c ? part[s_src[t[i]] + (g[i] - s_rs[t[i]])] : 0u;
  }
}

// Ranks of items [H0, H0 + HALF) of a sort pass (then the next block of
// items): ballot matches for the block, then the ordered per-wave counts.
template <int IT, int HALF, int H0, int NBITS>
__device__ __forceinline__ void rank_items(const uint32_t (&xe)[IT], uint32_t c, int vb, int shift,
                                           uint32_t (*s_h)[1 << kDigit], uint32_t (&rk)[IT]) {
  constexpr int nbits = NBITS;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (uint64_t(1) << lane) - 1;
  const uint32_t dm = (1u << nbits) - 1;
  uint32_t dg[HALF];
  uint64_t peers[HALF];
  bool vld[HALF];
#pragma unroll
  for (int i = 0; i < HALF; i++) {
    const uint32_t q = uint32_t(w) * 64 * IT + uint32_t(H0 + i) * 64 + lane;
    vld[i] = q < c;
    dg[i] = vld[i] ? ((xe[H0 + i] >> vb) >> shift) & dm : 0u;
  }
  match_many<NBITS, HALF>(dg, vld, peers);
#pragma unroll
  for (int i = 0; i < HALF; i++) {
    const uint32_t b0 = vld[i] ? s_h[w][dg[i]] : 0u;
    if (vld[i] && (peers[i] & lt) == 0) s_h[w][dg[i]] = b0 + uint32_t(__popcll(peers[i]));
    rk[H0 + i] = b0 + uint32_t(__popcll(peers[i] & lt));
  }
  if constexpr (H0 + HALF < IT)
    rank_items<IT, HALF, H0 + HALF, NBITS>(xe, c, vb, shift, s_h, rk);
}

// One stable pass over the elements [0, c) held in registers (xe, layout of
// gather_items) by slot bits [shift, shift + nbits), scattered into dst.
// Element q is item (q / 64) % IT of lane q % 64 in wave q / (64 IT), so
// (wave, item, lane) order is element order and ballot ranks keep it stable.
// s_h must be zero on entry when `zeroed`.
template <int IT, int NBITS>
__device__ __forceinline__ void slot_sort_pass(const uint32_t (&xe)[IT], uint32_t *dst, uint32_t c,
                                               int vb, int shift, uint32_t (*s_h)[1 << kDigit],
                                               uint32_t *s_db, bool zeroed) {
  constexpr int nbits = NBITS;
  constexpr int ND = 1 << kDigit;
  constexpr int HALF = IT < kMatchBlock ? IT : IT % kMatchBlock == 0 ? kMatchBlock : IT % 3 == 0 ? 3 : 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (!zeroed) {
    for (int i = tid; i < kOWaves * ND; i += kOThreads) (&s_h[0][0])[i] = 0;
    __syncthreads();
  }
  uint32_t rk[IT];
  const uint32_t dm = (1u << nbits) - 1;
  rank_items<IT, HALF, 0, NBITS>(xe, c, vb, shift, s_h, rk);
  __syncthreads();
  if (w == 0) {
    // digit totals over waves (lane = digit), then the digit bases
    uint32_t cw[kOWaves];
#pragma unroll
    for (int ww = 0; ww < kOWaves; ww++) cw[ww] = s_h[ww][lane];
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < kOWaves; ww++) {
      s_h[ww][lane] = tot;
      tot += cw[ww];
    }
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < ND; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    s_db[lane] = x - tot;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const uint32_t q = uint32_t(w) * 64 * IT + uint32_t(i) * 64 + lane;
    if (q < c) {
      const uint32_t e = xe[i], d = ((e >> vb) >> shift) & dm;
      dst[s_db[d] + s_h[w][d] + rk[i]] = e;
    }
  }
  __syncthreads();
}

// one pass with the digit width chosen at run time (the passes themselves
// are compiled per width, so their inner loops have no width branches)
template <int IT>
__device__ __forceinline__ void slot_sort_pass_n(const uint32_t (&xe)[IT], uint32_t *dst,
                                                 uint32_t c, int vb, int shift, int nbits,
                                                 uint32_t (*s_h)[1 << kDigit], uint32_t *s_db,
                                                 bool zeroed) {
  switch (nbits) {
#define FH_PASS_CASE(K) \
  case K: slot_sort_pass<IT, K>(xe, dst, c, vb, shift, s_h, s_db, zeroed); break;
    FH_PASS_CASE(1) FH_PASS_CASE(2) FH_PASS_CASE(3) FH_PASS_CASE(4) FH_PASS_CASE(5)
#undef FH_PASS_CASE
    default: slot_sort_pass<IT, 6>(xe, dst, c, vb, shift, s_h, s_db, zeroed); break;
  }
}

// Sorts the c elements in xe (gather_items layout) by slot (0..2 passes)
// into a or b; returns the buffer holding the result.  The passes use the
// digit tables s_h0 / s_h1, zero on entry when `zeroed`.
template <int IT>
__device__ __forceinline__ const uint32_t *sort_chunk(const uint32_t (&xe)[IT], uint32_t *a,
                                                      uint32_t *b, uint32_t c, int vb, int hb,
                                                      uint32_t (*s_h0)[1 << kDigit],
                                                      uint32_t (*s_h1)[1 << kDigit],
                                                      uint32_t *s_db, bool zeroed) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (hb == 0) {
#pragma unroll
    for (int i = 0; i < IT; i++) {
      const uint32_t q = w * 64 * IT + uint32_t(i) * 64 + lane;
      if (q < c) a[q] = xe[i];
    }
    __syncthreads();
    return a;
  }
  if (hb <= kDigit) {
    slot_sort_pass_n<IT>(xe, b, c, vb, 0, hb, s_h0, s_db, zeroed);
    return b;
  }
  slot_sort_pass<IT, kDigit>(xe, b, c, vb, 0, s_h0, s_db, zeroed);
  uint32_t x2[IT];
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const uint32_t q = w * 64 * IT + uint32_t(i) * 64 + lane;
    x2[i] = q < c ? b[q] : 0u;
  }
  slot_sort_pass_n<IT>(x2, a, c, vb, kDigit, hb - kDigit, s_h1, s_db, zeroed);
  return a;
}

// What the order role writes for each command, in key-grouped order (the
// position of a command is its bucket's base + its rank in the sorted
// bucket): the key id (sk) and the command's dot (seq); by command index: its
// dependency as a dot (rows, ~0 for none); per key: the bounds of its run
// (runs[2 key] = first position, runs[2 key + 1] = (last + 1) | tag; keys
// the batch does not hold keep an older tag).  The run bounds feed one scan over the key space
// (ascending per-key offsets) and one scatter; no pass re-reads the keys to
// find the runs.
struct OrderOut {
  uint32_t *sk;
  uint64_t *seq;
  uint64_t *rows;
  uint32_t *runs;
  uint32_t tag;          // this batch's run tag (KeyBucketOut)
  const uint64_t *bdot;  // the batch's dots (command index -> dot)
  const uint64_t *dlog;  // the dot log (latest entries of earlier batches)
  // a dependency code (0 none, in-batch index + 1, a log reference, or a
  // dot) as the dot it names
  __device__ __forceinline__ uint64_t dep_dot(uint64_t x) const {
    return x == 0 ? ~0ull
           : is_log_ref(x) ? dlog[x - kLogFlag]
           : (x >> 56) == 0 ? bdot[x - 1]
                            : x;
  }
  __device__ __forceinline__ void put(uint32_t pos, uint32_t key, uint32_t vid,
                                      uint64_t dep) const {
    sk[pos] = key;
    seq[pos] = bdot[vid];
    rows[vid] = dep_dot(dep);
  }
};
// The order sweeps go over a thread's items in groups of kPutGroup: every
// gather of a group (the command's dot, its dependency's dot) is issued
// before the group's stores, so a group costs one gather latency rather than
// one per item, and the second half recomputes its indices from LDS instead
// of holding them.  Element j - 1 of a sweep is lane - 1's item, so a
// non-head's dependency dot (its left neighbour's dot) comes from a lane
// shuffle; heads (latest of an earlier batch) and lane 0 gather it.
constexpr int kPutGroup = 4;
__device__ __forceinline__ uint64_t left_lane(uint64_t x) {
  const uint32_t lo = __shfl_up(uint32_t(x), 1, 64), hi = __shfl_up(uint32_t(x >> 32), 1, 64);
  return (uint64_t(hi) << 32) | lo;
}

// A bucket that fits one chunk: gather into registers, sort, write the
// sorted chunk as is (contiguous output).  With the bucket's latest slice
// staged in LDS (s_lat, `staged`) heads read it there and tails write latest
// in the same sweep; otherwise heads read latest and tails write it after a
// barrier.
// A key run of at least `hot_min` commands ending at sorted position j
// (its tail) is offered as a hot-key candidate (count, mapped key).
__device__ __forceinline__ void note_hot(const uint32_t *S, uint32_t j, uint32_t slot, int vb,
                                         uint32_t mk, uint32_t hot_min, uint32_t *cand) {
  if (!cand || hot_min == 0 || j + 1 < hot_min || (S[j + 1 - hot_min] >> vb) != slot) return;
  uint32_t lo = 0, hi = j + 1 - hot_min;  // first position of the run
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((S[mid] >> vb) < slot) lo = mid + 1;
    else hi = mid;
  }
  const uint32_t i = atomicAdd(&cand[kHot], 1u);
  if (i < uint32_t(kCand)) {
    cand[kHot + 1 + 2 * i] = j - lo + 1;
    cand[kHot + 2 + 2 * i] = mk;
  }
}

template <int IT>
__device__ __forceinline__ void order_single(uint32_t Nb, uint32_t gbase, uint32_t b, int hb,
                                             int vb, uint32_t kinv, uint32_t kmask,
                                             uint32_t tiles, const uint32_t *__restrict__ part,
                                             uint64_t log_base, uint64_t *__restrict__ latest,
                                             const OrderOut &out, uint32_t *s_a,
                                             uint32_t *s_b, uint32_t (*s_h0)[1 << kDigit],
                                             uint32_t (*s_h1)[1 << kDigit], uint32_t *s_db,
                                             const uint32_t *s_rs, const uint32_t *s_src,
                                             const uint64_t *s_lat, bool staged,
                                             uint32_t hot_min, uint32_t *cand) {
  const uint32_t tid = threadIdx.x;
  const uint32_t vmask = (1u << vb) - 1;
  uint32_t xe[IT];
  gather_items<IT>(part, s_rs, s_src, tiles, 0, Nb, xe);
  const uint32_t *S = sort_chunk<IT>(xe, s_a, s_b, Nb, vb, hb, s_h0, s_h1, s_db, true);
#pragma unroll
  for (int r0 = 0; r0 < IT; r0 += kPutGroup) {
    uint64_t d[kPutGroup], w[kPutGroup];
    bool nb[kPutGroup];  // the dependency is the left lane's dot
#pragma unroll
    for (int g = 0; g < kPutGroup; g++) {
      const uint32_t j = uint32_t(r0 + g) * kOThreads + tid;
      d[g] = 0;
      nb[g] = false;
      if (r0 + g >= IT || j >= Nb) continue;
      const uint32_t e = S[j], slot = e >> vb;
      const bool head = j == 0 || (S[j - 1] >> vb) != slot;
      d[g] = out.bdot[e & vmask];
      nb[g] = !head && (tid & 63) != 0;
      if (!nb[g])
        w[g] = out.dep_dot(!head   ? uint64_t(S[j - 1] & vmask) + 1
                           : staged ? s_lat[slot]
                                    : latest[(b << hb) | slot]);
    }
#pragma unroll
    for (int g = 0; g < kPutGroup; g++) {
      const uint64_t l = left_lane(d[g]);
      if (nb[g]) w[g] = l;
    }
#pragma unroll
    for (int g = 0; g < kPutGroup; g++) {
      const uint32_t j = uint32_t(r0 + g) * kOThreads + tid;
      if (r0 + g >= IT || j >= Nb) continue;
      const uint32_t e = S[j], slot = e >> vb, vid = e & vmask;
      const uint32_t mk = (b << hb) | slot;  // mapped key
      const uint32_t key = (mk * kinv) & kmask, pos = gbase + j;
      out.sk[pos] = key;
      out.seq[pos] = d[g];
      out.rows[vid] = w[g];
      if (j == 0 || (S[j - 1] >> vb) != slot) out.runs[2 * key] = pos;
      // staged: heads read latest from LDS, so tails write it in this sweep
      if (staged && (j + 1 == Nb || (S[j + 1] >> vb) != slot)) {
        out.runs[2 * key + 1] = (pos + 1) | out.tag;
        latest[mk] = kLogFlag | (log_base + vid);
        note_hot(S, j, slot, vb, mk, hot_min, cand);
      }
    }
  }
  if (staged) return;
  __syncthreads();  // every head has read latest
  for (uint32_t j = tid; j < Nb; j += kOThreads) {
    const uint32_t e = S[j], slot = e >> vb;
    if (j + 1 == Nb || (S[j + 1] >> vb) != slot) {
      const uint32_t mk = (b << hb) | slot;
      out.runs[2 * ((mk * kinv) & kmask) + 1] = (gbase + j + 1) | out.tag;
      latest[mk] = kLogFlag | (log_base + (e & vmask));
      note_hot(S, j, slot, vb, mk, hot_min, cand);
    }
  }
}

// A hot-key bucket: one key, so its commands in arrival order are its
// sequence; each depends on the previous one, the first on latest[mk].
__device__ __forceinline__ void order_hot(uint32_t Nb, uint32_t gbase, uint32_t mk, int vb,
                                          uint32_t kinv, uint32_t kmask, uint32_t tiles,
                                          const uint32_t *__restrict__ part, uint64_t log_base,
                                          uint64_t *__restrict__ latest, const OrderOut &out,
                                          uint32_t *s_a, const uint32_t *s_rs,
                                          const uint32_t *s_src) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t vmask = (1u << vb) - 1;
  const uint32_t key = (mk * kinv) & kmask;
  const uint64_t first = latest[mk];
  uint64_t prev = first;  // dependency of the next chunk's first command
  for (uint32_t c0 = 0; c0 < Nb; c0 += kChunk) {
    const uint32_t c = min(Nb - c0, uint32_t(kChunk));
    uint32_t xe[8];
    gather_items<8>(part, s_rs, s_src, tiles, c0, c, xe);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t q = w * 64 * 8 + uint32_t(i) * 64 + lane;
      if (q < c) s_a[q] = xe[i] & vmask;
    }
    __syncthreads();
#pragma unroll
    for (int r0 = 0; r0 < 8; r0 += kPutGroup) {
      uint64_t dd[kPutGroup], ww[kPutGroup];
#pragma unroll
      for (int g = 0; g < kPutGroup; g++) {
        const uint32_t j = uint32_t(r0 + g) * kOThreads + tid;
        dd[g] = 0;
        if (j >= c) continue;
        dd[g] = out.bdot[s_a[j]];
        if (lane == 0 || j == 0) ww[g] = out.dep_dot(j ? uint64_t(s_a[j - 1]) + 1 : prev);
      }
#pragma unroll
      for (int g = 0; g < kPutGroup; g++) {
        const uint64_t l = left_lane(dd[g]);
        const uint32_t j = uint32_t(r0 + g) * kOThreads + tid;
        if (lane != 0 && j != 0) ww[g] = l;
      }
#pragma unroll
      for (int g = 0; g < kPutGroup; g++) {
        const uint32_t j = uint32_t(r0 + g) * kOThreads + tid;
        if (j >= c) continue;
        const uint32_t pos = gbase + c0 + j, vid = s_a[j];
        out.sk[pos] = key;
        out.seq[pos] = dd[g];
        out.rows[vid] = ww[g];
      }
    }
    prev = uint64_t(s_a[c - 1]) + 1;
    __syncthreads();  // s_a is rewritten by the next chunk
  }
  if (tid == 0) {
    latest[mk] = kLogFlag | (log_base + (prev - 1));
    out.runs[2 * key] = gbase;
    out.runs[2 * key + 1] = (gbase + Nb) | out.tag;
  }
}

// One bucket per 1024-thread workgroup.  The bucket's commands are the
// concatenation of its run in every tile, in tile order: that is arrival
// order.  Up to 16K of them are staged in LDS and stably sorted by slot (key)
// with 6-bit passes (wave64 ballot ranks), which puts each key's commands
// together in arrival order: the predecessor of a command is its left
// neighbour, or, for the first one of a key, latest[key] (sequential.rs:83-87);
// the key's last command then becomes latest[key] (:88-95).  Larger buckets
// count every slot first and place each chunk's runs behind the earlier
// chunks' runs of the same slot (slot tables in the global workspace).
struct OrderSmem {
  static constexpr size_t a = 0;                                      // u32 [kChunk]
  static constexpr size_t b = a + size_t(kChunk) * 4;                 // u32 [kChunk]
  static constexpr size_t lat = b + size_t(kChunk) * 4;               // u64 [1 << kSlotBits]
  static constexpr size_t h = lat + (size_t(1) << kSlotBits) * 8;     // u32 [2][kOWaves][ND]
  static constexpr size_t db = h + 2 * size_t(kOWaves) * (1 << kDigit) * 4;  // u32 [ND]
  static constexpr size_t rs = db + (1 << kDigit) * 4;                // u32 [kMaxTiles + 1]
  static constexpr size_t src = rs + size_t(kMaxTiles + 1) * 4 + 12;  // u32 [kMaxTiles]
  static constexpr size_t tmp = src + size_t(kMaxTiles) * 4;          // u32 [2 kOWaves]
  static constexpr size_t bytes = tmp + 2 * kOWaves * 4;
};
template <int BB>
constexpr size_t step_smem_bytes() {
  return OrderSmem::bytes > PartSmem<BB>::bytes ? OrderSmem::bytes : PartSmem<BB>::bytes;
}

__device__ __forceinline__ void order_bucket(uint32_t b, uint32_t tiles, int bb, int hb, int vb,
                                             uint32_t kinv, uint32_t kmask,
                                             const uint32_t *__restrict__ part,
                                             const uint32_t *__restrict__ toff,
                                             uint64_t log_base, uint64_t *__restrict__ latest,
                                             const OrderOut &out, uint32_t *__restrict__ mc,
                                             unsigned long long *__restrict__ clk_fold,
                                             unsigned long long *__restrict__ frontier,
                                             unsigned long long *__restrict__ excount,
                                             uint32_t *__restrict__ sizes,
                                             const uint32_t *__restrict__ hot_snap,
                                             uint32_t hot_min, uint32_t *__restrict__ cand,
                                             unsigned char *smem) {
  constexpr int HMAX = 1 << kSlotBits;
  constexpr int ND = 1 << kDigit;
  uint32_t *s_a = reinterpret_cast<uint32_t *>(smem + OrderSmem::a);
  uint32_t *s_b = reinterpret_cast<uint32_t *>(smem + OrderSmem::b);
  uint32_t(*s_h)[ND] = reinterpret_cast<uint32_t(*)[ND]>(smem + OrderSmem::h);
  uint32_t(*s_h1)[ND] = s_h + kOWaves;
  uint64_t *s_lat = reinterpret_cast<uint64_t *>(smem + OrderSmem::lat);
  uint32_t *s_db = reinterpret_cast<uint32_t *>(smem + OrderSmem::db);
  uint32_t *s_rs = reinterpret_cast<uint32_t *>(smem + OrderSmem::rs);  // run start per tile
  uint32_t *s_src = reinterpret_cast<uint32_t *>(smem + OrderSmem::src);  // run start in part[]
  uint32_t *s_tmp = reinterpret_cast<uint32_t *>(smem + OrderSmem::tmp);
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t B = 1u << bb, H = 1u << hb;
  const bool hot = b >= B;  // hot-key bucket B + h
  if (clk_fold && b == 0 && tid < 256) {
    // the executed clock advances by this batch (its partition wrote the
    // shards in an earlier launch): frontier = max, excount += count
    unsigned long long mx = frontier[tid], cnt = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const unsigned long long m = clk_fold[k * 512 + tid];
      mx = m > mx ? m : mx;
      cnt += clk_fold[k * 512 + 256 + tid];
      clk_fold[k * 512 + tid] = 0;
      clk_fold[k * 512 + 256 + tid] = 0;
    }
    frontier[tid] = mx;
    excount[tid] += cnt;
  }
  const uint32_t vmask = (1u << vb) - 1;
  const uint64_t lt = (uint64_t(1) << lane) - 1;

  // this bucket's run in every tile (tiles <= threads): one row of the
  // bucket-major table, lo | count << 16
  uint32_t lo = 0, cn = 0;
  if (uint32_t(tid) < tiles) {
    const uint32_t x = toff[size_t(b) * tiles + tid];
    lo = x & 0xFFFFu;
    cn = x >> 16;
  }
  // The bucket's latest slice (H entries, contiguous under the key mapping)
  // is loaded now and staged in LDS before the sort, when it is not much
  // larger than an average bucket; the loads overlap the scan and gather.
  constexpr int LR = (1 << kSlotBits) / kOThreads;
  const bool staged = !hot && H <= 2u * ((uint32_t(tiles) * uint32_t(kTile)) >> bb);
  uint64_t lv[LR];
  if (staged) {
#pragma unroll
    for (int r = 0; r < LR; r++) {
      const uint32_t k = uint32_t(r) * kOThreads + tid;
      lv[r] = k < H ? latest[(size_t(b) << hb) + k] : 0ull;
    }
  }
  // digit tables of both sort passes start at zero
  for (int i = tid; i < 2 * kOWaves * ND; i += kOThreads) (&s_h[0][0])[i] = 0;
  uint32_t pre, lpre, Nb, gbase;
  block_scan2<kOWaves>(cn, lo, s_tmp, &pre, &lpre, &Nb, &gbase);  // gbase: lower buckets
  if (sizes && tid == 0) sizes[b] = Nb;
  if (uint32_t(tid) < tiles) {
    s_rs[tid] = pre;
    s_src[tid] = uint32_t(tid) * uint32_t(kTile) + lo;
  }
  if (tid == 0) s_rs[tiles] = Nb;
  if (Nb == 0) {  // uniform
    return;
  }
  if (staged) {
#pragma unroll
    for (int r = 0; r < LR; r++) {
      const uint32_t k = uint32_t(r) * kOThreads + tid;
      if (k < H) s_lat[k] = lv[r];
    }
  }
  __syncthreads();

  if (hot) {
    order_hot(Nb, gbase, hot_snap[b - B], vb, kinv, kmask, tiles, part, log_base, latest, out, s_a,
              s_rs, s_src);
    return;
  }
  if (Nb <= uint32_t(kChunk)) {
#define FH_ORDER_SINGLE(IT)                                                                 \
  order_single<IT>(Nb, gbase, b, hb, vb, kinv, kmask, tiles, part, log_base, latest, out, s_a, \
                   s_b, s_h, s_h1, s_db, s_rs, s_src, s_lat, staged, hot_min, cand)
    if (Nb <= 2048) FH_ORDER_SINGLE(2);
    else if (Nb <= 4096) FH_ORDER_SINGLE(4);
    else if (Nb <= 6144) FH_ORDER_SINGLE(6);
    else FH_ORDER_SINGLE(8);
#undef FH_ORDER_SINGLE
    return;
  }

  // ---- larger buckets: slot tables in the workspace (kbase, ccnt, clast,
  // hpos per slot); slot totals first, from a pass over the whole bucket
  uint32_t *g_kbase = mc + size_t(b) * 4 * HMAX, *g_ccnt = g_kbase + HMAX;
  uint32_t *g_clast = g_ccnt + HMAX, *g_hpos = g_clast + HMAX;
  for (uint32_t k = tid; k < H; k += kOThreads) s_b[k] = 0;
  __syncthreads();
  for (uint32_t r0 = 0; r0 < Nb; r0 += kOThreads) {
    const uint32_t q = r0 + tid;
    const bool valid = q < Nb;
    uint32_t slot = 0;
    if (valid) {
      const uint32_t t = run_of(s_rs, tiles, q);
      slot = part[s_src[t] + (q - s_rs[t])] >> vb;
    }
    uint32_t sl[1] = {slot};
    bool vl[1] = {valid};
    uint64_t pe[1];
    match_n<1>(hb, sl, vl, pe);
    if (valid && (pe[0] & lt) == 0) atomicAdd(&s_b[slot], uint32_t(__popcll(pe[0])));
  }
  __syncthreads();
  {
    constexpr int RS = HMAX / kOThreads;
    uint32_t tl[RS], sum = 0;
#pragma unroll
    for (int r = 0; r < RS; r++) {
      const uint32_t k = uint32_t(tid) * RS + r;
      tl[r] = k < H ? s_b[k] : 0u;
      sum += tl[r];
    }
    uint32_t tot;
    uint32_t p2 = block_scan<kOWaves>(sum, s_tmp, &tot);
#pragma unroll
    for (int r = 0; r < RS; r++) {
      const uint32_t k = uint32_t(tid) * RS + r;
      if (k < H) {
        g_kbase[k] = p2;
        g_ccnt[k] = 0;
      }
      p2 += tl[r];
    }
  }
  __syncthreads();
  for (uint32_t c0 = 0; c0 < Nb; c0 += kChunk) {
    const uint32_t c = min(Nb - c0, uint32_t(kChunk));
    uint32_t xe[8];
    gather_items<8>(part, s_rs, s_src, tiles, c0, c, xe);
    const uint32_t *S = sort_chunk<8>(xe, s_a, s_b, c, vb, hb, s_h, s_h1, s_db, false);
    for (uint32_t j = tid; j < c; j += kOThreads) {
      const uint32_t slot = S[j] >> vb;
      if (j == 0 || (S[j - 1] >> vb) != slot) g_hpos[slot] = j;
    }
    __threadfence_block();
    __syncthreads();
    for (uint32_t j = tid; j < c; j += kOThreads) {
      const uint32_t e = S[j], slot = e >> vb, vid = e & vmask;
      const uint32_t mk = (b << hb) | slot;
      const uint32_t hp = g_hpos[slot], cc = g_ccnt[slot];
      const uint32_t pos = gbase + g_kbase[slot] + cc + (j - hp);
      uint64_t dep;
      if (j != hp) dep = uint64_t(S[j - 1] & vmask) + 1;
      else dep = cc ? uint64_t(g_clast[slot]) + 1 : latest[mk];
      out.put(pos, (mk * kinv) & kmask, vid, dep);
    }
    __threadfence_block();
    __syncthreads();
    for (uint32_t j = tid; j < c; j += kOThreads) {
      const uint32_t e = S[j], slot = e >> vb;
      if (j + 1 == c || (S[j + 1] >> vb) != slot) {
        g_ccnt[slot] += j - g_hpos[slot] + 1;
        g_clast[slot] = e & vmask;
      }
    }
    __threadfence_block();
    __syncthreads();
  }
  // the key's last command becomes latest (after every head read above)
  for (uint32_t k = tid; k < H; k += kOThreads) {
    const uint32_t cnt = g_ccnt[k];
    if (cnt) {
      const uint32_t key = (((b << hb) | k) * kinv) & kmask, p0 = gbase + g_kbase[k];
      latest[(b << hb) | k] = kLogFlag | (log_base + g_clast[k]);
      out.runs[2 * key] = p0;
      out.runs[2 * key + 1] = (p0 + cnt) | out.tag;
    }
    if (cand && hot_min && cnt >= hot_min) {  // hot-key candidate (see note_hot)
      const uint32_t i = atomicAdd(&cand[kHot], 1u);
      if (i < uint32_t(kCand)) {
        cand[kHot + 1 + 2 * i] = cnt;
        cand[kHot + 2 + 2 * i] = (b << hb) | k;
      }
    }
  }
}

// Arguments of the two roles (kernel arguments by value).
struct OrderArgs {
  uint32_t tiles;
  int bb, hb, vb;
  uint32_t kinv, kmask;
  const uint32_t *part;
  const uint32_t *toff;
  uint64_t log_base;
  uint64_t *latest;
  OrderOut out;
  uint32_t *mc;
  unsigned long long *clk_fold, *frontier, *excount;
  const uint32_t *perm;      // workgroup -> bucket (null: identity)
  uint32_t *sizes;           // per-bucket sizes for the schedule (nullable)
  const uint32_t *hot_snap;  // hot keys the batch was partitioned with
  uint32_t hot_min;
  uint32_t *cand;            // hot table words (candidates), nullable
};
struct PartArgs {
  uint32_t n;
  int bb, hb, vb;
  uint32_t kmul, kmask;
  const uint32_t *key32;
  const uint64_t *dot;
  uint32_t *part, *toff;
  unsigned long long *clk;
  const uint32_t *hot;  // hot table (nullable)
  uint32_t *hot_snap;
};

template <int BB>
__device__ __forceinline__ void part_role(const PartArgs &a, uint32_t t, const TileLoad &tl,
                                          unsigned char *smem) {
  partition_tile<BB>(t, a.n, a.bb, a.hb, a.vb, a.kmul, a.kmask, tl, a.part, a.toff, a.clk, a.hot,
                     a.hot_snap, smem);
}

__device__ __forceinline__ void order_role(const OrderArgs &a, uint32_t r, unsigned char *smem) {
  order_bucket(a.perm ? a.perm[r] : r, a.tiles, a.bb, a.hb, a.vb, a.kinv, a.kmask, a.part, a.toff,
               a.log_base, a.latest, a.out, a.mc, a.clk_fold, a.frontier,
               a.excount, a.sizes, a.hot_snap, a.hot_min, a.cand, smem);
}

template <int BB>
__global__ void __launch_bounds__(kThreads) k_kb_partition(PartArgs a) {
  __shared__ __align__(16) unsigned char smem[PartSmem<BB>::bytes];
  TileLoad tl;
  tile_load(blockIdx.x, a.n, a.key32, a.dot, tl);
  part_role<BB>(a, blockIdx.x, tl, smem);
}

__global__ void __launch_bounds__(kOThreads) k_kb_order(OrderArgs a) {
  __shared__ __align__(16) unsigned char smem[OrderSmem::bytes];
  order_role(a, blockIdx.x, smem);
}

// One launch per pipelined step: the order role over batch b (its partition
// is in a's workspace) and the partition role over batch b+1; the roles
// touch disjoint memory.  Workgroups [0, BT) order the buckets by schedule
// rank (largest first), the rest partition; workgroups dispatch in index
// order, so the partition fills the CUs the short buckets release.
// (Measured alternatives, all slower on MI355X: partition first or
// interleaved; order + partition in one workgroup; two workgroups per CU.)
template <int BB>
__global__ void __launch_bounds__(kOThreads) k_kb_step(OrderArgs a, uint32_t BT, PartArgs pa) {
  __shared__ __align__(16) unsigned char smem[step_smem_bytes<BB>()];
  const uint32_t g = blockIdx.x;
  if (g < BT) {
    order_role(a, g, smem);
    return;
  }
  TileLoad tl;
  tile_load(g - BT, pa.n, pa.key32, pa.dot, tl);
  part_role<BB>(pa, g - BT, tl, smem);
}

// Schedule refresh (one workgroup), from the last order launch:
//  * hot table: the hot keys still above hot_min / 2 commands and the
//    candidates offered (runs >= hot_min), deduplicated, the kHot largest;
//  * perm: buckets by recorded size, largest first (ties by index), so the
//    longest workgroups start in the first round.
constexpr int kMaxBT = 512 + kHot;
__global__ void __launch_bounds__(1024)
    k_kb_sched(uint32_t BT, uint32_t B, uint32_t hot_min, const uint32_t *__restrict__ sizes,
               uint32_t *__restrict__ perm, uint32_t *__restrict__ hot) {
  constexpr int NE = kHot + kCand;
  __shared__ uint32_t s_sz[kMaxBT];
  __shared__ uint32_t s_cnt[NE], s_key[NE], s_new[kHot];
  const uint32_t t = threadIdx.x;
  if (t < BT) s_sz[t] = sizes[t];
  if (t < uint32_t(kHot)) s_new[t] = ~0u;
  uint32_t c = 0, k = ~0u;
  if (t < uint32_t(kHot)) {
    k = hot[t];
    c = k != ~0u ? sizes[B + t] : 0u;
    if (2 * c < hot_min) k = ~0u;
  } else if (t < uint32_t(NE)) {
    const uint32_t i = t - kHot;
    if (i < min(hot[kHot], uint32_t(kCand))) {
      c = hot[kHot + 1 + 2 * i];
      k = hot[kHot + 2 + 2 * i];
    }
  }
  if (t < uint32_t(NE)) {
    s_key[t] = k;
    s_cnt[t] = k == ~0u ? 0u : c;
  }
  __syncthreads();
  if (t < uint32_t(NE) && k != ~0u) {
    for (uint32_t j = 0; j < t; j++)
      if (s_key[j] == k) k = ~0u;  // keep the first entry of a key
  }
  __syncthreads();
  if (t < uint32_t(NE)) {
    s_key[t] = k;
    s_cnt[t] = k == ~0u ? 0u : c;
  }
  __syncthreads();
  if (t < uint32_t(NE) && k != ~0u) {
    uint32_t r = 0;
    for (uint32_t j = 0; j < uint32_t(NE); j++) {
      const uint32_t o = s_cnt[j];
      r += s_key[j] != ~0u && (o > c || (o == c && j < t));
    }
    if (r < uint32_t(kHot)) s_new[r] = k;
  }
  __syncthreads();
  if (t < uint32_t(kHot)) hot[t] = s_new[t];
  if (t == 0) hot[kHot] = 0;
  if (t < BT) {
    const uint32_t my = s_sz[t];
    uint32_t r = 0;
    for (uint32_t j = 0; j < BT; j++) {
      const uint32_t o = s_sz[j];
      r += (o > my) || (o == my && j < t);
    }
    perm[r] = t;
  }
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
  // 256 buckets when the key space allows (Zipf-hot keys go to the kHot
  // hot-key buckets, so the regular ones stay near n / 256), at most 4096
  // keys each
  p.bb = std::min(kb, 8);
  p.hb = kb - p.bb;
  if (p.hb > kSlotBits) {
    p.hb = kSlotBits;
    p.bb = kb - kSlotBits;
  }
  p.vb = bits_for(n ? n : 1);
  p.tiles = uint32_t((n + kTile - 1) / kTile);
  keybucket_map(kb, &p.kmul, &p.kinv, &p.kmask);
  p.ok = n >= 1 && n < (size_t(1) << 30) && kb >= 1 && kb <= 21 && p.bb <= 9 &&
         p.hb + p.vb <= 32 && p.tiles <= uint32_t(kMaxTiles);
  return p;
}

static uint32_t buckets_total(const KeyBucketPlan &p) { return (1u << p.bb) + kHot; }

// commands of one key in one batch that make it a hot-key candidate
static uint32_t hot_min_for(const KeyBucketPlan &p) {
  return std::max<uint32_t>(64, (p.tiles * uint32_t(kTile)) >> (p.bb + 3));
}

// the schedule's buffers for a plan of BT buckets (reset when BT changes:
// no hot keys, identity order, until the next refresh)
static void sched_prepare(KeyBucketSched *sc, const KeyBucketPlan &p, hipStream_t s) {
  if (!sc) return;
  const uint32_t BT = buckets_total(p);
  if (sc->B == BT && sc->bb == p.bb) return;
  sc->B = BT;
  sc->bb = p.bb;
  sc->hot_min = hot_min_for(p);
  FH_HIP(hipMemsetAsync(sc->sizes.ensure(BT), 0, BT * sizeof(uint32_t), s));
  sc->perm.ensure(BT);
  uint32_t *h = sc->hot.ensure(kHotWords);
  FH_HIP(hipMemsetAsync(h, 0xFF, kHot * sizeof(uint32_t), s));
  FH_HIP(hipMemsetAsync(h + kHot, 0, (kHotWords - kHot) * sizeof(uint32_t), s));
  sc->valid = false;
}

void keybucket_sched(KeyBucketSched &sc, hipStream_t s) {
  if (sc.B == 0) return;
  k_kb_sched<<<1, 1024, 0, s>>>(sc.B, sc.B - kHot, sc.hot_min, sc.sizes.get(), sc.perm.get(),
                                 sc.hot.get());
  FH_HIP(hipGetLastError());
  sc.valid = true;
}

static PartArgs part_args(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32,
                          const uint64_t *dot, unsigned long long *clk, KeyBucketWorkspace &ws,
                          KeyBucketSched *sc) {
  PartArgs a;
  a.n = n;
  a.bb = p.bb;
  a.hb = p.hb;
  a.vb = p.vb;
  a.kmul = p.kmul;
  a.kmask = p.kmask;
  a.key32 = key32;
  a.dot = dot;
  a.part = ws.part.ensure(size_t(n) + 1);
  a.toff = ws.toff.ensure(size_t(p.tiles) * buckets_total(p));
  a.clk = clk;
  a.hot = sc ? sc->hot.get() : nullptr;
  a.hot_snap = ws.hot.ensure(kHot);
  return a;
}

static OrderArgs order_args(const KeyBucketPlan &p, uint64_t log_base, uint64_t *latest,
                            KeyBucketWorkspace &ws, const KeyBucketOut &out,
                            const KeyBucketClock &clock, KeyBucketSched *sc) {
  OrderArgs a;
  a.tiles = p.tiles;
  a.bb = p.bb;
  a.hb = p.hb;
  a.vb = p.vb;
  a.kinv = p.kinv;
  a.kmask = p.kmask;
  a.part = ws.part.get();
  a.toff = ws.toff.get();
  a.log_base = log_base;
  a.latest = latest;
  a.out.sk = out.sk;
  a.out.seq = out.seq;
  a.out.rows = out.rows;
  a.out.runs = out.runs;
  a.out.tag = out.run_tag << kRunEndBits;
  a.out.bdot = out.bdot;
  a.out.dlog = out.dlog;
  // slot tables of buckets larger than one LDS chunk (rare)
  a.mc = ws.mc.ensure(size_t(1u << p.bb) * 4 * (size_t(1) << kSlotBits));
  a.clk_fold = clock.fold;
  a.frontier = clock.frontier;
  a.excount = clock.excount;
  a.perm = sc && sc->valid ? sc->perm.get() : nullptr;
  a.sizes = sc ? sc->sizes.get() : nullptr;
  a.hot_snap = ws.hot.get();
  a.hot_min = sc ? sc->hot_min : 0u;
  a.cand = sc ? sc->hot.get() : nullptr;
  return a;
}

template <typename K>
static K by_bits(int mbits, K k8, K k9, K k10) {
  return mbits <= 8 ? k8 : mbits == 9 ? k9 : k10;
}
static int id_bits(const KeyBucketPlan &p) { return 32 - __builtin_clz(buckets_total(p) - 1); }

void keybucket_partition(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32,
                         const uint64_t *dot, unsigned long long *clk, KeyBucketWorkspace &ws,
                         hipStream_t s, KeyBucketSched *sc) {
  FH_CHECK(p.ok, FH_EINVARIANT, "keybucket: batch does not fit the bucket plan");
  if (n == 0) return;
  sched_prepare(sc, p, s);
  const PartArgs a = part_args(p, n, key32, dot, clk, ws, sc);
  auto k1 = by_bits(id_bits(p), k_kb_partition<8>, k_kb_partition<9>, k_kb_partition<10>);
  // read key (4) + dot (8), write the packed element (4)
  probed_launch("kb_partition", double(n) * 16.0, k1, dim3(p.tiles), dim3(kThreads), s, a);
}

void keybucket_order(const KeyBucketPlan &p, uint32_t n, uint64_t log_base, uint64_t *latest,
                     KeyBucketWorkspace &ws, const KeyBucketOut &out, const KeyBucketClock &clock,
                     hipStream_t s, KeyBucketSched *sc) {
  FH_CHECK(p.ok, FH_EINVARIANT, "keybucket: batch does not fit the bucket plan");
  if (n == 0) return;
  sched_prepare(sc, p, s);
  const OrderArgs a = order_args(p, log_base, latest, ws, out, clock, sc);
  // read the packed element (4) and the dot (8), write key + dot + row (20)
  probed_launch("kb_order", double(n) * 32.0, k_kb_order, dim3(buckets_total(p)),
                dim3(kOThreads), s, a);
}

void keybucket_step(const KeyBucketPlan &p, uint32_t n, uint64_t log_base, uint64_t *latest,
                    KeyBucketWorkspace &ws, const KeyBucketOut &out, const KeyBucketClock &clock, const KeyBucketPlan &p2, uint32_t n2,
                    const uint32_t *key32_2, const uint64_t *dot_2, unsigned long long *clk,
                    KeyBucketWorkspace &ws2, hipStream_t s, KeyBucketSched *sc) {
  FH_CHECK(p.ok && p2.ok, FH_EINVARIANT, "keybucket: batch does not fit the bucket plan");
  FH_CHECK(p.bb == p2.bb, FH_EINVARIANT, "keybucket: step over plans of different widths");
  sched_prepare(sc, p, s);
  const OrderArgs a = order_args(p, log_base, latest, ws, out, clock, sc);
  const PartArgs pa = part_args(p2, n2, key32_2, dot_2, clk, ws2, sc);
  const uint32_t BT = buckets_total(p);
  auto k = by_bits(id_bits(p2), k_kb_step<8>, k_kb_step<9>, k_kb_step<10>);
  // order (32 B / command of batch b) + partition (16 B / command of b+1)
  probed_launch("kb_step", double(n) * 32.0 + double(n2) * 16.0, k, dim3(BT + p2.tiles),
                dim3(kOThreads), s, a, BT, pa);
}

void keybucket_run(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32, const uint64_t *dot,
                   uint64_t log_base, uint64_t *latest, const KeyBucketClock &clock,
                   KeyBucketWorkspace &ws, const KeyBucketOut &out, hipStream_t s,
                   KeyBucketSched *sc) {
  keybucket_partition(p, n, key32, dot, clock.fold, ws, s, sc);
  keybucket_order(p, n, log_base, latest, ws, out, clock, s, sc);
}

}  // namespace fh
