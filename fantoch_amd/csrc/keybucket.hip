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

#ifdef FH_KB_STAMPS
// diagnostic builds (tools/kbbench.cpp): per-workgroup {start, end, work}
// and phase ends in s_memrealtime ticks (100 MHz); never in the library
__device__ unsigned long long *g_kb_stamps[2];
__device__ unsigned long long *g_kb_phase[2];  // [wg][8]
#define FH_STAMP_BEGIN() const unsigned long long fh_t0 = __builtin_amdgcn_s_memrealtime()
#define FH_STAMP_END(k, work)                                                \
  do {                                                                       \
    if (threadIdx.x == 0 && g_kb_stamps[k]) {                                \
      g_kb_stamps[k][3 * fh_bid] = fh_t0;                                \
      g_kb_stamps[k][3 * fh_bid + 1] = __builtin_amdgcn_s_memrealtime(); \
      g_kb_stamps[k][3 * fh_bid + 2] = (work);                           \
    }                                                                        \
  } while (0)
#define FH_PHASE(k, i)                                                        \
  do {                                                                        \
    if (threadIdx.x == 0 && g_kb_phase[k])                                    \
      g_kb_phase[k][8 * blockIdx.x + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define FH_STAMP_BEGIN() (void)0
#define FH_STAMP_END(k, work) (void)0
#define FH_PHASE(k, i) (void)0
#endif

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
constexpr int kChunk = kOThreads * 16;    // bucket commands staged in LDS at once
constexpr int kSlotBits = 12;             // at most 4096 keys per bucket
constexpr int kDigit = 6;                 // LDS sort digit bits

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
      const uint32_t bit = (d[i] >> b) & 1u;
      const uint64_t m = __ballot(bit);
      const uint32_t nm = bit - 1u;  // 0 if bit, else all ones
      peers[i] &= m ^ ((uint64_t(nm) << 32) | nm);
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

template <int BB>
__device__ __forceinline__ void partition_tile(uint32_t bid, uint32_t n, int bb, int hb, int vb,
                                               uint32_t kmul, uint32_t kmask,
                                               const uint32_t *__restrict__ key32,
                                               const uint64_t *__restrict__ dot,
                                               uint32_t *__restrict__ part,
                                               uint16_t *__restrict__ toff,
                                               unsigned long long *__restrict__ clk,
                                               unsigned char *smem) {
  const uint32_t fh_bid = bid;
  (void)fh_bid;
  FH_STAMP_BEGIN();
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
  const uint32_t B = 1u << bb;
  for (int i = tid; i < kWaves * BMAX; i += kThreads) (&s_wh[0][0])[i] = 0;
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
    pk[i] = vld[i] ? key32[idx] : 0u;
    d[i] = vld[i] ? dot[idx] : 0ull;
  }
  __syncthreads();
  FH_PHASE(0, 0);
  const uint64_t lt = (uint64_t(1) << lane) - 1;
  const uint32_t smask = (1u << hb) - 1;
  // matches first (independent across items), then the ordered LDS counts
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + uint32_t(w) * 64 * kItems + uint32_t(i) * 64 + lane;
    const uint32_t p = (pk[i] * kmul) & kmask;
    bkt[i] = p >> hb;
    pk[i] = ((p & smask) << vb) | idx;
  }
  match_n<kItems>(bb, bkt, vld, peers);
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
  FH_PHASE(0, 1);
  // per-bucket tile counts -> per-wave exclusive offsets and bucket starts
  uint32_t loc[RB];
  uint32_t sum = 0;
#pragma unroll
  for (int r = 0; r < RB; r++) {
    const uint32_t bk = uint32_t(tid) * RB + r;
    uint32_t c = 0;
    if (bk < B) {
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
  uint16_t *row = toff + size_t(bid) * (B + 1);
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
  FH_PHASE(0, 2);
#pragma unroll
  for (int i = 0; i < kItems; i++)
    if (vld[i]) s_out[s_dex[bkt[i]] + s_wh[w][bkt[i]] + rank[i]] = pk[i];
  __syncthreads();
  FH_PHASE(0, 3);
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
  FH_STAMP_END(0, tile_n);
}

// ---------------------------------------------------------------- order
// Helpers of k_kb_order (all inlined; LDS arrays passed explicitly).

// tile run holding bucket element q: s_rs[t] <= q < s_rs[t + 1]
__device__ __forceinline__ uint32_t run_of(const uint32_t *s_rs, uint32_t tiles, uint32_t q) {
  uint32_t tl = 0, th = tiles;
  while (th - tl > 1) {
    const uint32_t mid = (tl + th) >> 1;
    if (s_rs[mid] <= q) tl = mid;
    else th = mid;
  }
  return tl;
}

// bucket elements [c0, c0 + c) -> dst[0, c): thread t copies the part of
// tile t's run that falls in the window (tiles <= threads)
__device__ __forceinline__ void gather_runs(const uint32_t *__restrict__ part, const uint32_t *s_rs,
                                            const uint32_t *s_src, uint32_t tiles, uint32_t c0,
                                            uint32_t c, uint32_t *dst) {
  const uint32_t t = threadIdx.x;
  if (t >= tiles) return;
  const uint32_t r0 = s_rs[t], r1 = s_rs[t + 1];
  const uint32_t a = max(r0, c0), e = min(r1, c0 + c);
  if (a >= e) return;
  const uint32_t *src = part + s_src[t] + (a - r0);
  uint32_t *out = dst + (a - c0);
  const uint32_t len = e - a;
  uint32_t j = 0;
  for (; j + 4 <= len; j += 4) {
    const uint32_t x0 = src[j], x1 = src[j + 1], x2 = src[j + 2], x3 = src[j + 3];
    out[j] = x0;
    out[j + 1] = x1;
    out[j + 2] = x2;
    out[j + 3] = x3;
  }
  for (; j < len; j++) out[j] = src[j];
}

// Ranks of items [H0, H0 + HALF) of a sort pass (then the next block of
// items): ballot matches for the block, then the ordered per-wave counts.
template <int IT, int HALF, int H0>
__device__ __forceinline__ void rank_items(const uint32_t *src, uint32_t c, int vb, int shift,
                                           int nbits, uint32_t (*s_h)[1 << kDigit],
                                           uint32_t (&rk)[IT]) {
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
    dg[i] = vld[i] ? ((src[q] >> vb) >> shift) & dm : 0u;
  }
  match_n<HALF>(nbits, dg, vld, peers);
#pragma unroll
  for (int i = 0; i < HALF; i++) {
    const uint32_t b0 = vld[i] ? s_h[w][dg[i]] : 0u;
    if (vld[i] && (peers[i] & lt) == 0) s_h[w][dg[i]] = b0 + uint32_t(__popcll(peers[i]));
    rk[H0 + i] = b0 + uint32_t(__popcll(peers[i] & lt));
  }
  if constexpr (H0 + HALF < IT) rank_items<IT, HALF, H0 + HALF>(src, c, vb, shift, nbits, s_h, rk);
}

// One stable LDS pass over src[0, c) by slot bits [shift, shift + nbits).
// Element q is item (q / 64) % IT of lane q % 64 in wave q / (64 IT), so
// (wave, item, lane) order is element order and ballot ranks keep it stable.
template <int IT>
__device__ __forceinline__ void slot_sort_pass(const uint32_t *src, uint32_t *dst, uint32_t c,
                                               int vb, int shift, int nbits,
                                               uint32_t (*s_h)[1 << kDigit], uint32_t *s_db,
                                               bool stamp) {
  constexpr int ND = 1 << kDigit;
  constexpr int HALF = IT < 4 ? IT : 4;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < kOWaves * ND; i += kOThreads) (&s_h[0][0])[i] = 0;
  __syncthreads();
  if (stamp) FH_PHASE(1, 4);
  uint32_t rk[IT];
  const uint32_t dm = (1u << nbits) - 1;
  rank_items<IT, HALF, 0>(src, c, vb, shift, nbits, s_h, rk);
  __syncthreads();
  if (stamp) FH_PHASE(1, 5);
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
  if (stamp) FH_PHASE(1, 6);
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const uint32_t q = uint32_t(w) * 64 * IT + uint32_t(i) * 64 + lane;
    if (q < c) {
      const uint32_t e = src[q], d = ((e >> vb) >> shift) & dm;
      dst[s_db[d] + s_h[w][d] + rk[i]] = e;
    }
  }
  __syncthreads();
}

// sorts a[0, c) by slot (0..2 passes); returns the buffer holding the result
template <int IT>
__device__ __forceinline__ const uint32_t *sort_chunk(uint32_t *a, uint32_t *b, uint32_t c,
                                                      int vb, int hb,
                                                      uint32_t (*s_h)[1 << kDigit],
                                                      uint32_t *s_db) {
  if (hb == 0) return a;
  if (hb <= kDigit) {
    slot_sort_pass<IT>(a, b, c, vb, 0, hb, s_h, s_db, true);
    return b;
  }
  slot_sort_pass<IT>(a, b, c, vb, 0, kDigit, s_h, s_db, true);
  slot_sort_pass<IT>(b, a, c, vb, kDigit, hb - kDigit, s_h, s_db, false);
  return a;
}

// A bucket that fits one chunk: gather, sort, write the sorted chunk as is
// (contiguous output), heads read latest; the tails' dots are loaded in the
// same sweep and written to latest after every head has read it.
template <int IT>
__device__ __forceinline__ void order_single(uint32_t Nb, uint32_t gbase, uint32_t b, int hb,
                                             int vb, uint32_t kinv, uint32_t kmask,
                                             uint32_t tiles, const uint32_t *__restrict__ part,
                                             uint64_t log_base, uint64_t *__restrict__ latest,
                                             uint32_t *__restrict__ sk, uint32_t *__restrict__ sv,
                                             uint64_t *__restrict__ dep_sorted, uint32_t *s_a,
                                             uint32_t *s_b, uint32_t (*s_h)[1 << kDigit],
                                             uint32_t *s_db, const uint32_t *s_rs,
                                             const uint32_t *s_src) {
  const uint32_t tid = threadIdx.x;
  const uint32_t vmask = (1u << vb) - 1;
  gather_runs(part, s_rs, s_src, tiles, 0, Nb, s_a);
  __syncthreads();
  FH_PHASE(1, 1);
  const uint32_t *S = sort_chunk<IT>(s_a, s_b, Nb, vb, hb, s_h, s_db);
  FH_PHASE(1, 2);
  for (uint32_t j = tid; j < Nb; j += kOThreads) {
    const uint32_t e = S[j], slot = e >> vb, vid = e & vmask;
    const uint32_t mk = (b << hb) | slot;  // mapped key
    const bool head = j == 0 || (S[j - 1] >> vb) != slot;
    const uint32_t pos = gbase + j;
    sk[pos] = (mk * kinv) & kmask;
    sv[pos] = vid;
    dep_sorted[pos] = head ? latest[mk] : uint64_t(S[j - 1] & vmask) + 1;
  }
  __syncthreads();  // every head has read latest
  FH_PHASE(1, 3);
  for (uint32_t j = tid; j < Nb; j += kOThreads) {
    const uint32_t e = S[j], slot = e >> vb;
    if (j + 1 == Nb || (S[j + 1] >> vb) != slot)
      latest[(b << hb) | slot] = kLogFlag | (log_base + (e & vmask));
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
  static constexpr size_t h = b + size_t(kChunk) * 4;                 // u32 [kOWaves][ND]
  static constexpr size_t db = h + size_t(kOWaves) * (1 << kDigit) * 4;  // u32 [ND]
  static constexpr size_t rs = db + (1 << kDigit) * 4;                // u32 [kMaxTiles + 1]
  static constexpr size_t src = rs + size_t(kMaxTiles + 1) * 4 + 12;  // u32 [kMaxTiles]
  static constexpr size_t tmp = src + size_t(kMaxTiles) * 4;          // u32 [2 kOWaves]
  static constexpr size_t bytes = tmp + 2 * kOWaves * 4;
};
constexpr size_t kSmemBytes = OrderSmem::bytes > PartSmem<10>::bytes ? OrderSmem::bytes
                                                                      : PartSmem<10>::bytes;

__device__ __forceinline__ void order_bucket(uint32_t b, uint32_t tiles, int bb, int hb, int vb,
                                             uint32_t kinv, uint32_t kmask,
                                             const uint32_t *__restrict__ part,
                                             const uint16_t *__restrict__ toff,
                                             uint64_t log_base, uint64_t *__restrict__ latest,
                                             uint32_t *__restrict__ sk, uint32_t *__restrict__ sv,
                                             uint64_t *__restrict__ dep_sorted,
                                             uint32_t *__restrict__ mc,
                                             unsigned long long *__restrict__ clk_fold,
                                             unsigned long long *__restrict__ frontier,
                                             unsigned long long *__restrict__ excount,
                                             unsigned char *smem) {
  const uint32_t fh_bid = b;
  (void)fh_bid;
  FH_STAMP_BEGIN();
  constexpr int HMAX = 1 << kSlotBits;
  constexpr int ND = 1 << kDigit;
  uint32_t *s_a = reinterpret_cast<uint32_t *>(smem + OrderSmem::a);
  uint32_t *s_b = reinterpret_cast<uint32_t *>(smem + OrderSmem::b);
  uint32_t(*s_h)[ND] = reinterpret_cast<uint32_t(*)[ND]>(smem + OrderSmem::h);
  uint32_t *s_db = reinterpret_cast<uint32_t *>(smem + OrderSmem::db);
  uint32_t *s_rs = reinterpret_cast<uint32_t *>(smem + OrderSmem::rs);  // run start per tile
  uint32_t *s_src = reinterpret_cast<uint32_t *>(smem + OrderSmem::src);  // run start in part[]
  uint32_t *s_tmp = reinterpret_cast<uint32_t *>(smem + OrderSmem::tmp);
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t B = 1u << bb, H = 1u << hb;
  if (clk_fold && b + 1 == B && tid < 256) {
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

  // this bucket's run in every tile (tiles <= threads)
  uint32_t lo = 0, cn = 0;
  if (uint32_t(tid) < tiles) {
    const uint16_t *row = toff + size_t(tid) * (B + 1);
    lo = row[b];
    cn = uint32_t(row[b + 1]) - lo;
  }
  uint32_t pre, lpre, Nb, gbase;
  block_scan2<kOWaves>(cn, lo, s_tmp, &pre, &lpre, &Nb, &gbase);  // gbase: lower buckets
  if (uint32_t(tid) < tiles) {
    s_rs[tid] = pre;
    s_src[tid] = uint32_t(tid) * uint32_t(kTile) + lo;
  }
  if (tid == 0) s_rs[tiles] = Nb;
  if (Nb == 0) {  // uniform
    FH_STAMP_END(1, 0);
    return;
  }
  __syncthreads();
  FH_PHASE(1, 0);

  if (Nb <= uint32_t(kChunk)) {
#define FH_ORDER_SINGLE(IT)                                                                 \
  order_single<IT>(Nb, gbase, b, hb, vb, kinv, kmask, tiles, part, log_base, latest, sk, sv, \
                   dep_sorted, s_a, s_b, s_h, s_db, s_rs, s_src)
    if (Nb <= 2048) FH_ORDER_SINGLE(2);
    else if (Nb <= 4096) FH_ORDER_SINGLE(4);
    else if (Nb <= 8192) FH_ORDER_SINGLE(8);
    else FH_ORDER_SINGLE(16);
#undef FH_ORDER_SINGLE
    FH_STAMP_END(1, Nb);
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
    gather_runs(part, s_rs, s_src, tiles, c0, c, s_a);
    __syncthreads();
    const uint32_t *S = sort_chunk<16>(s_a, s_b, c, vb, hb, s_h, s_db);
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
      sk[pos] = (mk * kinv) & kmask;
      sv[pos] = vid;
      dep_sorted[pos] = dep;
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
  for (uint32_t k = tid; k < H; k += kOThreads)
    if (g_ccnt[k]) latest[(b << hb) | k] = kLogFlag | (log_base + g_clast[k]);
  FH_STAMP_END(1, Nb);
}

template <int BB>
__global__ void __launch_bounds__(kThreads)
    k_kb_partition(uint32_t n, int bb, int hb, int vb, uint32_t kmul, uint32_t kmask,
                   const uint32_t *__restrict__ key32, const uint64_t *__restrict__ dot,
                   uint32_t *__restrict__ part, uint16_t *__restrict__ toff,
                   unsigned long long *__restrict__ clk) {
  __shared__ __align__(16) unsigned char smem[PartSmem<BB>::bytes];
  partition_tile<BB>(blockIdx.x, n, bb, hb, vb, kmul, kmask, key32, dot, part, toff, clk, smem);
}

__global__ void __launch_bounds__(kOThreads)
    k_kb_order(uint32_t tiles, int bb, int hb, int vb, uint32_t kinv, uint32_t kmask,
               const uint32_t *__restrict__ part, const uint16_t *__restrict__ toff,
               uint64_t log_base, uint64_t *__restrict__ latest, uint32_t *__restrict__ sk,
               uint32_t *__restrict__ sv, uint64_t *__restrict__ dep_sorted,
               uint32_t *__restrict__ mc, unsigned long long *__restrict__ clk_fold,
               unsigned long long *__restrict__ frontier,
               unsigned long long *__restrict__ excount) {
  __shared__ __align__(16) unsigned char smem[OrderSmem::bytes];
  order_bucket(blockIdx.x, tiles, bb, hb, vb, kinv, kmask, part, toff, log_base, latest, sk, sv,
               dep_sorted, mc, clk_fold, frontier, excount, smem);
}

// One launch per pipelined step: workgroups [0, B) order batch b (its
// partition is in workspace wa), workgroups [B, B + tiles') partition batch
// b+1 into the other workspace.  The two roles touch disjoint memory.
template <int BB>
__global__ void __launch_bounds__(kOThreads)
    k_kb_step(uint32_t B_order, uint32_t tiles, int bb, int hb, int vb, uint32_t kinv,
              uint32_t kmask, const uint32_t *__restrict__ part, const uint16_t *__restrict__ toff,
              uint64_t log_base, uint64_t *__restrict__ latest, uint32_t *__restrict__ sk,
              uint32_t *__restrict__ sv, uint64_t *__restrict__ dep_sorted,
              uint32_t *__restrict__ mc, unsigned long long *__restrict__ clk_fold,
              unsigned long long *__restrict__ frontier, unsigned long long *__restrict__ excount,
              uint32_t n2, int bb2, int hb2, int vb2, uint32_t kmul2,
              uint32_t kmask2, const uint32_t *__restrict__ key32_2,
              const uint64_t *__restrict__ dot_2, uint32_t *__restrict__ part2,
              uint16_t *__restrict__ toff2, unsigned long long *__restrict__ clk) {
  __shared__ __align__(16) unsigned char smem[kSmemBytes];
  if (blockIdx.x < B_order)
    order_bucket(blockIdx.x, tiles, bb, hb, vb, kinv, kmask, part, toff, log_base, latest, sk,
                 sv, dep_sorted, mc, clk_fold, frontier, excount, smem);
  else
    partition_tile<BB>(blockIdx.x - B_order, n2, bb2, hb2, vb2, kmul2, kmask2, key32_2, dot_2,
                       part2, toff2, clk, smem);
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
  // >= 256 buckets when the key space allows, at most 4096 keys per bucket
  p.bb = std::min(kb, 8);
  p.hb = kb - p.bb;
  if (p.hb > kSlotBits) {
    p.hb = kSlotBits;
    p.bb = kb - kSlotBits;
  }
  p.vb = bits_for(n ? n : 1);
  p.tiles = uint32_t((n + kTile - 1) / kTile);
  keybucket_map(kb, &p.kmul, &p.kinv, &p.kmask);
  p.ok = n >= 1 && n < (size_t(1) << 30) && kb >= 1 && kb <= 22 && p.bb <= 10 &&
         p.hb + p.vb <= 32 && p.tiles <= uint32_t(kMaxTiles);
  return p;
}

void keybucket_partition(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32,
                         const uint64_t *dot, unsigned long long *clk, KeyBucketWorkspace &ws,
                         hipStream_t s) {
  FH_CHECK(p.ok, FH_EINVARIANT, "keybucket: batch does not fit the bucket plan");
  if (n == 0) return;
  const uint32_t B = 1u << p.bb;
  uint32_t *part = ws.part.ensure(size_t(n) + 1);
  uint16_t *toff = ws.toff.ensure(size_t(p.tiles) * (B + 1) + 1);
  auto k1 = p.bb <= 8 ? k_kb_partition<8> : k_kb_partition<10>;
  // read key (4) + dot (8), write the packed element (4)
  probed_launch("kb_partition", double(n) * 16.0, k1, dim3(p.tiles), dim3(kThreads), s, n, p.bb,
                p.hb, p.vb, p.kmul, p.kmask, key32, dot, part, toff, clk);
}

void keybucket_order(const KeyBucketPlan &p, uint32_t n, uint64_t log_base, uint64_t *latest,
                     KeyBucketWorkspace &ws, uint32_t *sk, uint32_t *sv, uint64_t *dep_sorted,
                     const KeyBucketClock &clock, hipStream_t s) {
  FH_CHECK(p.ok, FH_EINVARIANT, "keybucket: batch does not fit the bucket plan");
  if (n == 0) return;
  const uint32_t B = 1u << p.bb;
  // slot tables of buckets larger than one LDS chunk (rare; Zipf-hot keys)
  uint32_t *mc = ws.mc.ensure(size_t(B) * 4 * (size_t(1) << kSlotBits));
  // read the packed element (4), write key + command index + dependency (16)
  probed_launch("kb_order", double(n) * 20.0, k_kb_order, dim3(B), dim3(kOThreads), s, p.tiles,
                p.bb, p.hb, p.vb, p.kinv, p.kmask, (const uint32_t *)ws.part.get(),
                (const uint16_t *)ws.toff.get(), log_base, latest, sk, sv, dep_sorted, mc,
                clock.fold, clock.frontier, clock.excount);
}

void keybucket_step(const KeyBucketPlan &p, uint32_t n, uint64_t log_base, uint64_t *latest,
                    KeyBucketWorkspace &ws, uint32_t *sk, uint32_t *sv, uint64_t *dep_sorted,
                    const KeyBucketClock &clock, const KeyBucketPlan &p2, uint32_t n2,
                    const uint32_t *key32_2, const uint64_t *dot_2, unsigned long long *clk,
                    KeyBucketWorkspace &ws2, hipStream_t s) {
  FH_CHECK(p.ok && p2.ok, FH_EINVARIANT, "keybucket: batch does not fit the bucket plan");
  const uint32_t B = 1u << p.bb, B2 = 1u << p2.bb;
  uint32_t *mc = ws.mc.ensure(size_t(B) * 4 * (size_t(1) << kSlotBits));
  uint32_t *part2 = ws2.part.ensure(size_t(n2) + 1);
  uint16_t *toff2 = ws2.toff.ensure(size_t(p2.tiles) * (B2 + 1) + 1);
  auto k = p2.bb <= 8 ? k_kb_step<8> : k_kb_step<10>;
  // order (20 B / command of batch b) + partition (16 B / command of b+1)
  probed_launch("kb_step", double(n) * 20.0 + double(n2) * 16.0, k, dim3(B + p2.tiles),
                dim3(kOThreads), s, B, p.tiles, p.bb, p.hb, p.vb, p.kinv, p.kmask,
                (const uint32_t *)ws.part.get(), (const uint16_t *)ws.toff.get(), log_base, latest,
                sk, sv, dep_sorted, mc, clock.fold, clock.frontier, clock.excount, n2, p2.bb, p2.hb,
                p2.vb, p2.kmul, p2.kmask, key32_2, dot_2, part2, toff2, clk);
}

void keybucket_run(const KeyBucketPlan &p, uint32_t n, const uint32_t *key32, const uint64_t *dot,
                   uint64_t log_base, uint64_t *latest, const KeyBucketClock &clock,
                   KeyBucketWorkspace &ws, uint32_t *sk, uint32_t *sv, uint64_t *dep_sorted,
                   hipStream_t s) {
  keybucket_partition(p, n, key32, dot, clock.fold, ws, s);
  keybucket_order(p, n, log_base, latest, ws, sk, sv, dep_sorted, clock, s);
}

}  // namespace fh
