// scan.hip -- exclusive prefix sum / prefix max for gfx950, reduce-then-scan
// (see scan.h).  Three launches (two up to 4M elements), no inter-workgroup hand-off inside a launch
// (cross-XCD hand-offs cost microseconds each on MI355X; a chained scan
// serialises on them).  The operator is a template parameter with identity 0
// (sum, or max over u32).
#include <cstdlib>

#include <atomic>
#include <type_traits>

#include "scan.h"

namespace fh {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;

struct OpAdd {
  static __device__ __forceinline__ uint32_t f(uint32_t a, uint32_t b) { return a + b; }
};
// Element loaders: a plain array, or run bounds (start, end | tag << 23)
// pairs whose value is the run length (0 for an entry of another tag)
struct LdPlain {
  const uint32_t *in;
  __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return in[i]; }
};
struct LdRuns {
  const uint2 *runs;
  uint32_t tag;
  __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
    const uint2 r = runs[i];
    return (r.y >> 23) == tag ? (r.y & 0x7FFFFFu) - r.x : 0u;
  }
};
struct OpMax {
  static __device__ __forceinline__ uint32_t f(uint32_t a, uint32_t b) { return a > b ? a : b; }
};

template <class Op>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_tmp,
                                                    uint32_t *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(x, o, 64);
    if (lane >= o) x = Op::f(x, t);
  }
  // exclusive value inside the wave
  uint32_t ex = __shfl_up(x, 1, 64);
  if (lane == 0) ex = 0;
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kThreads / 64; i++) {
    if (i < w) pre = Op::f(pre, s_tmp[i]);
    tot = Op::f(tot, s_tmp[i]);
  }
  __syncthreads();
  if (total) *total = tot;
  return Op::f(pre, ex);
}

template <class Op, class Ld>
__global__ void __launch_bounds__(kThreads)
    k_scan_reduce(const Ld in, uint32_t n, uint32_t *__restrict__ bsum) {
  __shared__ uint32_t s_tmp[kThreads / 64];
  const uint32_t base = blockIdx.x * kTile;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + i * kThreads + threadIdx.x;
    s = Op::f(s, idx < n ? in(idx) : 0u);
  }
  uint32_t tot = 0;
  block_excl_scan<Op>(s, s_tmp, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// One 1024-thread workgroup scans the block sums: each thread reduces a
// contiguous run of them (independent loads), one block-wide scan, then each
// thread rewrites its run.  (A 256-wide loop over the sums paid two barriers
// and a dependent load round per 256 blocks: ~0.2 ms at 100M elements.)
constexpr int kTopThreads = 1024;
template <class Op>
__global__ void __launch_bounds__(kTopThreads) k_scan_top(uint32_t *__restrict__ bsum, uint32_t nb) {
  __shared__ uint32_t s_w[kTopThreads / 64];
  const uint32_t per = (nb + kTopThreads - 1) / kTopThreads;
  const uint32_t b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
  uint32_t s = 0;
  for (uint32_t b = b0; b < b1; b += 8) {
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = b + i < b1 ? bsum[b + i] : 0u;
#pragma unroll
    for (int i = 0; i < 8; i++) s = Op::f(s, v[i]);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(x, o, 64);
    if (lane >= o) x = Op::f(x, t);
  }
  uint32_t ex = __shfl_up(x, 1, 64);
  if (lane == 0) ex = 0;
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  uint32_t run = 0;
  for (int i = 0; i < w; i++) run = Op::f(run, s_w[i]);
  run = Op::f(run, ex);
  for (uint32_t b = b0; b < b1; b++) {
    const uint32_t v = bsum[b];
    bsum[b] = run;
    run = Op::f(run, v);
  }
}

// Striped ownership (coalesced): wave w of the block owns the 1024
// consecutive elements [w·1024, (w+1)·1024) of the tile, item i of lane l is
// element w·1024 + i·64 + l.  Each item row is scanned across the wave with
// shuffles and chained by the row total (lane 63), then the waves' totals.
// (A blocked layout -- 16 consecutive elements per thread -- made every load
// instruction touch 64 lines: 382 us per 100M-element scan, 2 TB/s.)
// With LdRuns, delta[i] = out[i] - the run's start as well (the shift that
// moves a run from key-grouped positions to ascending-key positions).
template <class Op, class Ld>
__global__ void __launch_bounds__(kThreads)
    k_scan_down(const Ld in, uint32_t *__restrict__ out, uint32_t n,
                const uint32_t *__restrict__ bsum, uint32_t *__restrict__ delta, int inl) {
  __shared__ uint32_t s_tmp[kThreads / 64], s_top[kThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t base = blockIdx.x * kTile + uint32_t(w) * 64 * kItems;
  uint32_t v[kItems];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + i * 64 + lane;
    v[i] = idx < n ? in(idx) : 0u;
  }
  // inclusive scan of each row across the lanes, chained row to row
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    uint32_t x = v[i];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(x, o, 64);
      if (lane >= o) x = Op::f(x, t);
    }
    uint32_t ex = __shfl_up(x, 1, 64);
    if (lane == 0) ex = 0;
    const uint32_t row = __shfl(x, 63, 64);
    v[i] = Op::f(carry, ex);  // exclusive prefix inside the wave's run
    carry = Op::f(carry, row);
  }
  uint32_t pre;
  if (inl) {
    // few blocks: this block's prefix from the raw block sums (no k_scan_top
    // launch; a launch costs more than the ~nb/256 loads per thread)
    uint32_t t = 0;
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kThreads) t = Op::f(t, bsum[i]);
    block_excl_scan<Op>(t, s_top, &pre);
  } else {
    pre = bsum[blockIdx.x];
  }
  if (lane == 0) s_tmp[w] = carry;
  __syncthreads();
  for (int i = 0; i < w; i++) pre = Op::f(pre, s_tmp[i]);
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + i * 64 + lane;
    if (idx < n) {
      out[idx] = Op::f(pre, v[i]);
      if constexpr (std::is_same<Ld, LdRuns>::value)
        if (delta) delta[idx] = Op::f(pre, v[i]) - in.runs[idx].x;
    }
  }
  // out[n] = the total: the wave holding element n - 1 (its elements past
  // n - 1 are the identity)
  if (lane == 0 && n - 1 >= base && n - 1 < base + 64 * kItems) out[n] = Op::f(pre, carry);
}

template <class Op, class Ld>
void scan_impl(const Ld in, uint32_t *out, size_t n, ScanWorkspace &ws, hipStream_t s,
               uint32_t *delta = nullptr) {
  FH_CHECK(n < (size_t(1) << 31), FH_EINVAL, "scan: too many elements");
  if (n == 0) {
    FH_HIP(hipMemsetAsync(out, 0, sizeof(uint32_t), s));
    return;
  }
  const uint32_t nb = uint32_t((n + kTile - 1) / kTile);
  uint32_t *bsum = ws.status.ensure(nb + 1);
  k_scan_reduce<Op, Ld><<<nb, kThreads, 0, s>>>(in, uint32_t(n), bsum);
  const bool inl = nb <= 1024;  // (4M elements)
  if (!inl) k_scan_top<Op><<<1, kTopThreads, 0, s>>>(bsum, nb);
  k_scan_down<Op, Ld><<<nb, kThreads, 0, s>>>(in, out, uint32_t(n), bsum, delta, int(inl));
}

}  // namespace

void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws,
                        hipStream_t s) {
  scan_impl<OpAdd>(LdPlain{in}, out, n, ws, s);
}

void run_offsets(const uint32_t *runs, uint32_t tag, uint32_t *off, uint32_t *delta, size_t n,
                 ScanWorkspace &ws, hipStream_t s) {
  FH_CHECK(tag >= 1 && tag < 512, FH_EINVAL, "run_offsets: tag out of range");
  scan_impl<OpAdd>(LdRuns{reinterpret_cast<const uint2 *>(runs), tag}, off, n, ws, s, delta);
}

void exclusive_scan_max_u32(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws,
                            hipStream_t s) {
  scan_impl<OpMax>(LdPlain{in}, out, n, ws, s);
}

namespace {

__global__ void k_fetch_u32(const uint32_t *__restrict__ src, uint32_t *dst, int n,
                            uint32_t seq) {
  if (threadIdx.x != 0) return;
  for (int t = 0; t < n; t++)
    __hip_atomic_store(&dst[2 + t], src[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&dst[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Mailbox {
  uint32_t *host = nullptr;  // [0] sequence, [2..16) words
  uint32_t *dev = nullptr;
  uint32_t seq = 0;
  int device = -1;
  ~Mailbox() {
    if (host) (void)hipHostFree(host);
  }
};

}  // namespace

void fetch_u32(const uint32_t *dev, uint32_t *host, int n, hipStream_t s) {
  FH_CHECK(n >= 0 && n <= 14, FH_EINVAL, "fetch_u32: at most 14 words");
  // one mailbox per thread and device (handles are single-threaded)
  thread_local Mailbox mb[16];
  int d = 0;
  FH_HIP(hipGetDevice(&d));
  Mailbox &m = mb[d & 15];
  if (!m.host || m.device != d) {
    if (m.host) (void)hipHostFree(m.host);
    m.host = nullptr;
    FH_HIP(hipHostMalloc(reinterpret_cast<void **>(&m.host), 64,
                         hipHostMallocMapped | hipHostMallocCoherent));
    FH_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&m.dev), m.host, 0));
    m.device = d;
    m.seq = 0;
    __atomic_store_n(&m.host[0], 0u, __ATOMIC_RELEASE);
  }
  const uint32_t seq = ++m.seq;
  k_fetch_u32<<<1, 1, 0, s>>>(dev, m.dev, n, seq);
  FH_HIP(hipGetLastError());
  // (the word waits behind everything queued on the stream before it: a
  // generous deadline, for a kernel upstream that never ends)
  poll_completion(reinterpret_cast<volatile uint32_t *>(m.host), seq,
                  [&] { return hipStreamQuery(s); }, 600000.0, "fetch_u32: the stream");
  std::atomic_thread_fence(std::memory_order_acquire);
  for (int i = 0; i < n; i++) host[i] = __atomic_load_n(&m.host[2 + i], __ATOMIC_RELAXED);
}

}  // namespace fh
