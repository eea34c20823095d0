// scan.hip -- exclusive prefix sum / prefix max for gfx950, reduce-then-scan
// (see scan.h).  Three launches, no inter-workgroup hand-off inside a launch
// (cross-XCD hand-offs cost microseconds each on MI355X; a chained scan
// serialises on them).  The operator is a template parameter with identity 0
// (sum, or max over u32).
#include <cstdlib>

#include "scan.h"

namespace fh {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;

struct OpAdd {
  static __device__ __forceinline__ uint32_t f(uint32_t a, uint32_t b) { return a + b; }
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

template <class Op>
__global__ void __launch_bounds__(kThreads)
    k_scan_reduce(const uint32_t *__restrict__ in, uint32_t n, uint32_t *__restrict__ bsum) {
  __shared__ uint32_t s_tmp[kThreads / 64];
  const uint32_t base = blockIdx.x * kTile;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + i * kThreads + threadIdx.x;
    s = Op::f(s, idx < n ? in[idx] : 0u);
  }
  uint32_t tot = 0;
  block_excl_scan<Op>(s, s_tmp, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

template <class Op>
__global__ void __launch_bounds__(kThreads) k_scan_top(uint32_t *__restrict__ bsum, uint32_t nb) {
  __shared__ uint32_t s_tmp[kThreads / 64];
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += kThreads) {
    const uint32_t b = b0 + threadIdx.x;
    const uint32_t v = b < nb ? bsum[b] : 0u;
    uint32_t tot = 0;
    const uint32_t ex = block_excl_scan<Op>(v, s_tmp, &tot);
    if (b < nb) bsum[b] = Op::f(carry, ex);
    carry = Op::f(carry, tot);
  }
}

template <class Op>
__global__ void __launch_bounds__(kThreads)
    k_scan_down(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
                const uint32_t *__restrict__ bsum) {
  __shared__ uint32_t s_tmp[kThreads / 64];
  // blocked: thread t owns kItems consecutive elements
  const uint32_t base = blockIdx.x * kTile + threadIdx.x * kItems;
  uint32_t v[kItems];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + i;
    v[i] = idx < n ? in[idx] : 0u;
    s = Op::f(s, v[i]);
  }
  uint32_t run = Op::f(bsum[blockIdx.x], block_excl_scan<Op>(s, s_tmp, nullptr));
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + i;
    if (idx < n) out[idx] = run;
    run = Op::f(run, v[i]);
    if (idx + 1 == n) out[n] = run;
  }
}

template <class Op>
void scan_impl(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws, hipStream_t s) {
  FH_CHECK(n < (size_t(1) << 31), FH_EINVAL, "scan: too many elements");
  if (n == 0) {
    FH_HIP(hipMemsetAsync(out, 0, sizeof(uint32_t), s));
    return;
  }
  const uint32_t nb = uint32_t((n + kTile - 1) / kTile);
  uint32_t *bsum = ws.status.ensure(nb + 1);
  k_scan_reduce<Op><<<nb, kThreads, 0, s>>>(in, uint32_t(n), bsum);
  k_scan_top<Op><<<1, kThreads, 0, s>>>(bsum, nb);
  k_scan_down<Op><<<nb, kThreads, 0, s>>>(in, out, uint32_t(n), bsum);
}

}  // namespace

void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws,
                        hipStream_t s) {
  scan_impl<OpAdd>(in, out, n, ws, s);
}

void exclusive_scan_max_u32(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws,
                            hipStream_t s) {
  scan_impl<OpMax>(in, out, n, ws, s);
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
  static const char *ab = getenv("FH_FETCH_MEMCPY");  // A/B measurement
  static const bool use_memcpy = ab && *ab && *ab != '0';
  if (use_memcpy) {
    FH_HIP(hipMemcpyAsync(host, dev, size_t(n) * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    FH_HIP(hipStreamSynchronize(s));
    return;
  }
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
  for (;;) {
    if (__atomic_load_n(&m.host[0], __ATOMIC_ACQUIRE) == seq) break;
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) {
      // the stream drained: the store must be visible now
      FH_CHECK(__atomic_load_n(&m.host[0], __ATOMIC_ACQUIRE) == seq, FH_EHIP,
               "fetch_u32: mailbox not written");
      break;
    }
    if (e != hipErrorNotReady) throw Error(FH_EHIP, std::string("fetch_u32: ") + hipGetErrorString(e));
  }
  for (int i = 0; i < n; i++) host[i] = __atomic_load_n(&m.host[2 + i], __ATOMIC_RELAXED);
}

}  // namespace fh
