// scan.hip -- single-pass exclusive scan for gfx950 (see scan.h).
#include "scan.h"

namespace fh {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;
constexpr uint32_t kAgg = 1u << 30;
constexpr uint32_t kInc = 2u << 30;
constexpr uint32_t kCnt = (1u << 30) - 1;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(kThreads)
    k_scan(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
           uint32_t *status) {
  __shared__ uint32_t s_wave[kThreads / 64];
  __shared__ uint32_t s_tile, s_prefix;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(&status[0], 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  // blocked arrangement: thread t owns items [base + t*kItems, +kItems)
  const uint32_t base = tile * kTile + uint32_t(tid) * kItems;
  uint32_t v[kItems];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + i;
    v[i] = idx < n ? in[idx] : 0u;
    sum += v[i];
  }
  // block exclusive scan of per-thread sums
  uint32_t x = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (lane == 63) s_wave[w] = x;
  __syncthreads();
  uint32_t wpre = 0, total = 0;
#pragma unroll
  for (int i = 0; i < kThreads / 64; i++) {
    if (i < w) wpre += s_wave[i];
    total += s_wave[i];
  }
  uint32_t texcl = wpre + x - sum;
  if (tid == 0) {
    uint32_t *my = status + 2 + tile;
    uint32_t excl = 0;
    if (tile == 0) {
      st_agent(my, kInc | total);
    } else {
      st_agent(my, kAgg | total);
      int t = int(tile) - 1;
      uint32_t spins = 0;
      while (t >= 0) {
        const uint32_t sv = ld_agent(status + 2 + t);
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
        if (++spins > (1u << 24)) {
          atomicOr(&status[1], 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      st_agent(my, kInc | (excl + total));
    }
    s_prefix = excl;
  }
  __syncthreads();
  uint32_t run = s_prefix + texcl;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const uint32_t idx = base + i;
    if (idx < n) out[idx] = run;
    run += v[i];
    if (idx + 1 == n) out[n] = run;
  }
}

}  // namespace

void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, ScanWorkspace &ws,
                        hipStream_t s) {
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "scan: too many elements");
  if (n == 0) {
    FH_HIP(hipMemsetAsync(out, 0, sizeof(uint32_t), s));
    return;
  }
  const size_t tiles = (n + kTile - 1) / kTile;
  uint32_t *st = ws.status.ensure(tiles + 2);
  FH_HIP(hipMemsetAsync(st, 0, (tiles + 2) * sizeof(uint32_t), s));
  k_scan<<<unsigned(tiles), kThreads, 0, s>>>(in, out, uint32_t(n), st);
}

}  // namespace fh
