// latbench.hip -- latency microbenchmarks behind the bucket-kernel design
// (diagnostic only): dependent global loads (pointer chase over a buffer of a
// given size), dependent LDS loads, and __syncthreads with 1024 threads, each
// with one workgroup alone and with every CU busy.  Times from
// s_memrealtime (100 MHz) per workgroup, reported as ns per step.
// Usage: latbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

constexpr int kSteps = 256;

__global__ void __launch_bounds__(1024) k_chase(const uint32_t *next, uint32_t start_stride,
                                                unsigned long long *out) {
  // every wave chases its own chain; lane 0's time is recorded
  uint32_t p = (blockIdx.x * 16 + (threadIdx.x >> 6)) * start_stride + (threadIdx.x & 63);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < kSteps; i++) p = next[p];
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = (t1 - t0) + (p == 0xFFFFFFFFu);
}

__global__ void __launch_bounds__(1024) k_lds(uint32_t seed, unsigned long long *out) {
  __shared__ uint32_t s[16384];
  for (int i = threadIdx.x; i < 16384; i += 1024) s[i] = (i * 2654435761u + seed) & 16383;
  __syncthreads();
  uint32_t p = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < kSteps; i++) p = s[p];
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = (t1 - t0) + (p == 0xFFFFFFFFu);
}

__global__ void __launch_bounds__(1024) k_barrier(unsigned long long *out) {
  __shared__ uint32_t s[1024];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  uint32_t acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < kSteps; i++) {
    acc += s[(threadIdx.x + i) & 1023];
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = (t1 - t0) + (acc == 0xFFFFFFFFu);
}

static void report(const char *name, unsigned long long *d, int n) {
  std::vector<unsigned long long> h(n);
  (void)hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-40s ns/step: p50 %.1f p90 %.1f max %.1f\n", name, h[n / 2] * 10.0 / kSteps,
         h[n * 9 / 10] * 10.0 / kSteps, h[n - 1] * 10.0 / kSteps);
}

int main() {
  unsigned long long *out;
  (void)hipMalloc(&out, 4096 * 16 * 8);
  const size_t sizes[] = {size_t(1) << 20, size_t(16) << 20, size_t(256) << 20, size_t(2) << 30};
  for (size_t bytes : sizes) {
    // random cyclic permutation within each lane's stripe, strided so lanes
    // touch different lines: element i -> next element in its chain
    const size_t n = bytes / 4;
    std::vector<uint32_t> next(n);
    std::vector<uint32_t> perm(n / 64);
    std::iota(perm.begin(), perm.end(), 0u);
    std::mt19937 rng(1);
    std::shuffle(perm.begin(), perm.end(), rng);
    for (size_t i = 0; i < perm.size(); i++)
      for (int l = 0; l < 64; l++)
        next[size_t(perm[i]) * 64 + l] = perm[(i + 1) % perm.size()] * 64 + l;
    uint32_t *d;
    (void)hipMalloc(&d, bytes);
    (void)hipMemcpy(d, next.data(), bytes, hipMemcpyHostToDevice);
    const uint32_t stride = uint32_t(n / (4096 * 16)) & ~63u;
    char nm[96];
    for (int grid : {1, 256, 1024}) {
      k_chase<<<grid, 1024>>>(d, stride, out);  // warm
      k_chase<<<grid, 1024>>>(d, stride, out);
      (void)hipDeviceSynchronize();
      snprintf(nm, sizeof nm, "global chase %zu MiB, %d WGs", bytes >> 20, grid);
      report(nm, out, grid * 16);
    }
    (void)hipFree(d);
  }
  for (int grid : {1, 256}) {
    k_lds<<<grid, 1024>>>(7, out);
    (void)hipDeviceSynchronize();
    char nm[96];
    snprintf(nm, sizeof nm, "LDS chase, %d WGs", grid);
    report(nm, out, grid * 16);
    k_barrier<<<grid, 1024>>>(out);
    (void)hipDeviceSynchronize();
    snprintf(nm, sizeof nm, "LDS read + __syncthreads, %d WGs", grid);
    report(nm, out, grid * 16);
  }
  return 0;
}
