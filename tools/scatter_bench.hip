// scatter_bench.hip -- what a key-order -> command-order transition costs on
// MI355X.  The engine's KeyDeps runs in (key, command) order and its outputs
// are indexed by command, so every design pays one such transition per
// command; this measures its forms at the C4 size (100M commands):
//   scatterB   one B-byte store per element at a random command slot;
//   region     the same, but each workgroup's destinations confined to one
//              region of R commands (the second half of a coarse bucket pass);
//   gatherB    one B-byte read per element from a random command slot;
//   copy16     a coalesced 16-B-per-lane copy (the streaming reference).
// Destinations: i -> (i * A + B) mod N (A odd and coprime to N), so every
// lane of a wave writes a different line.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr uint64_t kA = 0x9E3779B1ull;  // odd, coprime to the N used

__device__ __forceinline__ uint32_t perm(uint64_t i, uint64_t n) { return uint32_t((i * kA + 12345) % n); }

__global__ void __launch_bounds__(256) k_scatter12(uint32_t n, uint32_t *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t d = perm(i, n);
  *reinterpret_cast<HIP_vector_type<uint32_t, 3> *>(o + size_t(d) * 3) =
      HIP_vector_type<uint32_t, 3>(i, i + 1, i + 2);
}
__global__ void __launch_bounds__(256) k_scatter4(uint32_t n, uint32_t *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  o[perm(i, n)] = i;
}
__global__ void __launch_bounds__(256) k_scatter16(uint32_t n, uint4 *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  o[perm(i, n)] = make_uint4(i, i + 1, i + 2, i + 3);
}
__global__ void __launch_bounds__(256) k_scatter32(uint32_t n, uint4 *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t d = perm(i, n);
  o[2 * size_t(d)] = make_uint4(i, i + 1, i + 2, i + 3);
  o[2 * size_t(d) + 1] = make_uint4(i, i + 1, i + 2, i + 3);
}
// destinations of block b confined to region (b * 256 / R) of R slots
__global__ void __launch_bounds__(256) k_region12(uint32_t n, uint32_t R, uint32_t *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t base = (i / R) * R, len = min(R, n - base);
  const uint32_t d = base + perm(i - base, len);
  *reinterpret_cast<HIP_vector_type<uint32_t, 3> *>(o + size_t(d) * 3) =
      HIP_vector_type<uint32_t, 3>(i, i + 1, i + 2);
}
__global__ void __launch_bounds__(256) k_region16(uint32_t n, uint32_t R, uint4 *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t base = (i / R) * R, len = min(R, n - base);
  o[base + perm(i - base, len)] = make_uint4(i, i + 1, i + 2, i + 3);
}
__global__ void __launch_bounds__(256) k_gather8(uint32_t n, const uint64_t *__restrict__ a,
                                                 uint64_t *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  o[i] = a[perm(i, n)];
}
__global__ void __launch_bounds__(256) k_gather4(uint32_t n, const uint32_t *__restrict__ a,
                                                 uint32_t *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  o[i] = a[perm(i, n)];
}
__global__ void __launch_bounds__(256) k_region_gather8(uint32_t n, uint32_t R, const uint64_t *__restrict__ a,
                                                        uint64_t *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t base = (i / R) * R, len = min(R, n - base);
  o[i] = a[base + perm(i - base, len)];
}
__global__ void __launch_bounds__(256) k_copy16(uint32_t n, const uint4 *__restrict__ a, uint4 *__restrict__ o) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  o[i] = a[i];
}

int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? uint32_t(atol(argv[1])) : 100000000u;
  void *a = nullptr, *b = nullptr;
  CK(hipMalloc(&a, size_t(n) * 32));
  CK(hipMalloc(&b, size_t(n) * 32));
  CK(hipMemset(a, 1, size_t(n) * 32));
  CK(hipMemset(b, 1, size_t(n) * 32));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((n + 255) / 256);
  auto time = [&](const char *name, double bytes, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9f, sum = 0;
    const int reps = 5;
    for (int r = 0; r < reps; r++) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    printf("{\"kernel\": \"%s\", \"n\": %u, \"best_ms\": %.4f, \"avg_ms\": %.4f, \"GBs\": %.1f, \"Gops\": %.2f}\n",
           name, n, best, sum / reps, bytes / (best * 1e-3) / 1e9, n / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  time("copy16", 32.0 * n, [&] { k_copy16<<<g, 256>>>(n, (const uint4 *)a, (uint4 *)b); });
  time("scatter4", 4.0 * n, [&] { k_scatter4<<<g, 256>>>(n, (uint32_t *)b); });
  time("scatter12", 12.0 * n, [&] { k_scatter12<<<g, 256>>>(n, (uint32_t *)b); });
  time("scatter16", 16.0 * n, [&] { k_scatter16<<<g, 256>>>(n, (uint4 *)b); });
  time("scatter32", 32.0 * n, [&] { k_scatter32<<<g, 256>>>(n, (uint4 *)b); });
  for (uint32_t R : {1u << 16, 1u << 18, 1u << 20, 1u << 22, 1u << 24}) {
    char nm[64];
    snprintf(nm, sizeof nm, "region12_R%u", R);
    time(nm, 12.0 * n, [&] { k_region12<<<g, 256>>>(n, R, (uint32_t *)b); });
    snprintf(nm, sizeof nm, "region16_R%u", R);
    time(nm, 16.0 * n, [&] { k_region16<<<g, 256>>>(n, R, (uint4 *)b); });
    snprintf(nm, sizeof nm, "region_gather8_R%u", R);
    time(nm, 16.0 * n, [&] { k_region_gather8<<<g, 256>>>(n, R, (const uint64_t *)a, (uint64_t *)b); });
  }
  time("gather8", 16.0 * n, [&] { k_gather8<<<g, 256>>>(n, (const uint64_t *)a, (uint64_t *)b); });
  time("gather4", 8.0 * n, [&] { k_gather4<<<g, 256>>>(n, (const uint32_t *)a, (uint32_t *)b); });
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
