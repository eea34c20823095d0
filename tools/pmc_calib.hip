// pmc_calib.hip -- known-byte-count kernels for calibrating rocprofv3's
// FETCH_SIZE / WRITE_SIZE on gfx950 at the access widths the engine uses
// (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only after a x2 correction
// for 16-B/lane streams; other widths are uncalibrated until measured).
//
// Each kernel streams exactly kBytes (1 GiB, far past the 256 MiB Infinity
// Cache) once; tools/collect_pmc.py divides the counter by kBytes to get the
// read / write factor per access width.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr size_t kBytes = size_t(1) << 30;

template <class T>
__global__ void __launch_bounds__(256) calib_read(const T *__restrict__ a, size_t n,
                                                  uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    const T v = a[i];
    const uint32_t *w = reinterpret_cast<const uint32_t *>(&v);
#pragma unroll
    for (unsigned j = 0; j < sizeof(T) / 4; j++) acc ^= w[j];
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;  // keeps the loads alive
}

template <class T>
__global__ void __launch_bounds__(256) calib_write(T *__restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    T v;
    uint32_t *w = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
    for (unsigned j = 0; j < sizeof(T) / 4; j++) w[j] = uint32_t(i) + j;
    a[i] = v;
  }
}

// Random gathers and scatters (the engine's union, fill and code stores):
// element i reads / writes slot perm(i) of the same 1 GiB buffer, a
// bijection that puts every lane of a wave on a different line, so each
// access costs a line from HBM while the algorithmic bytes stay sizeof(T) per
// element.  The counters divided by kBytes give the gather / scatter factors
// (bytes counted per algorithmic byte) that make a gather kernel's FETCH_SIZE
// comparable with its byte count.
__device__ __forceinline__ size_t calib_perm(size_t i, size_t n) {
  return size_t((uint64_t(i) * 0x9E3779B1ull + 12345ull) % n);
}

template <class T>
__global__ void __launch_bounds__(256) calib_gather(const T *__restrict__ a, size_t n,
                                                    uint32_t *__restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    const T v = a[calib_perm(i, n)];
    const uint32_t *w = reinterpret_cast<const uint32_t *>(&v);
#pragma unroll
    for (unsigned j = 0; j < sizeof(T) / 4; j++) acc ^= w[j];
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

template <class T>
__global__ void __launch_bounds__(256) calib_scatter(T *__restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    T v;
    uint32_t *w = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
    for (unsigned j = 0; j < sizeof(T) / 4; j++) w[j] = uint32_t(i) + j;
    a[calib_perm(i, n)] = v;
  }
}

int main() {
  void *buf = nullptr;
  uint32_t *sink = nullptr;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(buf, 1, kBytes));
  const unsigned grid = 256 * 16;
  for (int rep = 0; rep < 3; rep++) {
    calib_read<uint32_t><<<grid, 256>>>((const uint32_t *)buf, kBytes / 4, sink);
    CK(hipDeviceSynchronize());
    calib_read<uint2><<<grid, 256>>>((const uint2 *)buf, kBytes / 8, sink);
    CK(hipDeviceSynchronize());
    calib_read<uint4><<<grid, 256>>>((const uint4 *)buf, kBytes / 16, sink);
    CK(hipDeviceSynchronize());
    calib_write<uint32_t><<<grid, 256>>>((uint32_t *)buf, kBytes / 4);
    CK(hipDeviceSynchronize());
    calib_write<uint2><<<grid, 256>>>((uint2 *)buf, kBytes / 8);
    CK(hipDeviceSynchronize());
    calib_write<uint4><<<grid, 256>>>((uint4 *)buf, kBytes / 16);
    CK(hipDeviceSynchronize());
    calib_gather<uint32_t><<<grid, 256>>>((const uint32_t *)buf, kBytes / 4, sink);
    CK(hipDeviceSynchronize());
    calib_gather<uint2><<<grid, 256>>>((const uint2 *)buf, kBytes / 8, sink);
    CK(hipDeviceSynchronize());
    calib_scatter<uint32_t><<<grid, 256>>>((uint32_t *)buf, kBytes / 4);
    CK(hipDeviceSynchronize());
    calib_scatter<uint2><<<grid, 256>>>((uint2 *)buf, kBytes / 8);
    CK(hipDeviceSynchronize());
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  printf("pmc_calib: %zu bytes per kernel\n", kBytes);
  return 0;
}
