// srcstats.h -- per-source (max sequence, count) of a batch's dots: the
// fused engine's executed-clock advance (every batch executes completely).
// Sources 1..kRegSrc accumulate in registers (a batch has few sources: n of
// the configuration), others in LDS; flush() reduces each source over the
// wave and adds it to the workgroup's LDS partials, commit() folds those into
// the global (max, count) arrays with one atomic per source per workgroup.
// (Per-element LDS atomics serialised on the ~5 hot addresses: 365 us at
// 100M; a ballot loop per wave was compute bound.)
#pragma once

#include "fh_common.h"

namespace fh {

constexpr int kRegSrc = 8;

struct SrcAcc {
  uint64_t mx[kRegSrc];
  uint32_t cnt[kRegSrc];
  unsigned long long *s_mx;  // [256] LDS
  unsigned int *s_cnt;       // [256] LDS

  // every thread of the block; a barrier must follow before add()
  __device__ __forceinline__ void init(unsigned long long *smx, unsigned int *scnt) {
    s_mx = smx;
    s_cnt = scnt;
#pragma unroll
    for (int q = 0; q < kRegSrc; q++) mx[q] = 0, cnt[q] = 0;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_mx[i] = 0, s_cnt[i] = 0;
  }
  __device__ __forceinline__ void add(uint64_t d) {
    const uint32_t src = uint32_t(d >> 56);
    const uint64_t seq = d & 0x00FFFFFFFFFFFFFFull;
    if (src >= 1 && src <= uint32_t(kRegSrc)) {
#pragma unroll
      for (int q = 0; q < kRegSrc; q++)
        if (src == uint32_t(q + 1)) {
          mx[q] = seq > mx[q] ? seq : mx[q];
          cnt[q]++;
        }
    } else {
      atomicMax(&s_mx[src], (unsigned long long)seq);
      atomicAdd(&s_cnt[src], 1u);
    }
  }
  // every thread of the block (wave shuffles + a barrier inside)
  __device__ __forceinline__ void commit(unsigned long long *gmx, unsigned int *gcnt) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < kRegSrc; q++) {
      uint64_t m = mx[q];
      uint32_t c = cnt[q];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t m2 = __shfl_xor(m, o, 64);
        m = m2 > m ? m2 : m;
        c += __shfl_xor(c, o, 64);
      }
      if (lane == 0 && c) {
        atomicMax(&s_mx[q + 1], (unsigned long long)m);
        atomicAdd(&s_cnt[q + 1], c);
      }
    }
    __syncthreads();
    for (int s = threadIdx.x; s < 256; s += blockDim.x)
      if (s_cnt[s]) {
        atomicMax(&gmx[s], s_mx[s]);
        atomicAdd(&gcnt[s], s_cnt[s]);
      }
  }
};

}  // namespace fh
