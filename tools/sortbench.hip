// sortbench.hip -- standalone timing of fh::sort_pairs (u32 keys, iota values)
// for A/B of tile shapes (FH_SORT_CFG) and sizes.  Verifies sortedness.
//   build: see tools/build_tools.sh   run: ./sortbench n bits cfgs iters
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "sort.h"

using namespace fh;

int main(int argc, char **argv) {
  size_t n = argc > 1 ? std::stoul(argv[1]) : 1000000;
  int bits = argc > 2 ? std::atoi(argv[2]) : 20;
  std::string cfgs = argc > 3 ? argv[3] : "0,1,2,3,4";
  int iters = argc > 4 ? std::atoi(argv[4]) : 20;
  double zipf = argc > 5 ? std::atof(argv[5]) : 0.7;
  std::vector<uint32_t> h(n);
  // zipf-ish keys (inverse-power sampling) or uniform
  std::mt19937_64 rng(1);
  uint32_t K = 1u << bits;
  std::vector<double> cdf(K);
  double s = 0;
  for (uint32_t r = 0; r < K; r++) {
    s += zipf > 0 ? std::pow(double(r + 1), -zipf) : 1.0;
    cdf[r] = s;
  }
  std::uniform_real_distribution<double> U(0, s);
  for (size_t i = 0; i < n; i++)
    h[i] = uint32_t(std::lower_bound(cdf.begin(), cdf.end(), U(rng)) - cdf.begin());
  uint32_t *dk, *ka, *kb, *va, *vb;
  hipMalloc(&dk, n * 4);
  hipMalloc(&ka, n * 4);
  hipMalloc(&kb, n * 4);
  hipMalloc(&va, n * 4);
  hipMalloc(&vb, n * 4);
  hipMemcpy(dk, h.data(), n * 4, hipMemcpyHostToDevice);
  hipStream_t st;
  hipStreamCreate(&st);
  SortWorkspace ws;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<int> cl;
  for (size_t p = 0; p < cfgs.size(); p++)
    if (isdigit(cfgs[p])) cl.push_back(cfgs[p] - '0');
  for (int round = 0; round < 3; round++)
    for (int c : cl) {
      setenv("FH_SORT_CFG", std::to_string(c).c_str(), 1);
      uint32_t *ko, *vo;
      sort_pairs<uint32_t, uint32_t>(dk, nullptr, ka, va, kb, vb, n, bits, ws, st, &ko, &vo);
      hipEventRecord(e0, st);
      for (int i = 0; i < iters; i++)
        sort_pairs<uint32_t, uint32_t>(dk, nullptr, ka, va, kb, vb, n, bits, ws, st, &ko, &vo);
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      std::vector<uint32_t> ok(n), ov(n);
      hipMemcpy(ok.data(), ko, n * 4, hipMemcpyDeviceToHost);
      hipMemcpy(ov.data(), vo, n * 4, hipMemcpyDeviceToHost);
      bool good = true;
      for (size_t i = 1; i < n && good; i++)
        good = ok[i - 1] < ok[i] || (ok[i - 1] == ok[i] && ov[i - 1] < ov[i]);
      for (size_t i = 0; i < n && good; i++) good = h[ov[i]] == ok[i];
      printf("round %d cfg %d n %zu bits %d: %.2f us/sort  %s\n", round, c, n, bits,
             ms * 1e3 / iters, good ? "sorted+stable" : "WRONG");
    }
  return 0;
}
