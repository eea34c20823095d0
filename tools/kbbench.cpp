// kbbench.cpp -- diagnostic harness for the two single-view bucket kernels.
// Builds keybucket.hip with per-workgroup stamps (FH_KB_STAMPS) and reports
// kernel times (HIP events) and the distribution of workgroup durations.
// Usage: kbbench keys.u32 dots.u64 n key_bits [reps]
#define FH_KB_STAMPS 1
#include "../fantoch_amd/csrc/keybucket.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <vector>

namespace fh {
thread_local Probe *t_probe = nullptr;
}

using namespace fh;

static std::vector<char> slurp(const char *path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static void report(const char *name, const std::vector<unsigned long long> &st, size_t nwg) {
  std::vector<double> dur;
  unsigned long long t0 = ~0ull, t1 = 0, last_start = 0;
  size_t imax = 0;
  double dmax = 0;
  for (size_t i = 0; i < nwg; i++) {
    const double d = double(st[3 * i + 1] - st[3 * i]) * 0.01;  // us
    dur.push_back(d);
    t0 = std::min(t0, st[3 * i]);
    t1 = std::max(t1, st[3 * i + 1]);
    last_start = std::max(last_start, st[3 * i]);
    if (d > dmax) {
      dmax = d;
      imax = i;
    }
  }
  std::vector<double> s = dur;
  std::sort(s.begin(), s.end());
  printf("%s: %zu WGs span %.2f us; WG dur p10 %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f "
         "(wg %zu work %llu); last start at +%.2f us\n",
         name, nwg, double(t1 - t0) * 0.01, s[nwg / 10], s[nwg / 2], s[nwg * 9 / 10],
         s[nwg * 99 / 100], dmax, imax, st[3 * imax + 2], double(last_start - t0) * 0.01);
  // start-time histogram (4 us bins)
  std::vector<int> hist(64, 0);
  for (size_t i = 0; i < nwg; i++) {
    size_t bin = size_t(double(st[3 * i] - t0) * 0.01 / 4.0);
    hist[std::min<size_t>(bin, 63)]++;
  }
  printf("  starts per 4us:");
  for (int i = 0; i < 64; i++)
    if (hist[i]) printf(" [%d]=%d", i, hist[i]);
  printf("\n");
}

int main(int argc, char **argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: kbbench keys.u32 dots.u64 n key_bits [reps]\n");
    return 2;
  }
  auto kbuf = slurp(argv[1]);
  auto dbuf = slurp(argv[2]);
  const uint32_t n = uint32_t(atol(argv[3]));
  const int kb = atoi(argv[4]);
  const int reps = argc > 5 ? atoi(argv[5]) : 10;
  if (kbuf.size() < size_t(n) * 4 || dbuf.size() < size_t(n) * 8) {
    fprintf(stderr, "short input\n");
    return 2;
  }
  KeyBucketPlan p = keybucket_plan(n, kb);
  if (!p.ok) {
    fprintf(stderr, "plan not ok\n");
    return 2;
  }
  printf("plan: bb %d hb %d vb %d tiles %u\n", p.bb, p.hb, p.vb, p.tiles);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  uint32_t *key32, *sk, *sv;
  uint64_t *dot, *latest, *dep;
  unsigned long long *fr, *ex, *st0, *st1;
  const uint32_t B = (1u << p.bb) + kHot;  // order workgroups (regular + hot-key buckets)
  (void)hipMalloc(&key32, n * 4);
  (void)hipMalloc(&dot, n * 8);
  (void)hipMalloc(&sk, n * 4);
  (void)hipMalloc(&sv, n * 4);
  (void)hipMalloc(&dep, n * 8);
  (void)hipMalloc(&latest, (size_t(1) << kb) * 8);
  (void)hipMalloc(&fr, 8 * 512 * 8);
  (void)hipMalloc(&ex, 256 * 8);
  (void)hipMalloc(&st0, p.tiles * 3 * 8);
  (void)hipMalloc(&st1, B * 3 * 8);
  (void)hipMemcpy(key32, kbuf.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dot, dbuf.data(), n * 8, hipMemcpyHostToDevice);
  (void)hipMemset(latest, 0, (size_t(1) << kb) * 8);
  (void)hipMemset(fr, 0, 8 * 512 * 8);
  (void)hipMemset(ex, 0, 256 * 8);
  unsigned long long *hst[2] = {st0, st1};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kb_stamps), hst, sizeof(hst));
  unsigned long long *ph0, *ph1;
  // phase rows are indexed by blockIdx.x: the fused step puts tiles after B
  (void)hipMalloc(&ph0, (p.tiles + B) * 8 * 8);
  (void)hipMalloc(&ph1, (p.tiles + B) * 8 * 8);
  (void)hipMemset(ph0, 0, (p.tiles + B) * 8 * 8);
  (void)hipMemset(ph1, 0, (p.tiles + B) * 8 * 8);
  unsigned long long *hph[2] = {ph0, ph1};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kb_phase), hph, sizeof(hph));
  KeyBucketWorkspace ws;
  unsigned long long *frt, *exc;
  (void)hipMalloc(&frt, 256 * 8);
  (void)hipMalloc(&exc, 256 * 8);
  (void)hipMemset(frt, 0, 256 * 8);
  (void)hipMemset(exc, 0, 256 * 8);
  KeyBucketClock clock;
  clock.fold = fr;
  clock.frontier = frt;
  clock.excount = exc;
  const bool step = getenv("KB_STEP") != nullptr;
  // KB_SCHED: largest-first schedule from one untimed warm-up launch
  KeyBucketSched sched, *sc = getenv("KB_SCHED") ? &sched : nullptr;
  if (sc) {
    keybucket_run(p, n, key32, dot, 0, latest, clock, ws, sk, sv, dep, s, sc);
    keybucket_sched(sched, s);
  }
  Probe probe;
  probe.set("kb_partition,kb_order,kb_step");
  if (!step) {
    t_probe = &probe;
    for (int r = 0; r < reps; r++)
      keybucket_run(p, n, key32, dot, 0, latest, clock, ws, sk, sv, dep, s, sc);
  } else {
    // fused steps: each launch orders the batch partitioned by the previous
    // one and partitions the same input again into the other workspace
    KeyBucketWorkspace ws2;
    unsigned long long *fr2;
    (void)hipMalloc(&fr2, 8 * 512 * 8);
    (void)hipMemset(fr2, 0, 8 * 512 * 8);
    KeyBucketWorkspace *w[2] = {&ws, &ws2};
    unsigned long long *f[2] = {fr, fr2};
    keybucket_partition(p, n, key32, dot, f[0], *w[0], s, sc);
    t_probe = &probe;
    for (int r = 0; r < reps; r++) {
      KeyBucketClock c = clock;
      c.fold = f[r & 1];
      keybucket_step(p, n, 0, latest, *w[r & 1], sk, sv, dep, c, p, n, key32, dot, f[(r & 1) ^ 1],
                     *w[(r & 1) ^ 1], s, sc);
    }
  }
  (void)hipStreamSynchronize(s);
  t_probe = nullptr;
  for (auto &sl : probe.slots) {
    if (sl.next == 0) continue;
    double tot = 0;
    for (size_t i = 0; i + 1 < sl.next; i += 2) {
      float ms;
      (void)hipEventElapsedTime(&ms, sl.ev[i], sl.ev[i + 1]);
      tot += ms;
    }
    printf("%s: avg %.2f us over %zu launches\n", sl.name.c_str(), tot / (sl.next / 2) * 1e3,
           sl.next / 2);
  }
  std::vector<unsigned long long> h0(p.tiles * 3), h1(B * 3);
  (void)hipMemcpy(h0.data(), st0, h0.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(h1.data(), st1, h1.size() * 8, hipMemcpyDeviceToHost);
  std::vector<uint32_t> wg_of(B);  // bucket -> workgroup index (phase rows)
  for (uint32_t i = 0; i < B; i++) wg_of[i] = i;
  if (sc && sched.valid) {
    std::vector<uint32_t> pm(B);
    (void)hipMemcpy(pm.data(), sched.perm.get(), B * 4, hipMemcpyDeviceToHost);
    for (uint32_t i = 0; i < B; i++) wg_of[pm[i]] = i;
  }
  // fused step grid: the B order workgroups (by schedule rank), then the tiles
  std::vector<uint32_t> prow(p.tiles);
  for (uint32_t t = 0; t < p.tiles; t++) prow[t] = step ? t + B : t;
  report("kb_partition", h0, p.tiles);
  report("kb_order", h1, B);
  if (step) {
    // one timeline: start/end of both roles relative to the earliest start
    unsigned long long t0 = ~0ull;
    for (size_t i = 0; i < p.tiles; i++) t0 = std::min(t0, h0[3 * i]);
    for (size_t i = 0; i < B; i++) t0 = std::min(t0, h1[3 * i]);
    auto span = [&](const std::vector<unsigned long long> &h, size_t nwg, const char *nm) {
      double s0 = 1e9, s1 = 0, e0 = 1e9, e1 = 0;
      for (size_t i = 0; i < nwg; i++) {
        const double a = double(h[3 * i] - t0) * 0.01, e = double(h[3 * i + 1] - t0) * 0.01;
        s0 = std::min(s0, a), s1 = std::max(s1, a), e0 = std::min(e0, e), e1 = std::max(e1, e);
      }
      printf("  step %s: starts %.2f..%.2f ends %.2f..%.2f us\n", nm, s0, s1, e0, e1);
    };
    span(h0, p.tiles, "partition");
    span(h1, B, "order");
  }
  {
    std::vector<unsigned long long> q0((p.tiles + B) * 8), q1((p.tiles + B) * 8);
    (void)hipMemcpy(q0.data(), ph0, q0.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(q1.data(), ph1, q1.size() * 8, hipMemcpyDeviceToHost);
    // median phase durations (us): phase i ends at stamp i; phase 0 starts at WG start
    auto med = [](std::vector<double> v) {
      std::sort(v.begin(), v.end());
      return v.empty() ? 0.0 : v[v.size() / 2];
    };
    const char *n0[] = {"loads", "match+rank", "scan+toff", "lds scatter", "store+clock"};
    printf("kb_partition phases (median us):");
    for (int ph = 0; ph <= 4; ph++) {
      std::vector<double> v;
      for (size_t i = 0; i < p.tiles; i++) {
        unsigned long long a = ph == 0 ? h0[3 * i] : q0[8 * prow[i] + ph - 1];
        unsigned long long e = ph == 4 ? h0[3 * i + 1] : q0[8 * prow[i] + ph];
        v.push_back(double(e - a) * 0.01);
      }
      printf(" %s %.2f", n0[ph], med(v));
    }
    printf("\n");
    const char *n1[] = {"toff+scan", "gather", "sort", "out+latest", "tails"};
    printf("kb_order single-chunk phases (median us):");
    for (int ph = 0; ph <= 4; ph++) {
      std::vector<double> v;
      for (size_t i = 0; i < B; i++) {
        if (h1[3 * i + 2] == 0 || h1[3 * i + 2] > 8192) continue;
        unsigned long long a = ph == 0 ? h1[3 * i] : q1[8 * wg_of[i] + ph - 1];
        unsigned long long e = ph == 4 ? h1[3 * i + 1] : q1[8 * wg_of[i] + ph];
        v.push_back(double(e - a) * 0.01);
      }
      printf(" %s %.2f", n1[ph], med(v));
    }
    printf("\n  sort pass 1 (median us):");
    const char *n2[] = {"zero", "ranks", "scan", "scatter+pass2"};
    const int from[] = {1, 4, 5, 6}, to[] = {4, 5, 6, 2};
    for (int k = 0; k < 4; k++) {
      std::vector<double> v;
      for (size_t i = 0; i < B; i++) {
        if (h1[3 * i + 2] == 0 || h1[3 * i + 2] > 8192) continue;
        v.push_back(double(q1[8 * wg_of[i] + to[k]] - q1[8 * wg_of[i] + from[k]]) * 0.01);
      }
      printf(" %s %.2f", n2[k], med(v));
    }
    printf("\n");
  }
  std::vector<std::pair<unsigned long long, size_t>> big;
  for (size_t i = 0; i < B; i++) big.push_back({h1[3 * i + 2], i});
  std::sort(big.rbegin(), big.rend());
  std::vector<unsigned long long> q1((p.tiles + B) * 8);
  (void)hipMemcpy(q1.data(), ph1, q1.size() * 8, hipMemcpyDeviceToHost);
  for (int i = 0; i < 6; i++) {
    const size_t bk = big[i].second;
    printf("  bucket %zu: %llu cmds, %.2f us", bk, big[i].first,
           double(h1[3 * bk + 1] - h1[3 * bk]) * 0.01);
    if (big[i].first <= 8192) {
      const unsigned long long *q = &q1[8 * wg_of[bk]];
      printf("  [toff %.2f gather %.2f sort %.2f (ranks1 %.2f) out %.2f tails %.2f]",
             double(q[0] - h1[3 * bk]) * 0.01, double(q[1] - q[0]) * 0.01,
             double(q[2] - q[1]) * 0.01, double(q[5] - q[4]) * 0.01, double(q[3] - q[2]) * 0.01,
             double(h1[3 * bk + 1] - q[3]) * 0.01);
    }
    printf("\n");
  }
  return 0;
}
