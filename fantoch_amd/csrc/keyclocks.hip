// keyclocks.hip -- Caesar's KeyClocks on the device (fh_keyclocks_*).
//
// SequentialKeyClocks (fantoch_ps/src/protocol/common/pred/clocks/keys/
// sequential.rs:14-152): per key, the commands added with their tentative
// timestamp (CommandsPerKey = HashMap<Clock, Dot>, :11-12); add / remove
// (:43-75) insert and drop (key, clock) -> dot entries, predecessors
// (:77-119) reports, over the command's keys, every dot with a lower clock
// (and, optionally, every dot with a higher one).  Clocks are packed
// (seq << 8) | process_id: the integer order is Clock's derived Ord
// (clocks/mod.rs:15-30).
//
// Device layout: the entries sorted by a 64-bit composite (key << cb) |
// clock (cb = bits of the largest clock seen), with their dots alongside.
//   add          new entries appended, one radix sort of the composites,
//                adjacent equal composites = a timestamp added twice
//   remove       removal composites sorted; each entry binary-searches them;
//                a removal that matches no entry = never added; compaction
//   predecessors per query, each key's segment is clock-sorted: the prefix
//                below the query clock (predecessors) and the suffix above it
//                (higher); one thread k-way merges the query's segments by
//                (clock, dot), dropping repeats of a (clock, dot) pair (the
//                same dot on another key of a multi-key command); two
//                different dots with one clock on different keys are both
//                reported, as the reference's HashSet<Dot> keeps them; two
//                passes (count, scan, write).  Output order: ascending
//                (clock, dot).  At most kMaxKeys keys per command
//                (FH_ENOTIMPL beyond).
#include <algorithm>
#include <vector>

#include "fh_common.h"
#include "scan.h"
#include "sort.h"

namespace fh {
namespace {

constexpr unsigned B = 256;
constexpr int kMaxKeys = 8;

__device__ __forceinline__ uint32_t lower_u64(const uint64_t *__restrict__ a, uint32_t n,
                                              uint64_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (a[m] < x)
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}

__global__ void k_kc_new(uint32_t n, const uint32_t *__restrict__ koff,
                         const uint32_t *__restrict__ key, const uint64_t *__restrict__ clock,
                         const uint64_t *__restrict__ dot, int cb, uint32_t base,
                         uint64_t *__restrict__ comp, uint64_t *__restrict__ edot) {
  for (uint32_t i = blockIdx.x * B + threadIdx.x; i < n; i += gridDim.x * B)
    for (uint32_t e = koff[i]; e < koff[i + 1]; e++) {
      comp[base + e] = (uint64_t(key[e]) << cb) | clock[i];
      if (edot) edot[base + e] = dot[i];
    }
}

// existing entries re-keyed when the clock width grows
__global__ void k_kc_rekey(uint32_t E, uint64_t *__restrict__ comp, int cb_old, int cb) {
  for (uint32_t i = blockIdx.x * B + threadIdx.x; i < E; i += gridDim.x * B) {
    const uint64_t c = comp[i];
    const uint64_t key = c >> cb_old, clk = c & ((uint64_t(1) << cb_old) - 1);
    comp[i] = (key << cb) | clk;
  }
}

__global__ void k_kc_gather(uint32_t E, const uint32_t *__restrict__ perm,
                            const uint64_t *__restrict__ dot_in, uint64_t *__restrict__ dot_out,
                            const uint64_t *__restrict__ comp, uint32_t *__restrict__ dup) {
  for (uint32_t i = blockIdx.x * B + threadIdx.x; i < E; i += gridDim.x * B) {
    dot_out[i] = dot_in[perm[i]];
    if (i > 0 && comp[i] == comp[i - 1]) atomicOr(dup, 1u);
  }
}

__global__ void k_kc_mark(uint32_t E, const uint64_t *__restrict__ comp, uint32_t R,
                          const uint64_t *__restrict__ rem, uint32_t *__restrict__ keep,
                          uint32_t *__restrict__ removed) {
  for (uint32_t i = blockIdx.x * B + threadIdx.x; i < E; i += gridDim.x * B) {
    const uint32_t p = lower_u64(rem, R, comp[i]);
    const bool gone = p < R && rem[p] == comp[i];
    keep[i] = gone ? 0u : 1u;
    if (gone) atomicAdd(removed, 1u);
  }
}

__global__ void k_kc_compact(uint32_t E, const uint32_t *__restrict__ keep,
                             const uint32_t *__restrict__ pos, const uint64_t *__restrict__ comp,
                             const uint64_t *__restrict__ dot, uint64_t *__restrict__ comp2,
                             uint64_t *__restrict__ dot2) {
  for (uint32_t i = blockIdx.x * B + threadIdx.x; i < E; i += gridDim.x * B)
    if (keep[i]) {
      comp2[pos[i]] = comp[i];
      dot2[pos[i]] = dot[i];
    }
}

// adjacent-duplicate count of a sorted array (distinct removal records)
__global__ void k_kc_distinct(uint32_t R, const uint64_t *__restrict__ a, uint32_t *__restrict__ d) {
  for (uint32_t i = blockIdx.x * B + threadIdx.x; i < R; i += gridDim.x * B)
    if (i == 0 || a[i] != a[i - 1]) atomicAdd(d, 1u);
}

// Per query: the clock-sorted segments [lo, hi) of its keys below (side 0)
// or above (side 1) its clock, merged by clock with repeats dropped.
// write == false: count only.  err |= 1: a different dot with the same
// timestamp (sequential.rs:108-112 panics).
__global__ void k_kc_query(uint32_t n, const uint32_t *__restrict__ koff,
                           const uint32_t *__restrict__ key, const uint64_t *__restrict__ clock,
                           const uint64_t *__restrict__ qdot, const uint64_t *__restrict__ comp,
                           const uint64_t *__restrict__ edot, uint32_t E, int cb, int side,
                           const uint32_t *__restrict__ out_off, uint32_t *__restrict__ cnt,
                           uint64_t *__restrict__ out, uint32_t *__restrict__ err) {
  for (uint32_t i = blockIdx.x * B + threadIdx.x; i < n; i += gridDim.x * B) {
    const uint32_t ka = koff[i], kn = min(koff[i + 1] - ka, uint32_t(kMaxKeys));
    uint32_t cur[kMaxKeys], end[kMaxKeys];
    const uint64_t mask = (uint64_t(1) << cb) - 1;
    for (uint32_t s = 0; s < kn; s++) {
      const uint64_t kb = uint64_t(key[ka + s]) << cb;
      const uint32_t lo = lower_u64(comp, E, kb);
      const uint32_t hi = lower_u64(comp, E, kb + (uint64_t(1) << cb));
      const uint32_t p = lower_u64(comp, E, kb | clock[i]);
      const bool eq = p < hi && comp[p] == (kb | clock[i]);
      if (eq && edot[p] != qdot[i]) atomicOr(err, 1u);
      if (side == 0) {
        cur[s] = lo;
        end[s] = p;
      } else {
        cur[s] = eq ? p + 1 : p;
        end[s] = hi;
      }
    }
    uint32_t c = 0;
    const uint32_t o = out_off ? out_off[i] : 0u;
    uint64_t last = ~0ull, last_dot = 0;
    for (;;) {
      int best = -1;
      uint64_t bc = ~0ull, bd = ~0ull;
      for (uint32_t s = 0; s < kn; s++)
        if (cur[s] < end[s]) {
          const uint64_t x = comp[cur[s]] & mask, d = edot[cur[s]];
          if (x < bc || (x == bc && d < bd)) {
            bc = x;
            bd = d;
            best = int(s);
          }
        }
      if (best < 0) break;
      if (bc != last || bd != last_dot) {  // (the reference's predecessors HashSet<Dot>)
        if (out) out[o + c] = bd;
        c++;
        last = bc;
        last_dot = bd;
      }
      cur[best]++;
    }
    if (cnt) cnt[i] = c;
  }
}

}  // namespace

struct KeyClocksDevice {
  uint32_t process_id;
  fh_config cfg;
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t seq = 0;  // SequentialKeyClocks::seq (sequential.rs:18)
  int kb = 1, cb = 1;
  uint32_t E = 0;
  DBuf<uint64_t> comp, edot, comp2, edot2, tmpk, tmpk2;
  DBuf<uint32_t> perm, perm2, keep, pos, scal, qoff, qcnt, qkey, qkoff;
  DBuf<uint64_t> qclock, qdot;
  SortWorkspace sort_ws;
  ScanWorkspace scan_ws;

  KeyClocksDevice(uint32_t pid, uint64_t shard, const fh_config &c) : process_id(pid), cfg(c) {
    FH_CHECK(pid >= 1 && pid <= 255, FH_EINVAL, "process id must be in [1, 255]");
    FH_CHECK(c.key_space >= 1 && c.key_space <= (uint64_t(1) << 31), FH_EINVAL,
             "key_space must be in [1, 2^31]");
    kb = bits_for(c.key_space);
    device = pick_device(&c, shard);
    FH_HIP(hipSetDevice(device));
    FH_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    scal.ensure(8);
  }
  ~KeyClocksDevice() {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
  }

  // the batch's keys and clocks to the device; widens the composite's clock
  // field (re-keying the stored entries) when a larger clock arrives
  size_t upload(size_t n, const uint32_t *key_off, const uint64_t *key_id, const uint64_t *clock,
                const uint64_t *dot) {
    FH_CHECK(n == 0 || (key_off && key_id && clock), FH_EINVAL, "null argument");
    const size_t m = n ? key_off[n] : 0;
    FH_CHECK(m < (size_t(1) << 30), FH_EINVAL, "batch too large");
    uint64_t mx = 0;
    for (size_t i = 0; i < n; i++) mx = std::max(mx, clock[i]);
    std::vector<uint32_t> k32(m + 1);
    for (size_t i = 0; i < n; i++) {
      FH_CHECK(key_off[i + 1] >= key_off[i], FH_EINVAL, "keyclocks: key offsets decrease");
      FH_CHECK(key_off[i + 1] - key_off[i] <= uint32_t(kMaxKeys), FH_ENOTIMPL,
               "keyclocks: more than 8 keys in a command (the device merge holds 8 segments)");
      for (uint32_t e = key_off[i]; e < key_off[i + 1]; e++) {
        FH_CHECK(key_id[e] < cfg.key_space, FH_EINVAL, "key id >= key_space");
        k32[e] = uint32_t(key_id[e]);
      }
    }
    const int need = bits_for(mx + 1);
    if (need > cb) {
      FH_CHECK(kb + need <= 64, FH_ENOTIMPL, "keyclocks: key bits + clock bits exceed 64");
      if (E) k_kc_rekey<<<grid_for(E, B), B, 0, stream>>>(E, comp.get(), cb, need);
      cb = need;
    }
    FH_HIP(hipMemcpyAsync(qkoff.ensure(n + 2), key_off, (n + 1) * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    FH_HIP(hipMemcpyAsync(qkey.ensure(m + 1), k32.data(), m * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    FH_HIP(hipMemcpyAsync(qclock.ensure(n + 1), clock, n * sizeof(uint64_t),
                          hipMemcpyHostToDevice, stream));
    if (dot)
      FH_HIP(hipMemcpyAsync(qdot.ensure(n + 1), dot, n * sizeof(uint64_t), hipMemcpyHostToDevice,
                            stream));
    FH_HIP(hipStreamSynchronize(stream));
    return m;
  }

  uint32_t read(int i) {
    uint32_t v = 0;
    FH_HIP(hipMemcpyAsync(&v, scal.get() + i, sizeof(v), hipMemcpyDeviceToHost, stream));
    FH_HIP(hipStreamSynchronize(stream));
    return v;
  }

  // KeyClocks::add (sequential.rs:43-56) for every command of the batch
  void add(size_t n, const uint64_t *dot, const uint32_t *key_off, const uint64_t *key_id,
           const uint64_t *clock) {
    FH_CHECK(n == 0 || dot, FH_EINVAL, "null argument");
    FH_HIP(hipSetDevice(device));
    const size_t m = upload(n, key_off, key_id, clock, dot);
    if (m == 0) return;
    const uint32_t E2 = uint32_t(E + m);
    FH_CHECK(E2 < (uint32_t(1) << 30), FH_EINVAL, "keyclocks: too many entries");
    uint64_t *c = comp2.ensure(E2 + 1), *d = edot2.ensure(E2 + 1);
    if (E) {
      FH_HIP(hipMemcpyAsync(c, comp.get(), E * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream));
      FH_HIP(hipMemcpyAsync(d, edot.get(), E * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream));
    }
    k_kc_new<<<grid_for(n, B), B, 0, stream>>>(uint32_t(n), qkoff.get(), qkey.get(), qclock.get(),
                                                qdot.get(), cb, E, c, d);
    uint64_t *ks = nullptr;
    uint32_t *vs = nullptr;
    sort_pairs<uint64_t, uint32_t>(c, nullptr, tmpk.ensure(E2 + 1), perm.ensure(E2 + 1),
                         tmpk2.ensure(E2 + 1), perm2.ensure(E2 + 1), E2, kb + cb, sort_ws, stream,
                         &ks, &vs);
    uint64_t *nc = comp.ensure(E2 + 1), *nd = edot.ensure(E2 + 1);
    FH_HIP(hipMemsetAsync(scal.get(), 0, sizeof(uint32_t), stream));
    FH_HIP(hipMemcpyAsync(nc, ks, E2 * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream));
    k_kc_gather<<<grid_for(E2, B), B, 0, stream>>>(E2, vs, d, nd, nc, scal.get());
    // sequential.rs:49-54: a timestamp added twice on a key panics
    if (read(0)) {
      // state unchanged: drop the batch (the copies above went to scratch
      // only for the entries; rebuild the previous order from comp2/edot2)
      FH_HIP(hipMemcpyAsync(nc, c, E * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream));
      FH_HIP(hipMemcpyAsync(nd, d, E * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream));
      FH_HIP(hipStreamSynchronize(stream));
      throw Error(FH_EINVARIANT, "can't add a timestamp belonging to a command already added");
    }
    E = E2;
  }

  // KeyClocks::remove (sequential.rs:58-75)
  void remove(size_t n, const uint32_t *key_off, const uint64_t *key_id, const uint64_t *clock) {
    FH_HIP(hipSetDevice(device));
    const size_t m = upload(n, key_off, key_id, clock, nullptr);
    if (m == 0) return;
    uint64_t *r = comp2.ensure(m + 1);
    k_kc_new<<<grid_for(n, B), B, 0, stream>>>(uint32_t(n), qkoff.get(), qkey.get(), qclock.get(),
                                                nullptr, cb, 0, r, nullptr);
    uint64_t *rs = nullptr;
    uint32_t *vs = nullptr;
    sort_pairs<uint64_t, uint32_t>(r, nullptr, tmpk.ensure(m + 1), perm.ensure(m + 1), tmpk2.ensure(m + 1),
                         perm2.ensure(m + 1), m, kb + cb, sort_ws, stream, &rs, &vs);
    FH_HIP(hipMemsetAsync(scal.get(), 0, 2 * sizeof(uint32_t), stream));
    k_kc_distinct<<<grid_for(m, B), B, 0, stream>>>(uint32_t(m), rs, scal.get() + 1);
    uint32_t *kp = keep.ensure(E + 1), *ps = pos.ensure(E + 2);
    if (E) k_kc_mark<<<grid_for(E, B), B, 0, stream>>>(E, comp.get(), uint32_t(m), rs, kp, scal.get());
    const uint32_t removed = E ? read(0) : 0, distinct = read(1);
    // every removal names an entry, once (sequential.rs:68-73 panics)
    FH_CHECK(removed == distinct && distinct == m, FH_EINVARIANT,
             "can't remove a timestamp belonging to a command never added");
    exclusive_scan_u32(kp, ps, E, scan_ws, stream);
    uint64_t *c2 = comp2.ensure(E + 1), *d2 = edot2.ensure(E + 1);
    k_kc_compact<<<grid_for(E, B), B, 0, stream>>>(E, kp, ps, comp.get(), edot.get(), c2, d2);
    comp.swap(comp2);
    edot.swap(edot2);
    E -= removed;
    FH_HIP(hipStreamSynchronize(stream));
  }

  // KeyClocks::predecessors (sequential.rs:77-119) for a batch of queries
  void predecessors(size_t n, const uint64_t *dot, const uint32_t *key_off,
                    const uint64_t *key_id, const uint64_t *clock, uint32_t *p_off,
                    uint64_t *p_dot, size_t p_cap, size_t *p_len, uint32_t *h_off,
                    uint64_t *h_dot, size_t h_cap, size_t *h_len) {
    FH_CHECK(n == 0 || dot, FH_EINVAL, "null argument");
    FH_HIP(hipSetDevice(device));
    upload(n, key_off, key_id, clock, dot);
    FH_HIP(hipMemsetAsync(scal.get(), 0, sizeof(uint32_t), stream));
    bool ecap = false;
    for (int side = 0; side < 2; side++) {
      uint32_t *off_h = side ? h_off : p_off;
      uint64_t *dot_h = side ? h_dot : p_dot;
      size_t *len = side ? h_len : p_len;
      const size_t cap = side ? h_cap : p_cap;
      if (side == 1 && !h_len && !h_off && !h_dot) break;  // `higher` = None
      uint32_t *cnt = qcnt.ensure(n + 1), *off = qoff.ensure(n + 2);
      k_kc_query<<<grid_for(n, B), B, 0, stream>>>(uint32_t(n), qkoff.get(), qkey.get(),
                                                    qclock.get(), qdot.get(), comp.get(),
                                                    edot.get(), E, cb, side, nullptr, cnt,
                                                    nullptr, scal.get());
      exclusive_scan_u32(cnt, off, n, scan_ws, stream);
      uint32_t total = 0;
      FH_HIP(hipMemcpyAsync(&total, off + n, sizeof(total), hipMemcpyDeviceToHost, stream));
      FH_HIP(hipStreamSynchronize(stream));
      FH_CHECK(read(0) == 0, FH_EINVARIANT, "found different command with the same timestamp");
      if (len) *len = total;
      if (off_h)
        FH_HIP(hipMemcpyAsync(off_h, off, (n + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                              stream));
      if (!dot_h) continue;
      if (cap < total) {  // sizes reported, nothing written
        ecap = true;
        continue;
      }
      uint64_t *o = tmpk.ensure(total + 1);
      k_kc_query<<<grid_for(n, B), B, 0, stream>>>(uint32_t(n), qkoff.get(), qkey.get(),
                                                    qclock.get(), qdot.get(), comp.get(),
                                                    edot.get(), E, cb, side, off, nullptr, o,
                                                    scal.get());
      FH_HIP(hipMemcpyAsync(dot_h, o, total * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
      FH_HIP(hipStreamSynchronize(stream));
    }
    FH_HIP(hipStreamSynchronize(stream));
    FH_CHECK(!ecap, FH_ECAP, "predecessors output capacity too small");
  }
};

}  // namespace fh

struct fh_keyclocks {
  fh::KeyClocksDevice dev;
  fh_keyclocks(uint32_t p, uint64_t s, const fh_config &c) : dev(p, s, c) {}
};

extern "C" {

fh_status fh_keyclocks_create(uint32_t process_id, uint64_t shard_id, const fh_config *cfg,
                              fh_keyclocks **out) {
  FH_API_BEGIN
  FH_CHECK(cfg && out, FH_EINVAL, "null argument");
  *out = new fh_keyclocks(process_id, shard_id, *cfg);
  FH_API_END
}

fh_status fh_keyclocks_destroy(fh_keyclocks *h) {
  FH_API_BEGIN
  delete h;
  FH_API_END
}

fh_status fh_keyclocks_clock_next(fh_keyclocks *h, uint64_t *clock) {
  FH_API_BEGIN
  FH_CHECK(h && clock, FH_EINVAL, "null argument");
  h->dev.seq++;  // sequential.rs:33-37
  FH_CHECK(h->dev.seq < (uint64_t(1) << 56), FH_EINVARIANT, "clock sequence overflow");
  *clock = (h->dev.seq << 8) | h->dev.process_id;
  FH_API_END
}

fh_status fh_keyclocks_clock_join(fh_keyclocks *h, uint64_t clock) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.seq = std::max(h->dev.seq, clock >> 8);  // sequential.rs:39-42
  FH_API_END
}

fh_status fh_keyclocks_add(fh_keyclocks *h, size_t n, const uint64_t *dot, const uint32_t *key_off,
                           const uint64_t *key_id, const uint64_t *clock) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.add(n, dot, key_off, key_id, clock);
  FH_API_END
}

fh_status fh_keyclocks_remove(fh_keyclocks *h, size_t n, const uint32_t *key_off,
                              const uint64_t *key_id, const uint64_t *clock) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.remove(n, key_off, key_id, clock);
  FH_API_END
}

fh_status fh_keyclocks_predecessors(fh_keyclocks *h, size_t n, const uint64_t *dot,
                                    const uint32_t *key_off, const uint64_t *key_id,
                                    const uint64_t *clock, uint32_t *pred_off, uint64_t *pred_dot,
                                    size_t pred_cap, size_t *pred_len, uint32_t *higher_off,
                                    uint64_t *higher_dot, size_t higher_cap, size_t *higher_len) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.predecessors(n, dot, key_off, key_id, clock, pred_off, pred_dot, pred_cap, pred_len,
                      higher_off, higher_dot, higher_cap, higher_len);
  FH_API_END
}

fh_status fh_keyclocks_len(fh_keyclocks *h, size_t *entries) {
  FH_API_BEGIN
  FH_CHECK(h && entries, FH_EINVAL, "null argument");
  *entries = h->dev.E;
  FH_API_END
}

}  // extern "C"
