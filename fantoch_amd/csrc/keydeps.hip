// keydeps.hip -- batched KeyDeps (conflict detection) on gfx950.
//
// Restates SequentialKeyDeps::do_add_cmd
// (fantoch_ps/src/protocol/common/graph/deps/keys/sequential.rs:72-104) for a
// whole batch at once: the i-th command's deps are the previous command (in
// arrival order) on each of its keys -- or the persistent latest[key] for the
// first occurrence in the batch -- plus the latest noop and `past`.
//
//   1. k_build_elems  one element per (command, key): u32 key id, owner cmd
//   2. sort_pairs     stable radix sort of (key, element) -> key segments in
//                     arrival order
//   3. k_prev         element dep = previous element of its key segment, or
//                     latest[key] at the segment head; marks segment tails
//   4. k_cmd          per command: union of its element deps + noop + past,
//                     sorted, deduplicated; tails update latest[key]
//   5. scan + k_compact  CSR output
// Noops (do_add_noop :106-123) split the batch into command segments.
#include <algorithm>
#include <vector>

#include "keydeps.h"

namespace fh {
namespace {

__global__ void k_build_elems(const uint32_t *__restrict__ key_off,
                              const uint64_t *__restrict__ key64, uint32_t cmd_first,
                              uint32_t ncmd, uint64_t key_space, uint32_t *__restrict__ key32,
                              uint32_t *__restrict__ cmd_of, uint32_t *err) {
  const uint32_t ebase = key_off[cmd_first];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ncmd;
       i += gridDim.x * blockDim.x) {
    const uint32_t c = cmd_first + i;
    for (uint32_t e = key_off[c]; e < key_off[c + 1]; e++) {
      uint64_t k = key64[e];
      if (k >= key_space) {
        atomicOr(err, 1u);
        k = 0;
      }
      key32[e - ebase] = uint32_t(k);
      cmd_of[e - ebase] = c;
    }
  }
}

__global__ void k_prev(const uint32_t *__restrict__ ks, const uint32_t *__restrict__ vs,
                       uint32_t m, const uint32_t *__restrict__ cmd_of,
                       const uint64_t *__restrict__ dot, const uint64_t *__restrict__ latest,
                       uint64_t *__restrict__ elem_dep, uint8_t *__restrict__ elem_tail) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m;
       j += gridDim.x * blockDim.x) {
    const uint32_t k = ks[j];
    const uint32_t e = vs[j];
    const bool head = j == 0 || ks[j - 1] != k;
    const bool tail = j + 1 == m || ks[j + 1] != k;
    const uint64_t dep = head ? latest[k] : dot[cmd_of[vs[j - 1]]];
    elem_dep[e] = dep;
    elem_tail[e] = tail ? 1 : 0;
  }
}

__device__ __forceinline__ uint32_t sort_unique_dev(uint64_t *a, uint32_t n) {
  for (uint32_t i = 1; i < n; i++) {
    const uint64_t x = a[i];
    uint32_t j = i;
    while (j > 0 && a[j - 1] > x) {
      a[j] = a[j - 1];
      j--;
    }
    a[j] = x;
  }
  uint32_t w = n ? 1 : 0;
  for (uint32_t i = 1; i < n; i++)
    if (a[i] != a[w - 1]) a[w++] = a[i];
  return w;
}

// scratch slot of command i: dm deps per key (1 sequential, 2 read/write),
// one noop, its past
__device__ __forceinline__ uint32_t tmp_base(const uint32_t *key_off, const uint32_t *past_off,
                                             uint32_t cmd_first, uint32_t i, uint32_t dm) {
  const uint32_t c = cmd_first + i;
  uint32_t b = (key_off[c] - key_off[cmd_first]) * dm + i;
  if (past_off) b += past_off[c] - past_off[cmd_first];
  return b;
}

__global__ void k_cmd(uint32_t cmd_first, uint32_t ncmd, const uint32_t *__restrict__ key_off,
                      const uint32_t *__restrict__ key32, const uint64_t *__restrict__ dot,
                      const uint64_t *__restrict__ elem_dep,
                      const uint64_t *__restrict__ elem_dep2,
                      const uint8_t *__restrict__ elem_tail, uint64_t noop_latest,
                      const uint32_t *__restrict__ past_off, const uint64_t *__restrict__ past,
                      uint64_t *__restrict__ latest, uint64_t *__restrict__ tmp,
                      uint32_t *__restrict__ cnt) {
  const uint32_t ebase = key_off[cmd_first];
  const uint32_t dm = elem_dep2 ? 2u : 1u;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ncmd;
       i += gridDim.x * blockDim.x) {
    const uint32_t c = cmd_first + i;
    uint64_t *t = tmp + tmp_base(key_off, past_off, cmd_first, i, dm);
    uint32_t n = 0;
    if (past_off) /* sequential.rs:31-34: start from past */
      for (uint32_t p = past_off[c]; p < past_off[c + 1]; p++) t[n++] = past[p];
    const uint64_t self = dot[c];
    for (uint32_t e = key_off[c] - ebase; e < key_off[c + 1] - ebase; e++) {
      const uint64_t d = elem_dep[e];
      if (d) t[n++] = d; /* :84-87 */
      if (elem_dep2 && elem_dep2[e]) t[n++] = elem_dep2[e]; /* locked.rs:111-113 */
      if (elem_tail[e]) latest[key32[e]] = self; /* :88, :90-95 */
    }
    if (noop_latest) t[n++] = noop_latest; /* :100 */
    cnt[i] = sort_unique_dev(t, n);
  }
}

// Read/write rules (LockedKeyDeps::do_add_cmd, locked.rs:94-118), per key in
// arrival order: a read depends on the latest write and becomes the latest
// read; a write depends on the latest read and the latest write and becomes
// the latest write (the latest read stays).  Over a key-sorted batch: marks
// (position + 1) of segment heads, writes and reads, whose exclusive prefix
// maxima give each element's previous write / read inside its segment.
__global__ void k_rw_marks(const uint32_t *__restrict__ ks, const uint32_t *__restrict__ vs,
                           uint32_t m, const uint32_t *__restrict__ cmd_of,
                           const uint8_t *__restrict__ ro, uint32_t *__restrict__ mh,
                           uint32_t *__restrict__ mw, uint32_t *__restrict__ mr) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m;
       j += gridDim.x * blockDim.x) {
    const bool read = ro[cmd_of[vs[j]]] != 0;
    mh[j] = (j == 0 || ks[j - 1] != ks[j]) ? j + 1 : 0u;
    mw[j] = read ? 0u : j + 1;
    mr[j] = read ? j + 1 : 0u;
  }
}

__global__ void k_prev_rw(const uint32_t *__restrict__ ks, const uint32_t *__restrict__ vs,
                          uint32_t m, const uint32_t *__restrict__ cmd_of,
                          const uint8_t *__restrict__ ro, const uint64_t *__restrict__ dot,
                          const uint64_t *__restrict__ latest_w,
                          const uint64_t *__restrict__ latest_r, const uint32_t *__restrict__ mh,
                          const uint32_t *__restrict__ sh, const uint32_t *__restrict__ sw,
                          const uint32_t *__restrict__ sr, uint64_t *__restrict__ elem_dep,
                          uint64_t *__restrict__ elem_dep2) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m;
       j += gridDim.x * blockDim.x) {
    const uint32_t k = ks[j], e = vs[j];
    const uint32_t seg = max(sh[j], mh[j]);  // segment head position + 1
    const uint64_t pw = sw[j] >= seg ? dot[cmd_of[vs[sw[j] - 1]]] : latest_w[k];
    const uint64_t pr = sr[j] >= seg ? dot[cmd_of[vs[sr[j] - 1]]] : latest_r[k];
    elem_dep[e] = pw;
    elem_dep2[e] = ro[cmd_of[e]] ? 0ull : pr;
  }
}

// segment tails: the last write / read of the key in the batch becomes its
// latest write / read (after every head has read the tables: own launch)
__global__ void k_tails_rw(const uint32_t *__restrict__ ks, const uint32_t *__restrict__ vs,
                           uint32_t m, const uint32_t *__restrict__ cmd_of,
                           const uint64_t *__restrict__ dot, const uint32_t *__restrict__ mh,
                           const uint32_t *__restrict__ sh, const uint32_t *__restrict__ mw,
                           const uint32_t *__restrict__ sw, const uint32_t *__restrict__ mr,
                           const uint32_t *__restrict__ sr, uint64_t *__restrict__ latest_w,
                           uint64_t *__restrict__ latest_r) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m;
       j += gridDim.x * blockDim.x) {
    if (j + 1 < m && ks[j + 1] == ks[j]) continue;
    const uint32_t k = ks[j];
    const uint32_t seg = max(sh[j], mh[j]);
    const uint32_t lw = max(sw[j], mw[j]), lr = max(sr[j], mr[j]);
    if (lw >= seg) latest_w[k] = dot[cmd_of[vs[lw - 1]]];
    if (lr >= seg) latest_r[k] = dot[cmd_of[vs[lr - 1]]];
  }
}

__global__ void k_compact(uint32_t cmd_first, uint32_t ncmd, const uint32_t *__restrict__ key_off,
                          const uint32_t *__restrict__ past_off, uint32_t dm,
                          const uint64_t *__restrict__ tmp, const uint32_t *__restrict__ off,
                          uint64_t *__restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ncmd;
       i += gridDim.x * blockDim.x) {
    const uint64_t *t = tmp + tmp_base(key_off, past_off, cmd_first, i, dm);
    const uint32_t o = off[i], c = off[i + 1] - off[i];
    for (uint32_t j = 0; j < c; j++) out[o + j] = t[j];
  }
}

__global__ void k_nonzero_flags(const uint64_t *__restrict__ latest, uint32_t k,
                                uint32_t *__restrict__ flags) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x)
    flags[i] = latest[i] != 0;
}

__global__ void k_nonzero_gather(const uint64_t *__restrict__ latest, uint32_t k,
                                 const uint32_t *__restrict__ pos, uint64_t *__restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x)
    if (latest[i]) out[pos[i]] = latest[i];
}

__global__ void k_gather_keys(const uint64_t *__restrict__ latest, const uint64_t *__restrict__ keys,
                              uint32_t n, uint64_t key_space, uint64_t *__restrict__ out,
                              uint32_t *err) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    if (k >= key_space) {
      atomicOr(err, 1u);
      out[i] = 0;
    } else {
      out[i] = latest[k];
    }
  }
}

}  // namespace

KeyDepsDevice::KeyDepsDevice(uint64_t shard_id_, const fh_config &cfg) : shard_id(shard_id_) {
  FH_CHECK(cfg.key_space >= 1 && cfg.key_space <= (uint64_t(1) << 31), FH_EINVAL,
           "key_space must be in [1, 2^31]");
  key_space = cfg.key_space;
  key_bits = bits_for(key_space);
  device = pick_device(&cfg, shard_id);
  FH_HIP(hipSetDevice(device));
  FH_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  latest.ensure(key_space);
  FH_HIP(hipMemsetAsync(latest.get(), 0, key_space * sizeof(uint64_t), stream));
  err.ensure(4);
  FH_HIP(hipMemsetAsync(err.get(), 0, 4 * sizeof(uint32_t), stream));
  FH_HIP(hipStreamSynchronize(stream));
}

KeyDepsDevice::~KeyDepsDevice() {
  if (stream) {
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    (void)hipStreamDestroy(stream);
  }
}

void KeyDepsDevice::check_err(const char *what) {
  uint32_t e = 0;
  FH_HIP(hipMemcpyAsync(&e, err.get(), sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
  FH_HIP(hipStreamSynchronize(stream));
  if (e) {
    FH_HIP(hipMemsetAsync(err.get(), 0, sizeof(uint32_t), stream));
    FH_HIP(hipStreamSynchronize(stream));
    throw Error(FH_EINVAL, std::string(what) + ": key id >= key_space");
  }
}

// Runs the command pipeline for commands [a, b) of the staged batch; appends
// their CSR to (host) out.  Returns number of deps written.
void KeyDepsDevice::enable_rw() {
  if (rw) return;
  latest_r.ensure(key_space);
  FH_HIP(hipMemsetAsync(latest_r.get(), 0, key_space * sizeof(uint64_t), stream));
  rw = true;
}

size_t KeyDepsDevice::run_segment(uint32_t a, uint32_t b, bool has_past, bool has_ro,
                                  uint32_t *out_off, uint64_t *out_dep, size_t out_base,
                                  bool dev_out) {
  const uint32_t ncmd = b - a;
  if (ncmd == 0) return 0;
  const uint32_t e0 = h_key_off[a], e1 = h_key_off[b];
  const uint32_t m = e1 - e0;
  const uint32_t p0 = has_past ? h_past_off[a] : 0, p1 = has_past ? h_past_off[b] : 0;
  const uint32_t dm = has_ro ? 2u : 1u;
  const size_t tmp_n = size_t(m) * dm + ncmd + (p1 - p0);
  uint32_t *key32 = d_key32.ensure(m);
  uint32_t *cmd_of = d_cmd_of.ensure(m);
  uint64_t *edep = d_elem_dep.ensure(m);
  uint8_t *etail = d_elem_tail.ensure(m);
  uint64_t *tmp = d_tmp.ensure(tmp_n);
  uint32_t *cnt = d_cnt.ensure(ncmd);
  uint32_t *off = d_off.ensure(ncmd + 1);
  const unsigned B = 256;
  k_build_elems<<<grid_for(ncmd, B), B, 0, stream>>>(d_key_off.get(), d_key64.get(), a, ncmd,
                                                      key_space, key32, cmd_of, err.get());
  uint32_t *ks = nullptr, *vs = nullptr;
  uint32_t *ka = d_sk_a.ensure(m), *kb = d_sk_b.ensure(m);
  uint32_t *va = d_sv_a.ensure(m), *vb = d_sv_b.ensure(m);
  sort_pairs<uint32_t, uint32_t>(key32, nullptr, ka, va, kb, vb, m, key_bits, sort_ws, stream, &ks, &vs);
  uint64_t *edep2 = nullptr;
  if (has_ro) {
    // LockedKeyDeps read/write rules; tails update both tables in their own
    // launch, so k_cmd below writes nothing
    edep2 = d_elem_dep2.ensure(m);
    FH_HIP(hipMemsetAsync(etail, 0, m, stream));
    if (m) {
      uint32_t *mh = d_mh.ensure(m), *mw = d_mw.ensure(m), *mr = d_mr.ensure(m);
      uint32_t *sh = d_sh.ensure(m + 1), *sw = d_sw.ensure(m + 1), *sr = d_sr.ensure(m + 1);
      k_rw_marks<<<grid_for(m, B), B, 0, stream>>>(ks, vs, m, cmd_of, d_ro.get(), mh, mw, mr);
      exclusive_scan_max_u32(mh, sh, m, scan_ws, stream);
      exclusive_scan_max_u32(mw, sw, m, scan_ws, stream);
      exclusive_scan_max_u32(mr, sr, m, scan_ws, stream);
      k_prev_rw<<<grid_for(m, B), B, 0, stream>>>(ks, vs, m, cmd_of, d_ro.get(), d_dot.get(),
                                                  latest.get(), latest_r.get(), mh, sh, sw, sr,
                                                  edep, edep2);
      k_tails_rw<<<grid_for(m, B), B, 0, stream>>>(ks, vs, m, cmd_of, d_dot.get(), mh, sh, mw,
                                                   sw, mr, sr, latest.get(), latest_r.get());
    }
  } else if (m) {
    k_prev<<<grid_for(m, B), B, 0, stream>>>(ks, vs, m, cmd_of, d_dot.get(), latest.get(), edep,
                                             etail);
  }
  const uint32_t *poff = has_past ? d_past_off.get() : nullptr;
  k_cmd<<<grid_for(ncmd, B), B, 0, stream>>>(a, ncmd, d_key_off.get(), key32, d_dot.get(), edep,
                                             edep2, etail, noop_latest, poff, d_past.get(),
                                             latest.get(), tmp, cnt);
  exclusive_scan_u32(cnt, off, ncmd, scan_ws, stream);
  uint32_t total = 0;
  FH_HIP(hipMemcpyAsync(&total, off + ncmd, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
  FH_HIP(hipStreamSynchronize(stream));
  uint64_t *dout = d_out.ensure(total ? total : 1);
  k_compact<<<grid_for(ncmd, B), B, 0, stream>>>(a, ncmd, d_key_off.get(), poff, dm, tmp, off,
                                                 dout);
  if (dev_out) {
    // device-resident caller (one segment: a = 0, out_base = 0)
    FH_HIP(hipMemcpyAsync(out_off, off, (ncmd + 1) * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                          stream));
    if (total)
      FH_HIP(hipMemcpyAsync(out_dep, dout, size_t(total) * sizeof(uint64_t),
                            hipMemcpyDeviceToDevice, stream));
    FH_HIP(hipStreamSynchronize(stream));
  } else {
    std::vector<uint32_t> hoff(ncmd + 1);
    FH_HIP(hipMemcpyAsync(hoff.data(), off, (ncmd + 1) * sizeof(uint32_t),
                          hipMemcpyDeviceToHost, stream));
    if (total)
      FH_HIP(hipMemcpyAsync(out_dep + out_base, dout, size_t(total) * sizeof(uint64_t),
                            hipMemcpyDeviceToHost, stream));
    FH_HIP(hipStreamSynchronize(stream));
    for (uint32_t i = 0; i <= ncmd; i++) out_off[a + i] = uint32_t(out_base + hoff[i]);
  }
  check_err("add_batch");
  seen_ub = std::min<uint64_t>(key_space, seen_ub + m);
  return total;
}

// All non-zero entries of the latest table (+ extra dot if non-zero), sorted
// ascending, written to device buffer d_out; returns count.
size_t KeyDepsDevice::table_values(uint64_t extra) {
  const unsigned B = 256;
  const uint32_t K = uint32_t(key_space);
  uint32_t *flags = d_cnt.ensure(K);
  uint32_t *pos = d_off.ensure(K + 1);
  // the latest (write) table, then the latest reads under read/write rules
  // (do_noop_deps, locked.rs:156-169)
  const uint64_t *tables[2] = {latest.get(), rw ? latest_r.get() : nullptr};
  uint32_t tot[2] = {0, 0};
  for (int t = 0; t < 2 && tables[t]; t++) {
    k_nonzero_flags<<<grid_for(K, B), B, 0, stream>>>(tables[t], K, flags);
    exclusive_scan_u32(flags, pos, K, scan_ws, stream);
    FH_HIP(hipMemcpyAsync(&tot[t], pos + K, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    FH_HIP(hipStreamSynchronize(stream));
    if (t == 0) d_out.ensure(size_t(tot[0]) + (rw ? K : 0) + 2);
    k_nonzero_gather<<<grid_for(K, B), B, 0, stream>>>(tables[t], K, pos,
                                                        d_out.get() + (t ? tot[0] : 0));
  }
  const uint32_t total = tot[0] + tot[1];
  const size_t cnt = size_t(total) + (extra ? 1 : 0);
  uint64_t *vals = d_out.get();
  if (extra)
    FH_HIP(hipMemcpyAsync(vals + total, &extra, sizeof(uint64_t), hipMemcpyHostToDevice, stream));
  if (cnt > 1) {
    // sort the dot set (64-bit keys) and drop duplicates on the way out
    uint64_t *ka = d_q64a.ensure(cnt), *kb = d_q64b.ensure(cnt);
    uint32_t *va = d_sv_a.ensure(cnt), *vb = d_sv_b.ensure(cnt);
    uint64_t *ks = nullptr;
    uint32_t *vs = nullptr;
    sort_pairs<uint64_t, uint32_t>(vals, nullptr, ka, va, kb, vb, cnt, 64, sort_ws, stream, &ks, &vs);
    FH_HIP(hipMemcpyAsync(vals, ks, cnt * sizeof(uint64_t), hipMemcpyDeviceToDevice, stream));
  }
  return cnt;
}

size_t KeyDepsDevice::download_unique(size_t cnt, uint64_t *out, size_t cap) {
  std::vector<uint64_t> h(cnt);
  if (cnt)
    FH_HIP(hipMemcpyAsync(h.data(), d_out.get(), cnt * sizeof(uint64_t), hipMemcpyDeviceToHost,
                          stream));
  FH_HIP(hipStreamSynchronize(stream));
  size_t w = 0;
  for (size_t i = 0; i < cnt; i++)
    if (w == 0 || h[i] != h[w - 1]) h[w++] = h[i];
  for (size_t i = 0; i < w && i < cap; i++) out[i] = h[i];
  return w;
}

void KeyDepsDevice::add_batch(size_t n, const uint64_t *dot, const uint32_t *key_off,
                              const uint64_t *key_id, const uint8_t *is_noop,
                              const uint32_t *past_off, const uint64_t *past_dot,
                              uint32_t *out_off, uint64_t *out_dep, size_t out_cap,
                              size_t *out_len, const uint8_t *read_only) {
  FH_CHECK(out_off && out_len && (n == 0 || (dot && key_off)), FH_EINVAL, "null argument");
  FH_CHECK(n < (size_t(1) << 30), FH_EINVAL, "batch too large");
  const bool has_past = past_off != nullptr;
  const bool has_ro = read_only != nullptr;
  // capacity bound (checked before any state change); read/write rules give
  // up to two deps per key and noops see both tables
  size_t noops = 0;
  for (size_t i = 0; i < n; i++) noops += (is_noop && is_noop[i]) ? 1 : 0;
  const size_t nkeys = n ? key_off[n] : 0;
  const size_t tables = (has_ro || rw) ? 2 : 1;
  size_t bound = nkeys * (has_ro ? 2 : 1) + (n - noops) + (has_past ? past_off[n] : 0);
  if (noops)
    bound += noops * (tables * std::min<uint64_t>(key_space, seen_ub + nkeys) + 1);
  if (out_cap < bound || (bound && !out_dep)) {
    *out_len = bound;
    throw Error(FH_ECAP, "output capacity too small");
  }
  for (size_t e = 0; e < nkeys; e++)  // validate before any state change
    FH_CHECK(key_id[e] < key_space, FH_EINVAL, "add_batch: key id >= key_space");
  FH_HIP(hipSetDevice(device));
  out_off[0] = 0;
  if (n == 0) {
    *out_len = 0;
    return;
  }
  h_key_off.assign(key_off, key_off + n + 1);
  if (has_past) h_past_off.assign(past_off, past_off + n + 1);
  // stage inputs
  FH_HIP(hipMemcpyAsync(d_dot.ensure(n), dot, n * sizeof(uint64_t), hipMemcpyHostToDevice,
                        stream));
  FH_HIP(hipMemcpyAsync(d_key_off.ensure(n + 1), key_off, (n + 1) * sizeof(uint32_t),
                        hipMemcpyHostToDevice, stream));
  if (nkeys)
    FH_HIP(hipMemcpyAsync(d_key64.ensure(nkeys), key_id, nkeys * sizeof(uint64_t),
                          hipMemcpyHostToDevice, stream));
  else
    d_key64.ensure(1);
  if (has_past) {
    FH_HIP(hipMemcpyAsync(d_past_off.ensure(n + 1), past_off, (n + 1) * sizeof(uint32_t),
                          hipMemcpyHostToDevice, stream));
    if (past_off[n])
      FH_HIP(hipMemcpyAsync(d_past.ensure(past_off[n]), past_dot, past_off[n] * sizeof(uint64_t),
                            hipMemcpyHostToDevice, stream));
    else
      d_past.ensure(1);
  } else {
    d_past.ensure(1);
  }
  if (has_ro) {
    enable_rw();
    FH_HIP(hipMemcpyAsync(d_ro.ensure(n), read_only, n, hipMemcpyHostToDevice, stream));
  }
  size_t written = 0;
  size_t i = 0;
  while (i < n) {
    size_t j = i;
    while (j < n && !(is_noop && is_noop[j])) j++;
    if (j > i)
      written += run_segment(uint32_t(i), uint32_t(j), has_past, has_ro, out_off, out_dep,
                             written);
    if (j < n) {
      // noop (do_add_noop :106-123): deps = previous noop + latest of every key
      const uint64_t prev = noop_latest;
      const size_t cnt = table_values(prev);
      const size_t w = download_unique(cnt, out_dep + written, out_cap - written);
      written += w;
      out_off[j + 1] = uint32_t(written);
      noop_latest = dot[j];
      j++;
    }
    i = j;
  }
  *out_len = written;
}

void KeyDepsDevice::add_batch_device(size_t n, size_t nkeys, const uint64_t *dot,
                                     const uint32_t *key_off, const uint64_t *key_id,
                                     uint32_t *out_off, uint64_t *out_dep, size_t out_cap,
                                     size_t *out_len, hipStream_t user) {
  FH_CHECK(out_off && out_len && (n == 0 || (dot && key_off && (nkeys == 0 || key_id))),
           FH_EINVAL, "null argument");
  FH_CHECK(n < (size_t(1) << 30) && nkeys < (size_t(1) << 31), FH_EINVAL, "batch too large");
  FH_CHECK(!rw, FH_EINVAL, "add_batch_device: handle uses read/write rules");
  // every command: one dep per key + the latest noop (sequential.rs:72-104)
  const size_t bound = nkeys + n;
  if (out_cap < bound || (bound && !out_dep)) {
    *out_len = bound;
    throw Error(FH_ECAP, "output capacity too small");
  }
  FH_HIP(hipSetDevice(device));
  // the caller's stream produced the inputs; this handle's stream reads them
  FH_HIP(hipStreamSynchronize(user));
  if (n == 0) {
    const uint32_t z = 0;
    FH_HIP(hipMemcpyAsync(out_off, &z, sizeof(z), hipMemcpyHostToDevice, stream));
    FH_HIP(hipStreamSynchronize(stream));
    *out_len = 0;
    return;
  }
  FH_HIP(hipMemcpyAsync(d_dot.ensure(n), dot, n * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                        stream));
  FH_HIP(hipMemcpyAsync(d_key_off.ensure(n + 1), key_off, (n + 1) * sizeof(uint32_t),
                        hipMemcpyDeviceToDevice, stream));
  if (nkeys)
    FH_HIP(hipMemcpyAsync(d_key64.ensure(nkeys), key_id, nkeys * sizeof(uint64_t),
                          hipMemcpyDeviceToDevice, stream));
  else
    d_key64.ensure(1);
  d_past.ensure(1);
  // run_segment reads the segment's element bounds on the host
  h_key_off.assign(n + 1, 0);
  h_key_off[n] = uint32_t(nkeys);
  *out_len = run_segment(0, uint32_t(n), false, false, out_off, out_dep, 0, true);
}

size_t KeyDepsDevice::cmd_deps(size_t nkeys, const uint64_t *key_id, uint64_t *out, size_t cap) {
  FH_HIP(hipSetDevice(device));
  std::vector<uint64_t> vals(nkeys);
  if (nkeys) {
    uint64_t *dk = d_q64a.ensure(nkeys);
    uint64_t *dv = d_q64b.ensure(nkeys);
    FH_HIP(hipMemcpyAsync(dk, key_id, nkeys * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
    k_gather_keys<<<grid_for(nkeys, 256), 256, 0, stream>>>(latest.get(), dk, uint32_t(nkeys),
                                                            key_space, dv, err.get());
    FH_HIP(hipMemcpyAsync(vals.data(), dv, nkeys * sizeof(uint64_t), hipMemcpyDeviceToHost,
                          stream));
    check_err("cmd_deps");
    if (rw) {  // do_cmd_deps (locked.rs:172-185): latest read and write
      std::vector<uint64_t> rv(nkeys);
      k_gather_keys<<<grid_for(nkeys, 256), 256, 0, stream>>>(latest_r.get(), dk,
                                                              uint32_t(nkeys), key_space, dv,
                                                              err.get());
      FH_HIP(hipMemcpyAsync(rv.data(), dv, nkeys * sizeof(uint64_t), hipMemcpyDeviceToHost,
                            stream));
      check_err("cmd_deps");
      vals.insert(vals.end(), rv.begin(), rv.end());
    }
  }
  if (noop_latest) vals.push_back(noop_latest);
  std::vector<uint64_t> s;
  for (uint64_t v : vals)
    if (v) s.push_back(v);
  std::sort(s.begin(), s.end());
  s.erase(std::unique(s.begin(), s.end()), s.end());
  for (size_t i = 0; i < s.size() && i < cap; i++) out[i] = s[i];
  return s.size();
}

size_t KeyDepsDevice::noop_deps(uint64_t *out, size_t cap) {
  FH_HIP(hipSetDevice(device));
  const size_t cnt = table_values(noop_latest);
  return download_unique(cnt, out, cap);
}

}  // namespace fh

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
struct fh_keydeps {
  fh::KeyDepsDevice dev;
  fh_keydeps(uint64_t s, const fh_config &c) : dev(s, c) {}
};

extern "C" {

fh_status fh_keydeps_create(uint64_t shard_id, const fh_config *cfg, fh_keydeps **out) {
  FH_API_BEGIN
  FH_CHECK(cfg && out, FH_EINVAL, "null argument");
  *out = new fh_keydeps(shard_id, *cfg);
  FH_API_END
}

fh_status fh_keydeps_destroy(fh_keydeps *h) {
  FH_API_BEGIN
  delete h;
  FH_API_END
}

fh_status fh_keydeps_add_batch(fh_keydeps *h, size_t n, const uint64_t *dot,
                               const uint32_t *key_off, const uint64_t *key_id,
                               const uint8_t *is_noop, const uint32_t *past_off,
                               const uint64_t *past_dot, uint32_t *out_dep_off,
                               uint64_t *out_dep_dot, size_t out_cap, size_t *out_len) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.add_batch(n, dot, key_off, key_id, is_noop, past_off, past_dot, out_dep_off,
                   out_dep_dot, out_cap, out_len);
  FH_API_END
}

fh_status fh_keydeps_add_batch_device(fh_keydeps *h, size_t n, size_t nkeys,
                                      const uint64_t *dot_dev, const uint32_t *key_off_dev,
                                      const uint64_t *key_id_dev, uint32_t *out_off_dev,
                                      uint64_t *out_dep_dev, size_t out_cap, size_t *out_len,
                                      void *stream) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  h->dev.add_batch_device(n, nkeys, dot_dev, key_off_dev, key_id_dev, out_off_dev, out_dep_dev,
                          out_cap, out_len, reinterpret_cast<hipStream_t>(stream));
  FH_API_END
}

fh_status fh_keydeps_add_batch_rw(fh_keydeps *h, size_t n, const uint64_t *dot,
                                  const uint32_t *key_off, const uint64_t *key_id,
                                  const uint8_t *read_only, const uint8_t *is_noop,
                                  const uint32_t *past_off, const uint64_t *past_dot,
                                  uint32_t *out_dep_off, uint64_t *out_dep_dot, size_t out_cap,
                                  size_t *out_len) {
  FH_API_BEGIN
  FH_CHECK(h && (n == 0 || read_only), FH_EINVAL, "null argument");
  h->dev.add_batch(n, dot, key_off, key_id, is_noop, past_off, past_dot, out_dep_off,
                   out_dep_dot, out_cap, out_len, n ? read_only : nullptr);
  FH_API_END
}

fh_status fh_keydeps_cmd_deps(fh_keydeps *h, size_t nkeys, const uint64_t *key_id,
                              uint64_t *out, size_t cap, size_t *out_len) {
  FH_API_BEGIN
  FH_CHECK(h && out_len && (nkeys == 0 || key_id), FH_EINVAL, "null argument");
  uint64_t tmp[1];
  *out_len = h->dev.cmd_deps(nkeys, key_id, out ? out : tmp, out ? cap : 0);
  FH_CHECK(*out_len <= cap || !out, FH_ECAP, "output capacity too small");
  FH_API_END
}

fh_status fh_keydeps_noop_deps(fh_keydeps *h, uint64_t *out, size_t cap, size_t *out_len) {
  FH_API_BEGIN
  FH_CHECK(h && out_len, FH_EINVAL, "null argument");
  uint64_t tmp[1];
  *out_len = h->dev.noop_deps(out ? out : tmp, out ? cap : 0);
  FH_CHECK(*out_len <= cap || !out, FH_ECAP, "output capacity too small");
  FH_API_END
}

}  // extern "C"
