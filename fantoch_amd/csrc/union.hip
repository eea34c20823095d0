// union.hip -- per-command union of dependency records (partial replication).
//
// Atlas with partial replication commits a multi-shard command with the
// union of every shard's committed deps (MShardCommit, fantoch_ps/src/
// protocol/atlas.rs:559-639, the union at :580-583); each shard's KeyDeps
// only sees the command's keys on that shard (deps/keys/sequential.rs:81,
// Command::keys(shard) fantoch/src/command.rs:95-100).  In the multi-GPU
// engine every shard sends (command, dep) records to the command's owner
// (RCCL all-to-all, fantoch_amd/partial.py); this file is the owner's merge:
// records in any order, duplicates allowed -> CSR of ascending unique deps.
//
//   k_rec_hist     records per command (LDS-free global atomics; commands are
//                  many and records few per command)
//   scan           segment offsets
//   k_rec_place    records into their command's segment (any order)
//   k_seg_unique   one thread per command: insertion sort of its segment in
//                  place + count of distinct deps (segments hold the deps of
//                  <= keys x shards reports, a handful of entries)
//   scan           output offsets
//   k_seg_compact  distinct deps to the output CSR
#include "fh_common.h"
#include "scan.h"

namespace fh {
namespace {

constexpr int kB = 256;

// records naming a command >= n are dropped (the host wrapper rejects them
// first; the guard only keeps a bad call from writing out of bounds)
__global__ void k_rec_hist(size_t n, size_t nrec, const uint32_t *__restrict__ cmd,
                           uint32_t *__restrict__ cnt) {
  for (size_t i = size_t(blockIdx.x) * kB + threadIdx.x; i < nrec; i += size_t(gridDim.x) * kB)
    if (cmd[i] < n) atomicAdd(&cnt[cmd[i]], 1u);
}

__global__ void k_rec_place(size_t n, size_t nrec, const uint32_t *__restrict__ cmd,
                            const uint64_t *__restrict__ dep, const uint32_t *__restrict__ off,
                            uint32_t *__restrict__ cur, uint64_t *__restrict__ seg) {
  for (size_t i = size_t(blockIdx.x) * kB + threadIdx.x; i < nrec; i += size_t(gridDim.x) * kB) {
    const uint32_t c = cmd[i];
    if (c < n) seg[off[c] + atomicAdd(&cur[c], 1u)] = dep[i];
  }
}

__global__ void k_seg_unique(size_t n, const uint32_t *__restrict__ off, uint64_t *__restrict__ seg,
                             uint32_t *__restrict__ ucnt) {
  for (size_t c = size_t(blockIdx.x) * kB + threadIdx.x; c < n; c += size_t(gridDim.x) * kB) {
    const uint32_t a = off[c], e = off[c + 1];
    for (uint32_t i = a + 1; i < e; i++) {  // insertion sort
      const uint64_t x = seg[i];
      uint32_t j = i;
      while (j > a && seg[j - 1] > x) {
        seg[j] = seg[j - 1];
        j--;
      }
      seg[j] = x;
    }
    uint32_t u = 0;
    for (uint32_t i = a; i < e; i++) u += (i == a || seg[i] != seg[i - 1]);
    ucnt[c] = u;
  }
}

__global__ void k_seg_compact(size_t n, const uint32_t *__restrict__ off,
                              const uint64_t *__restrict__ seg, const uint32_t *__restrict__ uoff,
                              uint64_t *__restrict__ out) {
  for (size_t c = size_t(blockIdx.x) * kB + threadIdx.x; c < n; c += size_t(gridDim.x) * kB) {
    uint32_t o = uoff[c];
    const uint32_t a = off[c], e = off[c + 1];
    for (uint32_t i = a; i < e; i++)
      if (i == a || seg[i] != seg[i - 1]) out[o++] = seg[i];
  }
}

unsigned grid_of(size_t n) { return unsigned(std::min<size_t>((n + kB - 1) / kB, 8192)); }

struct UnionWorkspace {
  DBuf<uint32_t> cnt, off, cur, ucnt;
  DBuf<uint64_t> seg;
  ScanWorkspace scan;
};

}  // namespace

// out_off[n_cmd + 1], out_dep[<= nrec]; returns the number of distinct deps
size_t dep_union(size_t n_cmd, size_t nrec, const uint32_t *cmd, const uint64_t *dep,
                 uint32_t *out_off, uint64_t *out_dep, hipStream_t s) {
  static thread_local UnionWorkspace ws;
  FH_CHECK(nrec < (size_t(1) << 32), FH_EINVAL, "dep_union: more than 2^32 records");
  uint32_t *cnt = ws.cnt.ensure(n_cmd + 1), *off = ws.off.ensure(n_cmd + 2);
  uint32_t *cur = ws.cur.ensure(n_cmd + 1), *ucnt = ws.ucnt.ensure(n_cmd + 1);
  uint64_t *seg = ws.seg.ensure(nrec + 1);
  FH_HIP(hipMemsetAsync(cnt, 0, (n_cmd + 1) * sizeof(uint32_t), s));
  FH_HIP(hipMemsetAsync(cur, 0, (n_cmd + 1) * sizeof(uint32_t), s));
  if (nrec) k_rec_hist<<<grid_of(nrec), kB, 0, s>>>(n_cmd, nrec, cmd, cnt);
  exclusive_scan_u32(cnt, off, n_cmd, ws.scan, s);
  if (nrec) k_rec_place<<<grid_of(nrec), kB, 0, s>>>(n_cmd, nrec, cmd, dep, off, cur, seg);
  if (n_cmd) k_seg_unique<<<grid_of(n_cmd), kB, 0, s>>>(n_cmd, off, seg, ucnt);
  exclusive_scan_u32(ucnt, out_off, n_cmd, ws.scan, s);
  if (n_cmd) k_seg_compact<<<grid_of(n_cmd), kB, 0, s>>>(n_cmd, off, seg, out_off, out_dep);
  FH_HIP(hipGetLastError());
  uint32_t total = 0;
  FH_HIP(hipMemcpyAsync(&total, out_off + n_cmd, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  FH_HIP(hipStreamSynchronize(s));
  return total;
}

}  // namespace fh

extern "C" {

fh_status fh_dep_union(int device, size_t n_cmd, size_t nrec, const uint32_t *cmd,
                       const uint64_t *dep, uint32_t *out_off, uint64_t *out_dep,
                       size_t *out_len, void *stream) {
  FH_API_BEGIN
  FH_CHECK(out_off && out_len && (nrec == 0 || (cmd && dep && out_dep)), FH_EINVAL,
           "null argument");
  if (device >= 0) FH_HIP(hipSetDevice(device));
  *out_len = fh::dep_union(n_cmd, nrec, cmd, dep, out_off, out_dep,
                           reinterpret_cast<hipStream_t>(stream));
  FH_API_END
}

}  // extern "C"
