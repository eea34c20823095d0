// keydeps.h -- device-resident KeyDeps state (see keydeps.hip).
#pragma once

#include <vector>

#include "fh_common.h"
#include "scan.h"
#include "sort.h"

namespace fh {

struct KeyDepsDevice {
  uint64_t shard_id = 0;
  uint64_t key_space = 0;
  int key_bits = 1;
  int device = 0;
  hipStream_t stream = nullptr;
  DBuf<uint64_t> latest;      // latest_deps (sequential.rs:10), 0 = none; the
                              // latest write under read/write semantics
  DBuf<uint64_t> latest_r;    // latest read (LatestRW.read, locked.rs:12-15),
                              // allocated by the first read/write batch
  bool rw = false;            // latest_r is live
  uint64_t noop_latest = 0;   // noop_latest_dep (sequential.rs:11), 0 = None
  uint64_t seen_ub = 0;       // upper bound on distinct keys in the table
  DBuf<uint32_t> err;
  // staged batch + scratch
  std::vector<uint32_t> h_key_off, h_past_off;
  DBuf<uint64_t> d_dot, d_key64, d_past, d_elem_dep, d_elem_dep2, d_tmp, d_out, d_q64a, d_q64b;
  DBuf<uint32_t> d_key_off, d_past_off, d_key32, d_cmd_of, d_cnt, d_off;
  DBuf<uint32_t> d_sk_a, d_sk_b, d_sv_a, d_sv_b;
  DBuf<uint32_t> d_mh, d_mw, d_mr, d_sh, d_sw, d_sr;  // read/write segment marks + scans
  DBuf<uint8_t> d_elem_tail, d_ro;
  SortWorkspace sort_ws;
  ScanWorkspace scan_ws;

  KeyDepsDevice(uint64_t shard_id, const fh_config &cfg);
  ~KeyDepsDevice();
  // read_only == NULL: SequentialKeyDeps; otherwise LockedKeyDeps' read/write
  // rules (locked.rs:83-128) with read_only[i] = Command::read_only
  void add_batch(size_t n, const uint64_t *dot, const uint32_t *key_off, const uint64_t *key_id,
                 const uint8_t *is_noop, const uint32_t *past_off, const uint64_t *past_dot,
                 uint32_t *out_off, uint64_t *out_dep, size_t out_cap, size_t *out_len,
                 const uint8_t *read_only = nullptr);
  // device-resident batch (no noops, no past): inputs and outputs are device
  // pointers on this handle's device
  void add_batch_device(size_t n, size_t nkeys, const uint64_t *dot, const uint32_t *key_off,
                        const uint64_t *key_id, uint32_t *out_off, uint64_t *out_dep,
                        size_t out_cap, size_t *out_len, hipStream_t user);
  size_t cmd_deps(size_t nkeys, const uint64_t *key_id, uint64_t *out, size_t cap);
  size_t noop_deps(uint64_t *out, size_t cap);

 private:
  size_t run_segment(uint32_t a, uint32_t b, bool has_past, bool has_ro, uint32_t *out_off,
                     uint64_t *out_dep, size_t out_base, bool dev_out = false);
  void enable_rw();
  size_t table_values(uint64_t extra);
  size_t download_unique(size_t cnt, uint64_t *out, size_t cap);
  void check_err(const char *what);
};

}  // namespace fh
