//! The batched, device-resident path (`fh_engine_*`): a committed stream of
//! commands -> per-replica KeyDeps (fast-quorum views, QuorumDeps union,
//! quorum.rs:28-98) -> dependency graph -> SCCs -> execution order -> per-key
//! execution sequences, every output materialised on the device by `run`.
//! This is the entry the throughput metric is measured on; the replay of an
//! execution log (bin/graph_executor_replay.rs:13-38) or an offline checker
//! of a recorded run feeds it whole batches instead of one info at a time.
use crate::{check, ffi};
use std::ptr::null_mut;

pub struct Engine {
    h: *mut ffi::FhEngine,
    key_space: u64,
    n: usize,
    k: usize,
}

unsafe impl Send for Engine {}

impl Drop for Engine {
    fn drop(&mut self) {
        unsafe {
            ffi::fh_engine_destroy(self.h);
        }
    }
}

/// The outputs of one run.
#[derive(Debug, Default, Clone)]
pub struct EngineResults {
    pub dep_off: Vec<u32>,   // committed deps per command (CSR of packed dots)
    pub deps: Vec<u64>,
    pub scc_label: Vec<u64>, // min dot of each command's SCC
    pub exec_rank: Vec<u32>, // position of each command in the execution order
    pub key_off: Vec<u32>,   // per-key execution sequences (CSR over key ids)
    pub key_seq: Vec<u64>,
}

impl Engine {
    /// n processes, key ids < key_space; device -1 = FANTOCH_HIP_DEVICE or 0
    pub fn new(n: usize, key_space: u64, device: i32) -> Self {
        let cfg = ffi::FhConfig { n: n as u32, f: 1, shard_count: 1, device, key_space };
        let mut h = null_mut();
        check(unsafe { ffi::fh_engine_create(&cfg, &mut h) });
        Self { h, key_space, n: 0, k: 0 }
    }

    /// Replica views as the replicas' own arrival logs: log r lists the
    /// batch-local commands replica r + 1's KeyDeps processes, in order.
    pub fn stage_logs(&mut self, nproc: u32, views: u32, dots: &[u64], keys: &[u64], k: usize,
                      log_off: &[u64], log_cmd: &[u32]) {
        self.stage_logs_flags(nproc, views, dots, keys, k, log_off, log_cmd, 0);
    }

    /// Partial replication: element logs (FH_STREAM_ELEMENT_LOGS), entry =
    /// element position (c * views + j) * k + s; nproc = processes of every
    /// shard (log r = process r + 1).
    pub fn stage_element_logs(&mut self, nproc: u32, views: u32, dots: &[u64], keys: &[u64],
                              k: usize, log_off: &[u64], log_elem: &[u32]) {
        self.stage_logs_flags(nproc, views, dots, keys, k, log_off, log_elem,
                              ffi::FH_STREAM_ELEMENT_LOGS);
    }

    fn stage_logs_flags(&mut self, nproc: u32, views: u32, dots: &[u64], keys: &[u64], k: usize,
                        log_off: &[u64], log_cmd: &[u32], flags: u32) {
        let desc = ffi::FhStreamDesc {
            n: dots.len(),
            keys_per_cmd: k as u32,
            views,
            nproc,
            flags,
        };
        check(unsafe {
            ffi::fh_engine_stage_logs(self.h, &desc, 1, dots.as_ptr(), keys.as_ptr(),
                log_off.as_ptr(), log_cmd.as_ptr())
        });
        self.n = dots.len();
        self.k = k;
    }

    /// One replica's stream (SequentialKeyDeps in stream order).
    pub fn stage_single_view(&mut self, dots: &[u64], keys: &[u64], k: usize) {
        let desc = ffi::FhStreamDesc { n: dots.len(), keys_per_cmd: k as u32, ..Default::default() };
        check(unsafe {
            ffi::fh_engine_stage(self.h, &desc, dots.as_ptr(), keys.as_ptr(),
                std::ptr::null(), std::ptr::null())
        });
        self.n = dots.len();
        self.k = k;
    }

    pub fn run(&mut self) {
        check(unsafe { ffi::fh_engine_run(self.h, null_mut()) });
    }

    /// Deps-only runs: the per-shard stage of partial replication (the
    /// committed deps feed the cross-shard union before any graph work).
    pub fn set_deps_only(&mut self, on: bool) {
        check(unsafe { ffi::fh_engine_set_deps_only(self.h, on as i32) });
    }

    /// The next run starts from a fresh engine's tuning guesses (cold run).
    pub fn forget_tuning(&mut self) {
        check(unsafe { ffi::fh_engine_forget_tuning(self.h) });
    }

    /// The last run's committed deps (dep_off[n + 1], deps).
    pub fn deps(&self) -> (Vec<u32>, Vec<u64>) {
        let mut off = vec![0u32; self.n + 1];
        let mut len = 0usize;
        check(unsafe {
            ffi::fh_engine_results(self.h, off.as_mut_ptr(), null_mut(), 0, &mut len,
                null_mut(), null_mut(), null_mut(), null_mut())
        });
        let mut deps = vec![0u64; len];
        check(unsafe {
            ffi::fh_engine_results(self.h, off.as_mut_ptr(), deps.as_mut_ptr(), len, &mut len,
                null_mut(), null_mut(), null_mut(), null_mut())
        });
        (off, deps)
    }

    pub fn results(&self) -> EngineResults {
        let mut r = EngineResults {
            dep_off: vec![0; self.n + 1],
            scc_label: vec![0; self.n],
            exec_rank: vec![0; self.n],
            key_off: vec![0; self.key_space as usize + 1],
            ..Default::default()
        };
        let mut len = 0usize;
        check(unsafe {
            ffi::fh_engine_results(self.h, r.dep_off.as_mut_ptr(), null_mut(), 0, &mut len,
                null_mut(), null_mut(), r.key_off.as_mut_ptr(), null_mut())
        });
        r.deps = vec![0; len];
        r.key_seq = vec![0; *r.key_off.last().unwrap() as usize];
        check(unsafe {
            ffi::fh_engine_results(self.h, r.dep_off.as_mut_ptr(), r.deps.as_mut_ptr(), len,
                &mut len, r.scc_label.as_mut_ptr(), r.exec_rank.as_mut_ptr(),
                r.key_off.as_mut_ptr(), r.key_seq.as_mut_ptr())
        });
        r
    }
}
