//! `Executor` (fantoch/src/executor/mod.rs:27-88) with `GraphExecutor`'s
//! semantics (fantoch_ps/src/executor/graph/executor.rs:19-197) on the HIP
//! engine's dependency graph (`fh_graph_*`).
//!
//! One `fh_graph` per shard plays both executor roles, as the reference's
//! executor 0 (Add, RequestReply) and executor 1 (Request, Executed) share
//! one `VertexIndex` through an `Arc` (graph/index.rs:21): clones made by
//! the runner (run/task/executor.rs:33-48) share the handle, so the executed
//! clock the secondary role answers requests with is the main role's
//! (`handle_executed`, graph/mod.rs:199-212, becomes a no-op).
//!
//! Every FFI sequence on the shared handle runs under one `Mutex` guard (the
//! runner drives the clones from separate tokio tasks, and `fh_graph` is
//! single-threaded).  Roles follow the reference's message routing
//! (executor.rs:242-262): only the main role (executor index 0) adds
//! vertices, drains ready commands and executes them on its `KVStore`; the
//! secondary role (index 1) answers other shards' requests and sends the
//! replies.  A drained dot therefore always reaches the store, monitor and
//! client channel of the task that added it.
//!
//! `Executor::handle` is synchronous per `ExecutionInfo` (the runners drain
//! `to_clients` after every call: run/task/executor.rs:150-175,
//! sim/runner.rs:407-413), so an `Add` is one device pass over a batch of
//! one.  `handle_batch` takes a run of infos at once (replay, benchmarks):
//! consecutive `Add`s become one `fh_graph_add_batch`, with the same
//! execution order as one at a time.
//!
//! `RequestReply` lives in a private module of fantoch_ps; the binding needs
//! it re-exported next to `GraphExecutionInfo`
//! (`pub use graph::{GraphExecutionInfo, GraphExecutor, RequestReply};` in
//! fantoch_ps/src/executor/mod.rs:14), a one-word change.
use crate::{check, ffi, mask, pack, unmask, unpack, Interner};
use fantoch::command::Command;
use fantoch::config::Config;
use fantoch::executor::{
    ExecutionOrderMonitor, Executor, ExecutorMetrics, ExecutorMetricsKind, ExecutorResult,
};
use fantoch::id::{Dot, ProcessId, ShardId};
use fantoch::kvs::KVStore;
use fantoch::time::SysTime;
use fantoch::{HashMap, HashSet};
use fantoch_ps::executor::{GraphExecutionInfo, RequestReply};
use fantoch_ps::protocol::common::graph::Dependency;
use std::collections::VecDeque;
use std::ptr::null_mut;
use std::sync::{Arc, Mutex, MutexGuard};

/// MONITOR_PENDING_THRESHOLD (graph/mod.rs:31)
const MONITOR_PENDING_THRESHOLD_MS: u64 = 1000;

struct Handle(*mut ffi::FhGraph);
unsafe impl Send for Handle {}
unsafe impl Sync for Handle {}
impl Drop for Handle {
    fn drop(&mut self) {
        unsafe {
            ffi::fh_graph_destroy(self.0);
        }
    }
}

struct Shared {
    h: Handle,
    keys: Interner,
    // payloads stay on the host: dot -> command until it executes (the
    // device sees only dots, key ids and deps)
    cmds: HashMap<Dot, Command>,
}

#[derive(Clone)]
pub struct HipGraphExecutor {
    executor_index: usize,
    process_id: ProcessId,
    shard_id: ShardId,
    config: Config,
    shared: Arc<Mutex<Shared>>,
    store: KVStore,
    monitor: Option<ExecutionOrderMonitor>,
    metrics: ExecutorMetrics,
    to_clients: VecDeque<ExecutorResult>,
    to_executors: Vec<(ShardId, GraphExecutionInfo)>,
}

/// Arrays of one `fh_graph_add_batch(_sharded)` call.
#[derive(Default)]
struct Batch {
    dot: Vec<u64>,
    key_off: Vec<u32>,
    key_id: Vec<u64>,
    dep_off: Vec<u32>,
    dep_dot: Vec<u64>,
    cmd_shards: Vec<u64>,
    dep_shards: Vec<u64>,
}

impl Batch {
    fn new() -> Self {
        Self {
            key_off: vec![0],
            dep_off: vec![0],
            ..Default::default()
        }
    }

    fn push(&mut self, shard_id: ShardId, keys: &mut Interner, dot: Dot, cmd: &Command,
            deps: impl IntoIterator<Item = Dependency>) {
        self.dot.push(pack(dot));
        self.key_id.extend(cmd.keys(shard_id).map(|k| keys.id(k)));
        self.key_off.push(self.key_id.len() as u32);
        for d in deps {
            self.dep_dot.push(pack(d.dot));
            self.dep_shards.push(d.shards.as_ref().map(|s| mask(s.iter())).unwrap_or(0));
        }
        self.dep_off.push(self.dep_dot.len() as u32);
        self.cmd_shards.push(mask(cmd.shards()));
    }
}

impl HipGraphExecutor {
    /// The shared state, locked for a whole FFI sequence.  The guard borrows
    /// the `Arc` passed in (a clone), not `self`, so the caller can still
    /// update its own queues and metrics while holding it.
    fn lock(shared: &Arc<Mutex<Shared>>) -> MutexGuard<'_, Shared> {
        shared.lock().unwrap()
    }

    fn is_main(&self) -> bool {
        self.executor_index == 0
    }

    /// DependencyGraph::handle_add for a run of adds (graph/mod.rs:215-277):
    /// the device finds every SCC whose reachable set is complete, in the
    /// order the incremental Tarjan would have executed them.  Main role only.
    fn add_batch(&mut self, sh: &mut Shared, adds: Vec<(Dot, Command, Vec<Dependency>)>,
                 time: &dyn SysTime) {
        assert!(self.is_main(), "only executor 0 adds vertices (executor.rs:242-262)");
        let mut b = Batch::new();
        for (dot, cmd, deps) in adds {
            b.push(self.shard_id, &mut sh.keys, dot, &cmd, deps);
            sh.cmds.insert(dot, cmd);
        }
        let h = sh.h.0;
        check(unsafe { ffi::fh_graph_set_time(h, time.millis()) });
        let n = b.dot.len();
        check(unsafe {
            if self.config.shard_count() > 1 {
                ffi::fh_graph_add_batch_sharded(h, n, b.dot.as_ptr(), b.key_off.as_ptr(),
                    b.key_id.as_ptr(), b.dep_off.as_ptr(), b.dep_dot.as_ptr(),
                    b.cmd_shards.as_ptr(), b.dep_shards.as_ptr())
            } else {
                ffi::fh_graph_add_batch(h, n, b.dot.as_ptr(), b.key_off.as_ptr(),
                    b.key_id.as_ptr(), b.dep_off.as_ptr(), b.dep_dot.as_ptr())
            }
        });
    }

    /// fetch_actions (executor.rs:114-122), under the caller's guard
    fn fetch_actions(&mut self, sh: &mut Shared) {
        if self.is_main() {
            self.fetch_commands_to_execute(sh);
            self.fetch_metrics(sh);
        }
        if self.config.shard_count() > 1 {
            if self.is_main() {
                self.fetch_requests(sh);
            } else {
                self.fetch_request_replies(sh);
            }
        }
    }

    /// fetch_commands_to_execute (executor.rs:124-145): drained dots in
    /// execution order, executed on the KVStore + monitor.
    fn fetch_commands_to_execute(&mut self, sh: &mut Shared) {
        let h = sh.h.0;
        let len = crate::sized(|cap, len| unsafe {
            ffi::fh_graph_drain(h, null_mut(), null_mut(), cap, len)
        });
        if len == 0 {
            return;
        }
        let mut dots = vec![0u64; len];
        let mut got = 0usize;
        check(unsafe { ffi::fh_graph_drain(h, dots.as_mut_ptr(), null_mut(), len, &mut got) });
        for d in &dots[..got] {
            let cmd = sh.cmds.remove(&unpack(*d)).expect("drained dot has a command");
            self.execute(cmd);
        }
    }

    /// ChainSize / ExecutionDelay collected on the device side (save_scc,
    /// graph/mod.rs:490-525)
    fn fetch_metrics(&mut self, sh: &mut Shared) {
        let h = sh.h.0;
        let (mut nc, mut nd) = (0usize, 0usize);
        let st = unsafe {
            ffi::fh_graph_take_metrics(h, null_mut(), 0, null_mut(), 0, &mut nc, &mut nd)
        };
        if nc == 0 && nd == 0 {
            return check(st);
        }
        let (mut chain, mut delay) = (vec![0u64; nc], vec![0u64; nd]);
        check(unsafe {
            ffi::fh_graph_take_metrics(h, chain.as_mut_ptr(), nc, delay.as_mut_ptr(), nd,
                &mut nc, &mut nd)
        });
        for v in chain {
            self.metrics.collect(ExecutorMetricsKind::ChainSize, v);
        }
        for v in delay {
            self.metrics.collect(ExecutorMetricsKind::ExecutionDelay, v);
        }
    }

    /// fetch_requests (executor.rs:161-174; graph/mod.rs:147-150)
    fn fetch_requests(&mut self, sh: &mut Shared) {
        let h = sh.h.0;
        let len = crate::sized(|cap, len| unsafe {
            ffi::fh_graph_requests(h, null_mut(), null_mut(), cap, len)
        });
        if len == 0 {
            return;
        }
        let (mut dot, mut shard) = (vec![0u64; len], vec![0u64; len]);
        let mut got = 0usize;
        check(unsafe {
            ffi::fh_graph_requests(h, dot.as_mut_ptr(), shard.as_mut_ptr(), len, &mut got)
        });
        let mut by_shard: HashMap<ShardId, HashSet<Dot>> = HashMap::new();
        for (d, s) in dot.into_iter().zip(shard).take(got) {
            by_shard.entry(s).or_default().insert(unpack(d));
        }
        self.metrics.aggregate(ExecutorMetricsKind::OutRequests, got as u64);
        for (to, dots) in by_shard {
            let request = GraphExecutionInfo::Request { from: self.shard_id, dots };
            self.to_executors.push((to, request));
        }
    }

    /// fetch_request_replies (executor.rs:176-189; graph/mod.rs:152-157)
    fn fetch_request_replies(&mut self, sh: &mut Shared) {
        let h = sh.h.0;
        let (mut nr, mut nd) = (0usize, 0usize);
        let st = unsafe {
            ffi::fh_graph_request_replies(h, 0, null_mut(), null_mut(), null_mut(), null_mut(),
                null_mut(), 0, null_mut(), null_mut(), &mut nr, &mut nd)
        };
        if nr == 0 {
            return check(st);
        }
        let (mut to, mut kind, mut dot, mut cshard) =
            (vec![0u64; nr], vec![0u8; nr], vec![0u64; nr], vec![0u64; nr]);
        let (mut off, mut ddot, mut dshard) =
            (vec![0u32; nr + 1], vec![0u64; nd.max(1)], vec![0u64; nd.max(1)]);
        check(unsafe {
            ffi::fh_graph_request_replies(h, nr, to.as_mut_ptr(), kind.as_mut_ptr(),
                dot.as_mut_ptr(), cshard.as_mut_ptr(), off.as_mut_ptr(), nd, ddot.as_mut_ptr(),
                dshard.as_mut_ptr(), &mut nr, &mut nd)
        });
        let mut by_shard: HashMap<ShardId, Vec<RequestReply>> = HashMap::new();
        for i in 0..nr {
            let d = unpack(dot[i]);
            let reply = if kind[i] == 0 {
                // FH_REPLY_INFO: the command payload comes from this side
                let cmd = sh.cmds.get(&d).cloned().expect("Info reply for a held command");
                let deps = (off[i] as usize..off[i + 1] as usize)
                    .map(|e| Dependency { dot: unpack(ddot[e]), shards: unmask(dshard[e]) })
                    .collect();
                RequestReply::Info { dot: d, cmd, deps }
            } else {
                RequestReply::Executed { dot: d }
            };
            by_shard.entry(to[i]).or_default().push(reply);
        }
        for (to, infos) in by_shard {
            self.to_executors.push((to, GraphExecutionInfo::RequestReply { infos }));
        }
    }

    /// GraphExecutor::execute (executor.rs:191-196)
    fn execute(&mut self, cmd: Command) {
        let results = cmd.execute(self.shard_id, &mut self.store, &mut self.monitor);
        self.to_clients.extend(results);
    }

    /// A run of infos at once: consecutive `Add`s go to the device as one
    /// batch (one `fh_graph_add_batch`, the same execution order as one add
    /// at a time); anything else is handled in place, in order.
    pub fn handle_batch(&mut self, infos: Vec<GraphExecutionInfo>, time: &dyn SysTime) {
        let mut run = Vec::new();
        for info in infos {
            match info {
                GraphExecutionInfo::Add { dot, cmd, deps } if !self.config.execute_at_commit() => {
                    run.push((dot, cmd, deps.into_iter().collect()));
                }
                other => {
                    self.flush_adds(&mut run, time);
                    self.handle(other, time);
                }
            }
        }
        self.flush_adds(&mut run, time);
    }

    fn flush_adds(&mut self, run: &mut Vec<(Dot, Command, Vec<Dependency>)>, time: &dyn SysTime) {
        if run.is_empty() {
            return;
        }
        let shared = Arc::clone(&self.shared);
        let mut sh = Self::lock(&shared);
        self.add_batch(&mut sh, std::mem::take(run), time);
        self.fetch_actions(&mut sh);
    }
}

impl Executor for HipGraphExecutor {
    type ExecutionInfo = GraphExecutionInfo;

    fn new(process_id: ProcessId, shard_id: ShardId, config: Config) -> Self {
        let cfg = crate::config(config.n(), config.f(), config.shard_count());
        let mut h = null_mut();
        check(unsafe { ffi::fh_graph_create(process_id as u32, shard_id, &cfg, &mut h) });
        let shared = Shared {
            h: Handle(h),
            keys: Interner::default(),
            cmds: HashMap::new(),
        };
        let monitor = if config.executor_monitor_execution_order() {
            Some(ExecutionOrderMonitor::new())
        } else {
            None
        };
        Self {
            executor_index: 0,
            process_id,
            shard_id,
            config,
            shared: Arc::new(Mutex::new(shared)),
            store: KVStore::new(),
            monitor,
            metrics: ExecutorMetrics::new(),
            to_clients: VecDeque::new(),
            to_executors: Vec::new(),
        }
    }

    fn set_executor_index(&mut self, index: usize) {
        self.executor_index = index;
    }

    /// cleanup (executor.rs:65-70) -> check_pending_requests (mod.rs:168-179):
    /// buffered requests are retried by the role that answers them
    fn cleanup(&mut self, time: &dyn SysTime) {
        let _ = time;
        if self.config.shard_count() > 1 {
            let shared = Arc::clone(&self.shared);
            let mut sh = Self::lock(&shared);
            if !self.is_main() {
                check(unsafe { ffi::fh_graph_cleanup(sh.h.0) });
            }
            self.fetch_actions(&mut sh);
        }
    }

    /// monitor_pending (executor.rs:72-74; graph/mod.rs:181-196; index.rs:
    /// 53-103): pending commands older than 1 s are reported, and one without
    /// missing dependencies panics (FH_EINVARIANT -> check).
    fn monitor_pending(&mut self, time: &dyn SysTime) {
        if !self.is_main() {
            return;
        }
        let shared = Arc::clone(&self.shared);
        let sh = Self::lock(&shared);
        let h = sh.h.0;
        check(unsafe { ffi::fh_graph_set_time(h, time.millis()) });
        let len = crate::sized(|cap, len| unsafe {
            ffi::fh_graph_monitor_pending(h, MONITOR_PENDING_THRESHOLD_MS, null_mut(),
                null_mut(), null_mut(), cap, len)
        });
        let (mut dots, mut ms, mut missing) = (vec![0u64; len], vec![0u64; len], vec![0u64; len]);
        let mut got = 0usize;
        check(unsafe {
            ffi::fh_graph_monitor_pending(h, MONITOR_PENDING_THRESHOLD_MS, dots.as_mut_ptr(),
                ms.as_mut_ptr(), missing.as_mut_ptr(), len, &mut got)
        });
        drop(sh);
        for i in 0..got {
            tracing::info!(
                "p{}: {:?} is pending for {:?}ms | missing {} dependencies",
                self.process_id,
                unpack(dots[i]),
                ms[i],
                missing[i]
            );
        }
    }

    /// handle (executor.rs:76-100).  Add and RequestReply come to executor 0,
    /// Request and Executed to executor 1 (executor.rs:242-262).
    fn handle(&mut self, info: GraphExecutionInfo, time: &dyn SysTime) {
        let shared = Arc::clone(&self.shared);
        match info {
            GraphExecutionInfo::Add { dot, cmd, deps } => {
                if self.config.execute_at_commit() {
                    self.execute(cmd);
                } else {
                    let mut sh = Self::lock(&shared);
                    self.add_batch(&mut sh, vec![(dot, cmd, deps.into_iter().collect())], time);
                    self.fetch_actions(&mut sh);
                }
            }
            GraphExecutionInfo::Request { from, dots } => {
                self.metrics.aggregate(ExecutorMetricsKind::InRequests, 1);
                let d: Vec<u64> = dots.into_iter().map(pack).collect();
                let mut sh = Self::lock(&shared);
                check(unsafe { ffi::fh_graph_handle_requests(sh.h.0, from, d.len(), d.as_ptr()) });
                self.fetch_actions(&mut sh);
            }
            GraphExecutionInfo::RequestReply { infos } => {
                // in reply order (graph/mod.rs:377-408): runs of Info replies
                // are add batches, Executed updates the clock + retries
                self.metrics.aggregate(ExecutorMetricsKind::InRequestReplies, 1);
                let mut sh = Self::lock(&shared);
                let mut run = Vec::new();
                for info in infos {
                    match info {
                        RequestReply::Info { dot, cmd, deps } => run.push((dot, cmd, deps)),
                        RequestReply::Executed { dot } => {
                            if !run.is_empty() {
                                self.add_batch(&mut sh, std::mem::take(&mut run), time);
                            }
                            let d = [pack(dot)];
                            check(unsafe { ffi::fh_graph_mark_executed(sh.h.0, 1, d.as_ptr()) });
                            self.add_batch(&mut sh, Vec::new(), time); // check_pending
                        }
                    }
                }
                if !run.is_empty() {
                    self.add_batch(&mut sh, run, time);
                }
                self.fetch_actions(&mut sh);
            }
            GraphExecutionInfo::Executed { .. } => {
                // handle_executed: the shared handle already holds the clock
            }
        }
    }

    fn to_clients(&mut self) -> Option<ExecutorResult> {
        self.to_clients.pop_front()
    }

    fn to_executors(&mut self) -> Option<(ShardId, GraphExecutionInfo)> {
        self.to_executors.pop()
    }

    fn parallel() -> bool {
        true // GraphExecutor::parallel (executor.rs:110-112)
    }

    fn metrics(&self) -> &ExecutorMetrics {
        &self.metrics
    }

    fn monitor(&self) -> Option<&ExecutionOrderMonitor> {
        self.monitor.as_ref()
    }
}

#[cfg(test)]
mod tests {
    //! Needs a GPU (the handle is a real `fh_graph`): the two roles of one
    //! shard driven from two threads, as the runner's tokio tasks drive the
    //! clones (run/task/executor.rs:33-48).
    use super::*;
    use fantoch::id::Rifl;
    use fantoch::kvs::KVOp;
    use fantoch::time::RunTime;
    use std::thread;

    #[test]
    fn two_roles_from_two_threads() {
        let mut config = Config::new(3, 1);
        config.set_shard_count(2);
        let mut main = HipGraphExecutor::new(1, 0, config);
        let mut secondary = main.clone();
        secondary.set_executor_index(1);
        let n = 2000u64;
        let adder = thread::spawn(move || {
            let time = RunTime;
            for seq in 1..=n {
                let dot = Dot::new(1, seq);
                let key = format!("k{}", seq % 7);
                let cmd = Command::from(Rifl::new(1, seq), vec![(key, KVOp::Put(String::new()))]);
                // each command depends on the previous one: a chain
                let deps = if seq > 1 {
                    let mut s = HashSet::new();
                    s.insert(Dependency { dot: Dot::new(1, seq - 1), shards: Some(
                        std::iter::once(0u64).collect()) });
                    s
                } else {
                    HashSet::new()
                };
                main.handle(GraphExecutionInfo::Add { dot, cmd, deps }, &time);
            }
            let mut results = 0usize;
            while main.to_clients().is_some() {
                results += 1;
            }
            results
        });
        let answerer = thread::spawn(move || {
            let time = RunTime;
            for i in 0..n {
                // requests from the other shard for dots this shard holds or
                // will hold; answered (Info / Executed) or buffered
                let dots = std::iter::once(Dot::new(1, 1 + i % n)).collect();
                secondary.handle(GraphExecutionInfo::Request { from: 1, dots }, &time);
                secondary.cleanup(&time);
                // the secondary role never executes commands
                assert!(secondary.to_clients().is_none());
            }
        });
        // every command executed exactly once, all by the main role
        assert_eq!(adder.join().unwrap(), n as usize);
        answerer.join().unwrap();
    }
}
