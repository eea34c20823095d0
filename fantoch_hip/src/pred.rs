//! `Executor` with Caesar's `PredecessorsExecutor` semantics
//! (fantoch_ps/src/executor/pred/executor.rs, PredecessorsGraph mod.rs:26-352)
//! on `fh_pred_*`: a command runs once every dependency is committed and
//! every dependency with a lower clock has run; ready commands in clock order.
//!
//! Needs two accessors the reference keeps private: `Clock::{seq,
//! process_id}` (protocol/common/pred/clocks/mod.rs:27-30) and the fields of
//! `PredecessorsExecutionInfo` (executor/pred/executor.rs:103-108) -- one-line
//! `pub fn`s each.
use crate::{check, ffi, pack, unpack};
use fantoch::command::Command;
use fantoch::config::Config;
use fantoch::executor::{ExecutionOrderMonitor, Executor, ExecutorMetrics, ExecutorResult};
use fantoch::id::{Dot, ProcessId, ShardId};
use fantoch::kvs::KVStore;
use fantoch::protocol::Executed;
use fantoch::time::SysTime;
use fantoch::HashMap;
use fantoch_ps::executor::PredecessorsExecutionInfo;
use std::collections::VecDeque;
use std::ptr::null_mut;
use std::sync::{Arc, Mutex};

struct Handle(*mut ffi::FhPred);
unsafe impl Send for Handle {}
unsafe impl Sync for Handle {}
impl Drop for Handle {
    fn drop(&mut self) {
        unsafe {
            ffi::fh_pred_destroy(self.0);
        }
    }
}

#[derive(Clone)]
pub struct HipPredecessorsExecutor {
    process_id: ProcessId,
    shard_id: ShardId,
    config: Config,
    handle: Arc<Mutex<Handle>>,
    cmds: HashMap<Dot, Command>,
    executed: Executed,
    store: KVStore,
    monitor: Option<ExecutionOrderMonitor>,
    metrics: ExecutorMetrics,
    to_clients: VecDeque<ExecutorResult>,
}

impl HipPredecessorsExecutor {
    fn execute(&mut self, cmd: Command) {
        let results = cmd.execute(self.shard_id, &mut self.store, &mut self.monitor);
        self.to_clients.extend(results);
    }
}

impl Executor for HipPredecessorsExecutor {
    type ExecutionInfo = PredecessorsExecutionInfo;

    fn new(process_id: ProcessId, shard_id: ShardId, config: Config) -> Self {
        let cfg = crate::config(config.n(), config.f(), config.shard_count());
        let mut h = null_mut();
        check(unsafe { ffi::fh_pred_create(process_id as u32, shard_id, &cfg, &mut h) });
        let ids = fantoch::util::all_process_ids(config.shard_count(), config.n())
            .map(|(id, _)| id);
        let monitor = if config.executor_monitor_execution_order() {
            Some(ExecutionOrderMonitor::new())
        } else {
            None
        };
        Self {
            process_id,
            shard_id,
            config,
            handle: Arc::new(Mutex::new(Handle(h))),
            cmds: HashMap::new(),
            executed: Executed::with(ids),
            store: KVStore::new(),
            monitor,
            metrics: ExecutorMetrics::new(),
            to_clients: VecDeque::new(),
        }
    }

    /// handle (executor/pred/executor.rs:51-68) -> PredecessorsGraph::add
    /// (mod.rs:89-130) as a batch of one, then command_to_execute
    fn handle(&mut self, info: PredecessorsExecutionInfo, _time: &dyn SysTime) {
        let (dot, cmd, clock, deps) = (info.dot(), info.cmd().clone(), info.clock(), info.deps());
        if self.config.execute_at_commit() {
            return self.execute(cmd);
        }
        // Clock's Ord is (seq, process_id): packed (seq << 8) | process_id
        let c = [(clock.seq() << 8) | clock.process_id() as u64];
        let d = [pack(dot)];
        let dep: Vec<u64> = deps.iter().map(|x| pack(*x)).collect();
        let off = [0u32, dep.len() as u32];
        self.cmds.insert(dot, cmd);
        let h = self.handle.lock().unwrap().0;
        check(unsafe {
            ffi::fh_pred_add_batch(h, 1, d.as_ptr(), c.as_ptr(), off.as_ptr(), dep.as_ptr())
        });
        let len = crate::sized(|cap, len| unsafe { ffi::fh_pred_drain(h, null_mut(), cap, len) });
        let mut ready = vec![0u64; len];
        let mut got = 0usize;
        check(unsafe { ffi::fh_pred_drain(h, ready.as_mut_ptr(), len, &mut got) });
        for x in ready.into_iter().take(got) {
            let dot = unpack(x);
            self.executed.add(&dot.source(), dot.sequence());
            let cmd = self.cmds.remove(&dot).expect("drained dot has a command");
            self.execute(cmd);
        }
    }

    fn to_clients(&mut self) -> Option<ExecutorResult> {
        self.to_clients.pop_front()
    }

    /// the executed clock, for Caesar's GC (executor/pred/executor.rs:75-77)
    fn executed(&mut self, _time: &dyn SysTime) -> Option<Executed> {
        Some(self.executed.clone())
    }

    fn parallel() -> bool {
        false
    }

    fn metrics(&self) -> &ExecutorMetrics {
        &self.metrics
    }

    fn monitor(&self) -> Option<&ExecutionOrderMonitor> {
        self.monitor.as_ref()
    }
}
