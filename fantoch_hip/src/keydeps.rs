//! `KeyDeps` (fantoch_ps/src/protocol/common/graph/deps/keys/mod.rs:37-63) on
//! the HIP engine: `fh_keydeps_*`.
use crate::{check, ffi, pack, unpack, Interner};
use fantoch::command::Command;
use fantoch::id::{Dot, ShardId};
use fantoch::HashSet;
use fantoch_ps::protocol::common::graph::{Dependency, KeyDeps};
use std::collections::BTreeSet;
use std::fmt;
use std::ptr::{null, null_mut};
use std::sync::{Arc, Mutex};

struct Handle(*mut ffi::FhKeyDeps);
unsafe impl Send for Handle {}
unsafe impl Sync for Handle {}
impl Drop for Handle {
    fn drop(&mut self) {
        unsafe {
            ffi::fh_keydeps_destroy(self.0);
        }
    }
}

type Shards = Option<BTreeSet<ShardId>>;

struct State {
    h: Handle,
    keys: Interner,
    // Dependency::shards (a function of the dot: the command's shard set, or
    // None for a noop, deps/keys/mod.rs:24-35) of the dots the device state
    // can still return -- the latest dot of each (key, read/write) slot and
    // the latest noop -- with the number of slots holding each.  A dot leaves
    // when no slot holds it, so the map is bounded by the keys, as the
    // reference's latest table is (keys/sequential.rs:7-12, locked.rs:10-15).
    live: fantoch::HashMap<Dot, (Shards, u32)>,
    slots: fantoch::HashMap<(u64, bool), Dot>, // (key id, read slot) -> latest dot
    noop: Option<Dot>,
}

impl State {
    fn hold(&mut self, dot: Dot, shards: &Shards) {
        self.live.entry(dot).or_insert_with(|| (shards.clone(), 0)).1 += 1;
    }

    fn release(&mut self, dot: Dot) {
        if let Some(e) = self.live.get_mut(&dot) {
            e.1 -= 1;
            if e.1 == 0 {
                self.live.remove(&dot);
            }
        }
    }

    fn set_slot(&mut self, slot: (u64, bool), dot: Dot, shards: &Shards) {
        self.hold(dot, shards);
        if let Some(old) = self.slots.insert(slot, dot) {
            self.release(old);
        }
    }
}

/// `SequentialKeyDeps` (keys/sequential.rs:7-144) on the device.  `Clone`
/// shares the device state, like `LockedKeyDeps` (keys/locked.rs:17-22).
#[derive(Clone)]
pub struct HipKeyDeps {
    shard_id: ShardId,
    read_write: bool,
    inner: Arc<Mutex<State>>,
}

impl fmt::Debug for HipKeyDeps {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "HipKeyDeps(shard {})", self.shard_id)
    }
}

impl HipKeyDeps {
    fn create(shard_id: ShardId, read_write: bool) -> Self {
        let cfg = crate::config(0, 0, 1);
        let mut h = null_mut();
        check(unsafe { ffi::fh_keydeps_create(shard_id, &cfg, &mut h) });
        let state = State {
            h: Handle(h),
            keys: Interner::default(),
            live: Default::default(),
            slots: Default::default(),
            noop: None,
        };
        Self {
            shard_id,
            read_write,
            inner: Arc::new(Mutex::new(state)),
        }
    }

    /// One add_cmd / add_noop as a batch of one (the batch entry takes any
    /// number of arrival-ordered calls; the protocols call one at a time).
    fn call(&self, st: &mut State, dot: Dot, keys: &[u64], read_only: bool, noop: bool,
            past: Option<&[u64]>) -> Vec<u64> {
        let d = [pack(dot)];
        let key_off = [0u32, keys.len() as u32];
        let is_noop = [noop as u8];
        let ro = [read_only as u8];
        let (p_off, p_dot): (Vec<u32>, &[u64]) = match past {
            Some(p) => (vec![0, p.len() as u32], p),
            None => (vec![], &[]),
        };
        let mut cap = if self.read_write { 2 } else { 1 } * keys.len() + p_dot.len() + 1;
        loop {
            let mut out_off = [0u32; 2];
            let mut out = vec![0u64; cap.max(1)];
            let mut len = 0usize;
            let status = unsafe {
                let past_off = if past.is_some() { p_off.as_ptr() } else { null() };
                if self.read_write {
                    ffi::fh_keydeps_add_batch_rw(st.h.0, 1, d.as_ptr(), key_off.as_ptr(),
                        keys.as_ptr(), ro.as_ptr(), is_noop.as_ptr(), past_off, p_dot.as_ptr(),
                        out_off.as_mut_ptr(), out.as_mut_ptr(), cap, &mut len)
                } else {
                    ffi::fh_keydeps_add_batch(st.h.0, 1, d.as_ptr(), key_off.as_ptr(),
                        keys.as_ptr(), is_noop.as_ptr(), past_off, p_dot.as_ptr(),
                        out_off.as_mut_ptr(), out.as_mut_ptr(), cap, &mut len)
                }
            };
            if status == ffi::FH_ECAP {
                cap = len; // a noop depends on every key seen: retry with the bound
                continue;
            }
            check(status);
            out.truncate(len);
            return out;
        }
    }

    /// Output dots -> Dependency: shards from the live slots, or from the
    /// call's `past` (deps the caller handed in, returned in this call only).
    fn to_deps(st: &State, past: &fantoch::HashMap<Dot, Shards>, dots: Vec<u64>)
        -> HashSet<Dependency> {
        dots.into_iter()
            .map(|x| {
                let dot = unpack(x);
                let shards = match st.live.get(&dot) {
                    Some((s, _)) => s.clone(),
                    None => past.get(&dot).cloned().unwrap_or(None),
                };
                Dependency { dot, shards }
            })
            .collect()
    }

    fn add(&mut self, dot: Dot, cmd: &Command, past: Option<HashSet<Dependency>>)
        -> HashSet<Dependency> {
        let mut st = self.inner.lock().unwrap();
        let keys: Vec<u64> = cmd.keys(self.shard_id).map(|k| st.keys.id(k)).collect();
        let mut past_shards = fantoch::HashMap::default();
        let past: Option<Vec<u64>> = past.map(|p| {
            p.into_iter()
                .map(|d| {
                    past_shards.insert(d.dot, d.shards);
                    pack(d.dot)
                })
                .collect()
        });
        let read_only = cmd.read_only();
        let out = self.call(&mut st, dot, &keys, read_only, false, past.as_deref());
        let deps = Self::to_deps(&st, &past_shards, out);
        // the command becomes its keys' latest (the read slot for a read-only
        // command under LockedKeyDeps, locked.rs:100-117; else the write slot)
        let shards: Shards = Some(cmd.shards().cloned().collect());
        let read_slot = self.read_write && read_only;
        for k in keys {
            st.set_slot((k, read_slot), dot, &shards);
        }
        deps
    }

    fn noop(&mut self, dot: Dot) -> HashSet<Dependency> {
        let mut st = self.inner.lock().unwrap();
        let out = self.call(&mut st, dot, &[], false, true, None);
        let deps = Self::to_deps(&st, &Default::default(), out);
        // the latest noop (sequential.rs:66-70); keys' slots are unchanged
        st.hold(dot, &None);
        if let Some(old) = st.noop.replace(dot) {
            st.release(old);
        }
        deps
    }

    /// KeyDeps::cmd_deps (keys/mod.rs:54-56; sequential.rs:44-50): latest
    /// noop + latest dot of each of the command's keys, no update.
    pub fn query_cmd_deps(&self, cmd: &Command) -> HashSet<Dot> {
        let st = self.inner.lock().unwrap();
        // keys never interned have no latest dot: leave them out
        let keys: Vec<u64> = cmd.keys(self.shard_id).filter_map(|k| st.keys.get(k)).collect();
        let mut cap = 2 * keys.len() + 1;
        loop {
            let mut out = vec![0u64; cap];
            let mut len = 0usize;
            let status = unsafe {
                ffi::fh_keydeps_cmd_deps(st.h.0, keys.len(), keys.as_ptr(), out.as_mut_ptr(),
                    cap, &mut len)
            };
            if status == ffi::FH_ECAP {
                cap = len;
                continue;
            }
            check(status);
            return out[..len].iter().map(|x| unpack(*x)).collect();
        }
    }

    /// KeyDeps::noop_deps (keys/mod.rs:58-60; sequential.rs:52-58).
    pub fn query_noop_deps(&self) -> HashSet<Dot> {
        let st = self.inner.lock().unwrap();
        let len = crate::sized(|cap, len| unsafe {
            ffi::fh_keydeps_noop_deps(st.h.0, null_mut(), cap, len)
        });
        let mut out = vec![0u64; len.max(1)];
        let mut got = 0usize;
        check(unsafe { ffi::fh_keydeps_noop_deps(st.h.0, out.as_mut_ptr(), len, &mut got) });
        out[..got].iter().map(|x| unpack(*x)).collect()
    }
}

impl KeyDeps for HipKeyDeps {
    fn new(shard_id: ShardId) -> Self {
        Self::create(shard_id, false)
    }

    fn add_cmd(&mut self, dot: Dot, cmd: &Command, past: Option<HashSet<Dependency>>)
        -> HashSet<Dependency> {
        self.add(dot, cmd, past)
    }

    fn add_noop(&mut self, dot: Dot) -> HashSet<Dependency> {
        self.noop(dot)
    }

    // cmd_deps / noop_deps are #[cfg(test)] items of the trait
    // (keys/mod.rs:54-60): they exist only while fantoch_ps compiles its own
    // unit tests, and those never see this crate (it depends on fantoch_ps,
    // not the other way round).  Implementing them here under this crate's
    // cfg(test) would name trait items that do not exist (E0407) in
    // `cargo test -p fantoch_hip`, so the queries are the inherent
    // `query_cmd_deps` / `query_noop_deps` instead.

    fn parallel() -> bool {
        false // SequentialKeyDeps::parallel (sequential.rs:60-62)
    }
}

impl HipLockedKeyDeps {
    /// KeyDeps::cmd_deps (keys/mod.rs:54-56) as an inherent method.
    pub fn query_cmd_deps(&self, cmd: &Command) -> HashSet<Dot> {
        self.0.query_cmd_deps(cmd)
    }

    /// KeyDeps::noop_deps (keys/mod.rs:58-60) as an inherent method.
    pub fn query_noop_deps(&self) -> HashSet<Dot> {
        self.0.query_noop_deps()
    }
}

/// `LockedKeyDeps` (keys/locked.rs:17-186): read/write-aware rules
/// (fh_keydeps_add_batch_rw), behind `AtlasLocked` / `EPaxosLocked`.
#[derive(Clone, Debug)]
pub struct HipLockedKeyDeps(HipKeyDeps);

impl KeyDeps for HipLockedKeyDeps {
    fn new(shard_id: ShardId) -> Self {
        Self(HipKeyDeps::create(shard_id, true))
    }

    fn add_cmd(&mut self, dot: Dot, cmd: &Command, past: Option<HashSet<Dependency>>)
        -> HashSet<Dependency> {
        self.0.add(dot, cmd, past)
    }

    fn add_noop(&mut self, dot: Dot) -> HashSet<Dependency> {
        self.0.noop(dot)
    }

    // (cmd_deps / noop_deps: see HipKeyDeps)

    // LockedKeyDeps::parallel() is true (locked.rs:70-72); the handle is
    // behind the Arc<Mutex>, so concurrent protocol workers serialise on it
    fn parallel() -> bool {
        true
    }
}
