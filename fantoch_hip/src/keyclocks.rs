//! Caesar's `KeyClocks` (fantoch_ps/src/protocol/common/pred/clocks/keys/
//! mod.rs:13-45, SequentialKeyClocks sequential.rs:14-152) on
//! `fh_keyclocks_*`.  Needs `Clock::{seq, process_id}` accessors (the
//! reference keeps the fields private, clocks/mod.rs:27-30) -- one-line
//! `pub fn`s.  Limit: commands of at most 8 keys (the device merge holds 8
//! key segments); a larger command gets `FH_ENOTIMPL`, which `check` turns
//! into a panic naming the limit.
use crate::{check, ffi, pack, unpack, Interner};
use fantoch::command::Command;
use fantoch::id::{Dot, ProcessId, ShardId};
use fantoch::HashSet;
use fantoch_ps::protocol::common::pred::{Clock, KeyClocks};
use std::fmt;
use std::ptr::null_mut;
use std::sync::{Arc, Mutex};

struct Handle(*mut ffi::FhKeyClocks);
unsafe impl Send for Handle {}
unsafe impl Sync for Handle {}
impl Drop for Handle {
    fn drop(&mut self) {
        unsafe {
            ffi::fh_keyclocks_destroy(self.0);
        }
    }
}

fn pack_clock(c: &Clock) -> u64 {
    (c.seq() << 8) | c.process_id() as u64
}

fn unpack_clock(x: u64) -> Clock {
    Clock::from(x >> 8, (x & 0xFF) as ProcessId)
}

/// `Clone` shares the device state.
#[derive(Clone)]
pub struct HipKeyClocks {
    shard_id: ShardId,
    inner: Arc<Mutex<(Handle, Interner)>>,
}

impl fmt::Debug for HipKeyClocks {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "HipKeyClocks(shard {})", self.shard_id)
    }
}

impl HipKeyClocks {
    fn keys(&self, g: &mut Interner, cmd: &Command) -> Vec<u64> {
        cmd.keys(self.shard_id).map(|k| g.id(k)).collect()
    }
}

impl KeyClocks for HipKeyClocks {
    fn new(process_id: ProcessId, shard_id: ShardId) -> Self {
        let cfg = crate::config(0, 0, 1);
        let mut h = null_mut();
        check(unsafe { ffi::fh_keyclocks_create(process_id as u32, shard_id, &cfg, &mut h) });
        Self { shard_id, inner: Arc::new(Mutex::new((Handle(h), Interner::default()))) }
    }

    fn clock_next(&mut self) -> Clock {
        let g = self.inner.lock().unwrap();
        let mut c = 0u64;
        check(unsafe { ffi::fh_keyclocks_clock_next((g.0).0, &mut c) });
        unpack_clock(c)
    }

    fn clock_join(&mut self, other: &Clock) {
        let g = self.inner.lock().unwrap();
        check(unsafe { ffi::fh_keyclocks_clock_join((g.0).0, pack_clock(other)) });
    }

    fn add(&mut self, dot: Dot, cmd: &Command, clock: Clock) {
        let mut g = self.inner.lock().unwrap();
        let keys = self.keys(&mut g.1, cmd);
        let off = [0u32, keys.len() as u32];
        let (d, c) = ([pack(dot)], [pack_clock(&clock)]);
        check(unsafe {
            ffi::fh_keyclocks_add((g.0).0, 1, d.as_ptr(), off.as_ptr(), keys.as_ptr(), c.as_ptr())
        });
    }

    fn remove(&mut self, cmd: &Command, clock: Clock) {
        let mut g = self.inner.lock().unwrap();
        let keys = self.keys(&mut g.1, cmd);
        let off = [0u32, keys.len() as u32];
        let c = [pack_clock(&clock)];
        check(unsafe {
            ffi::fh_keyclocks_remove((g.0).0, 1, off.as_ptr(), keys.as_ptr(), c.as_ptr())
        });
    }

    fn predecessors(&self, dot: Dot, cmd: &Command, clock: Clock,
                    higher: Option<&mut HashSet<Dot>>) -> HashSet<Dot> {
        let mut g = self.inner.lock().unwrap();
        let keys = self.keys(&mut g.1, cmd);
        let h = (g.0).0;
        let off = [0u32, keys.len() as u32];
        let (d, c) = ([pack(dot)], [pack_clock(&clock)]);
        let want_higher = higher.is_some();
        let (mut po, mut ho) = ([0u32; 2], [0u32; 2]);
        let (mut pl, mut hl) = (0usize, 0usize);
        // sizes first (FH_ECAP convention), then the dots
        let st = unsafe {
            ffi::fh_keyclocks_predecessors(h, 1, d.as_ptr(), off.as_ptr(), keys.as_ptr(),
                c.as_ptr(), po.as_mut_ptr(), null_mut(), 0, &mut pl,
                if want_higher { ho.as_mut_ptr() } else { null_mut() }, null_mut(), 0,
                if want_higher { &mut hl } else { null_mut() })
        };
        check(st);
        let (mut pd, mut hd) = (vec![0u64; pl.max(1)], vec![0u64; hl.max(1)]);
        check(unsafe {
            ffi::fh_keyclocks_predecessors(h, 1, d.as_ptr(), off.as_ptr(), keys.as_ptr(),
                c.as_ptr(), po.as_mut_ptr(), pd.as_mut_ptr(), pl, &mut pl,
                if want_higher { ho.as_mut_ptr() } else { null_mut() },
                if want_higher { hd.as_mut_ptr() } else { null_mut() }, hl,
                if want_higher { &mut hl } else { null_mut() })
        });
        if let Some(higher) = higher {
            higher.extend(hd[..hl].iter().map(|x| unpack(*x)));
        }
        pd[..pl].iter().map(|x| unpack(*x)).collect()
    }

    fn parallel() -> bool {
        false // SequentialKeyClocks::parallel
    }
}
