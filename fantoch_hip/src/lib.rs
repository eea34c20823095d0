//! fantoch_hip -- fantoch's dependency hot path on an MI355X.
//!
//! Drop-in implementations of the reference's plug-in traits, backed by the
//! HIP engine's C ABI (`include/fantoch_hip.h`, `libfantoch_hip.so`):
//!
//! * [`HipKeyDeps`] / [`HipLockedKeyDeps`] implement `KeyDeps`
//!   (fantoch_ps/src/protocol/common/graph/deps/keys/mod.rs:37-63), the
//!   generic parameter of `Atlas<KD>` / `EPaxos<KD>` (atlas.rs:28-31,
//!   epaxos.rs:27-29): `pub type AtlasHip = Atlas<fantoch_hip::HipKeyDeps>;`
//! * [`HipGraphExecutor`] implements `Executor` (fantoch/src/executor/mod.rs:
//!   27-88) with `GraphExecutor`'s semantics (fantoch_ps/src/executor/graph/
//!   executor.rs:19-197), accepting `GraphExecutionInfo` unchanged; Atlas /
//!   EPaxos select it with a one-line `type Executor` change (atlas.rs:45,
//!   epaxos.rs:42).
//! * [`HipPredecessorsExecutor`] implements `Executor` with Caesar's
//!   `PredecessorsExecutor` semantics (fantoch_ps/src/executor/pred/).
//! * [`engine::Engine`] is the batched, device-resident path the throughput
//!   metric is measured on (committed streams, replica views, replay).
//!
//! Not compiled in the engine repository (no cargo / rustc in its image);
//! the same boundary is exercised there through the ctypes mirror
//! `fantoch_amd/` by the GPU test suite.
pub mod engine;
pub mod executor;
pub mod ffi;
pub mod keyclocks;
pub mod keydeps;
pub mod pred;

pub use executor::HipGraphExecutor;
pub use keyclocks::HipKeyClocks;
pub use keydeps::{HipKeyDeps, HipLockedKeyDeps};
pub use pred::HipPredecessorsExecutor;

use fantoch::id::{Dot, ProcessId, ShardId};
use fantoch::kvs::Key;
use fantoch::HashMap;
use std::collections::BTreeSet;
use std::ffi::CStr;

/// Non-OK status -> panic!, as every invariant violation on this path does
/// in the reference (e.g. fantoch_ps/src/executor/graph/mod.rs:235-240).
pub(crate) fn check(st: ffi::FhStatus) {
    if st != ffi::FH_OK {
        let msg = unsafe { CStr::from_ptr(ffi::fh_last_error()) };
        panic!("fantoch_hip status {}: {}", st, msg.to_string_lossy());
    }
}

/// Dot -> packed u64: ProcessId in bits 56..63, sequence below; the packed
/// order is Id's derived Ord (fantoch/src/id.rs:21-27).
pub(crate) fn pack(dot: Dot) -> u64 {
    ((dot.source() as u64) << 56) | dot.sequence()
}

pub(crate) fn unpack(x: u64) -> Dot {
    Dot::new((x >> 56) as ProcessId, x & ((1u64 << 56) - 1))
}

/// Shard set <-> 64-bit mask (Dependency::shards, Command::shards()).
pub(crate) fn mask<'a>(shards: impl Iterator<Item = &'a ShardId>) -> u64 {
    shards.fold(0u64, |m, s| {
        assert!(*s < 64, "fantoch_hip: shard ids must be < 64");
        m | (1u64 << *s)
    })
}

pub(crate) fn unmask(m: u64) -> Option<BTreeSet<ShardId>> {
    if m == 0 {
        None // a noop's Dependency (deps/keys/mod.rs:32-34)
    } else {
        Some((0..64).filter(|s| (m >> s) & 1 == 1).collect())
    }
}

/// Key = String (fantoch/src/kvs.rs:6) -> dense id: interned, never hashed,
/// so ids cannot collide.
#[derive(Debug, Default)]
pub(crate) struct Interner {
    ids: HashMap<Key, u64>,
}

impl Interner {
    pub(crate) fn id(&mut self, key: &Key) -> u64 {
        let n = self.ids.len() as u64;
        *self.ids.entry(key.clone()).or_insert(n)
    }

    pub(crate) fn get(&self, key: &Key) -> Option<u64> {
        self.ids.get(key).copied()
    }
}

/// Interned key ids are < KEY_SPACE (fh_config::key_space <= 2^31).
pub(crate) const KEY_SPACE: u64 = 1 << 24;

/// Device selection per SURVEY §8b: -1 = env FANTOCH_HIP_DEVICE, else
/// shard_id % device count.
pub(crate) fn config(n: usize, f: usize, shard_count: usize) -> ffi::FhConfig {
    ffi::FhConfig {
        n: n as u32,
        f: f as u32,
        shard_count: shard_count as u32,
        device: -1,
        key_space: KEY_SPACE,
    }
}

/// Size-query-then-fill helper for the ABI's FH_ECAP convention.
pub(crate) fn sized<F>(mut call: F) -> usize
where
    F: FnMut(usize, &mut usize) -> ffi::FhStatus,
{
    let mut len = 0usize;
    let st = call(0, &mut len);
    if st != ffi::FH_ECAP {
        check(st);
    }
    len
}
