"""HipKeyDeps -- the KeyDeps trait backed by the HIP engine.

Mirrors fantoch_ps/src/protocol/common/graph/deps/keys/mod.rs:37-63:

    KeyDeps::new(shard_id)                     -> HipKeyDeps(shard_id, ...)
    add_cmd(dot, &cmd, past) -> HashSet<Dep>   -> add_cmd(dot, cmd, past)
    add_noop(dot) -> HashSet<Dep>              -> add_noop(dot)
    cmd_deps(&cmd) / noop_deps() (test-only)   -> cmd_deps(cmd) / noop_deps()
    parallel() -> bool                         -> parallel()  (SequentialKeyDeps: False;
                                                  LockedKeyDeps, read_write=True: True)

plus the batched form the engine is built for, add_batch(), which computes a
whole arrival-ordered batch of add_cmd/add_noop calls in one device pass.

Results are sets of packed dots.  `Dependency.shards` (keys/mod.rs:18-35) is a
function of the dependency's dot (the shard set of that command), so dot-set
equality is the parity contract; `dependencies()` rebuilds
full Dependency values from the shard sets of the dots the device state can
still return (the latest dot of each key slot and the latest noop, as the Rust
crate's HipKeyDeps keeps them, fantoch_hip/src/keydeps.rs), so the bookkeeping
is bounded by the keys like the reference's latest table
(keys/sequential.rs:7-12, locked.rs:10-15).

Like LockedKeyDeps (keys/locked.rs:17-22, `Clone` shares the state), one
instance may be used from several threads: every call holds the instance's
lock, so concurrent workers serialise on the device handle.
"""
from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass
from typing import FrozenSet, Iterable, Optional

import numpy as np

from . import _lib as L


@dataclass(frozen=True)
class Dependency:
    """Dependency{dot, shards} (deps/keys/mod.rs:18-35); shards None = noop."""
    dot: int
    shards: Optional[FrozenSet[int]]


class KeyInterner:
    """Key = String (fantoch/src/kvs.rs:6) -> dense id < key_space (no hashing,
    no collisions)."""

    def __init__(self, key_space: int):
        self.key_space = key_space
        self.ids = {}

    def __call__(self, key) -> int:
        i = self.ids.get(key)
        if i is None:
            i = len(self.ids)
            if i >= self.key_space:
                raise L.FhError(L.FH_EINVAL, f"more than key_space={self.key_space} keys")
            self.ids[key] = i
        return i

    def many(self, keys: Iterable) -> list:
        return [self(k) for k in keys]


def make_config(n=1, f=0, shard_count=1, device=-1, key_space=1 << 20) -> L.fh_config:
    return L.fh_config(n=n, f=f, shard_count=shard_count, device=device, key_space=key_space)


class HipKeyDeps:
    """KeyDeps implementation over fh_keydeps_* (include/fantoch_hip.h).

    read_write=False: SequentialKeyDeps (deps/keys/sequential.rs);
    read_write=True: LockedKeyDeps' read/write rules (deps/keys/locked.rs:
    83-169), with Command.read_only selecting the rule per command."""

    def __init__(self, shard_id: int = 0, key_space: int = 1 << 20, device: int = -1,
                 intern: bool = True, read_write: bool = False):
        self._lib = L.load()
        self.shard_id = shard_id
        self.read_write = read_write
        self.cfg = make_config(device=device, key_space=key_space)
        h = C.c_void_p()
        L.check(self._lib.fh_keydeps_create(shard_id, C.byref(self.cfg), C.byref(h)))
        self._h = h
        self.keys = KeyInterner(key_space) if intern else None
        self._lock = threading.RLock()
        # Dependency.shards of the dots a slot still holds: dot -> [shards,
        # slots holding it]; (key id, read slot) -> its latest dot; the
        # latest noop (fantoch_hip/src/keydeps.rs State)
        self._live = {}
        self._slots = {}
        self._noop = None
        # the shards of the deps the last add_cmd / add_noop returned, taken
        # before that call released the slots it replaced (the returned deps
        # are exactly the dots it displaced: fantoch_hip/src/keydeps.rs builds
        # its Dependency values before set_slot for the same reason)
        self._returned = {}

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fh_keydeps_destroy(self._h)
            self._h = None

    __del__ = close

    def parallel(self) -> bool:
        # SequentialKeyDeps::parallel is false (sequential.rs:60-62),
        # LockedKeyDeps::parallel true (locked.rs:70-72): the Rust crate's
        # HipKeyDeps / HipLockedKeyDeps (fantoch_hip/src/keydeps.rs)
        return self.read_write

    # -- helpers ---------------------------------------------------------
    def _key_ids(self, cmd):
        keys = cmd.keys(self.shard_id) if hasattr(cmd, "keys") else cmd
        return self.keys.many(keys) if self.keys is not None else [int(k) for k in keys]

    def _hold(self, dot, shards):
        e = self._live.get(dot)
        if e is None:
            self._live[dot] = [shards, 1]
        else:
            e[1] += 1

    def _release(self, dot):
        e = self._live.get(dot)
        if e is not None:
            e[1] -= 1
            if e[1] == 0:
                del self._live[dot]

    def _shards_of(self, d):
        e = self._live.get(d)
        if e is not None:
            return e[0]
        return self._returned.get(d)

    def dependencies(self, dots) -> set:
        """Dots -> Dependency values, shards from the live slots or from the
        last add_cmd / add_noop's returned deps (None when neither holds the
        dot any more, or for a noop)."""
        with self._lock:
            return {Dependency(d, self._shards_of(d)) for d in dots}

    def _snapshot(self, deps) -> set:
        out = set(int(x) for x in deps)
        self._returned = {d: self._live[d][0] for d in out if d in self._live}
        return out

    # -- KeyDeps ---------------------------------------------------------
    def add_cmd(self, dot: int, cmd, past: Optional[Iterable[int]] = None) -> set:
        past_l = None if past is None else [p.dot if isinstance(p, Dependency) else int(p)
                                            for p in past]
        read_only = bool(getattr(cmd, "read_only", False))
        ro = [read_only] if self.read_write else None
        with self._lock:
            kid = self._key_ids(cmd)
            off, deps = self.add_batch([dot], [kid], None,
                                       None if past_l is None else [past_l], read_only=ro)
            # the command becomes its keys' latest (the read slot for a
            # read-only command under LockedKeyDeps, locked.rs:100-117)
            shards = frozenset(cmd.shards()) if hasattr(cmd, "shards") else None
            slot_ro = self.read_write and read_only
            result = self._snapshot(deps[off[0]:off[1]])
            for k in kid:
                self._hold(dot, shards)
                old = self._slots.get((k, slot_ro))
                self._slots[(k, slot_ro)] = dot
                if old is not None:
                    self._release(old)
            return result

    def add_noop(self, dot: int) -> set:
        with self._lock:
            off, deps = self.add_batch([dot], [[]], [True], None,
                                       read_only=[False] if self.read_write else None)
            # the latest noop (sequential.rs:66-70); keys' slots are unchanged
            result = self._snapshot(deps[off[0]:off[1]])
            self._hold(dot, None)
            old, self._noop = self._noop, dot
            if old is not None:
                self._release(old)
            return result

    def cmd_deps(self, cmd) -> set:
        with self._lock:
            k = np.asarray(self._key_ids(cmd), dtype=np.uint64)
            cap = 2 * len(k) + 1
            out = np.zeros(cap, dtype=np.uint64)
            n = C.c_size_t(0)
            L.check(self._lib.fh_keydeps_cmd_deps(self._h, len(k), L.ptr(k), L.ptr(out), cap,
                                                  C.byref(n)))
            return set(int(x) for x in out[:n.value])

    def noop_deps(self) -> set:
        with self._lock:
            n = C.c_size_t(0)
            L.check(self._lib.fh_keydeps_noop_deps(self._h, None, 0, C.byref(n)))
            out = np.zeros(max(1, n.value), dtype=np.uint64)
            L.check(self._lib.fh_keydeps_noop_deps(self._h, L.ptr(out), len(out), C.byref(n)))
            return set(int(x) for x in out[:n.value])

    # -- batched form ------------------------------------------------------
    def add_batch(self, dots, keys, is_noop=None, past=None, read_only=None):
        """dots: sequence of packed dots; keys: per-command key-id lists (or a
        (key_off, key_ids) pair of arrays); is_noop: optional bools; past:
        optional per-command dot lists (None = no past for every command);
        read_only: optional bools -- LockedKeyDeps' read/write rules
        (fh_keydeps_add_batch_rw).  Returns (dep_off[n+1], dep_dots) as numpy
        arrays."""
        with self._lock:
            return self._add_batch(dots, keys, is_noop, past, read_only)

    def _add_batch(self, dots, keys, is_noop, past, read_only):
        n = len(dots)
        dot_a = np.ascontiguousarray(dots, dtype=np.uint64)
        if isinstance(keys, tuple):
            key_off = np.ascontiguousarray(keys[0], dtype=np.uint32)
            key_ids = np.ascontiguousarray(keys[1], dtype=np.uint64)
        else:
            key_off = np.zeros(n + 1, dtype=np.uint32)
            key_off[1:] = np.cumsum([len(k) for k in keys]) if n else []
            key_ids = np.asarray([k for ks in keys for k in ks], dtype=np.uint64)
        noop = None if is_noop is None else np.ascontiguousarray(is_noop, dtype=np.uint8)
        past_off = past_dot = None
        if past is not None:
            past_off = np.zeros(n + 1, dtype=np.uint32)
            past_off[1:] = np.cumsum([len(p) for p in past]) if n else []
            past_dot = np.asarray([x for p in past for x in p], dtype=np.uint64)
        out_off = np.zeros(n + 1, dtype=np.uint32)
        ro = None if read_only is None else np.ascontiguousarray(read_only, dtype=np.uint8)
        cap = int(len(key_ids) * (1 if ro is None else 2) + n +
                  (0 if past_dot is None else len(past_dot)) + 1)
        while True:
            out = np.zeros(cap, dtype=np.uint64)
            ln = C.c_size_t(0)
            kp = L.ptr(key_ids) if len(key_ids) else None
            pp = L.ptr(past_dot) if past_dot is not None and len(past_dot) else None
            if ro is None:
                st = self._lib.fh_keydeps_add_batch(
                    self._h, n, L.ptr(dot_a), L.ptr(key_off), kp, L.ptr(noop), L.ptr(past_off),
                    pp, L.ptr(out_off), L.ptr(out), cap, C.byref(ln))
            else:
                st = self._lib.fh_keydeps_add_batch_rw(
                    self._h, n, L.ptr(dot_a), L.ptr(key_off), kp, L.ptr(ro), L.ptr(noop),
                    L.ptr(past_off), pp, L.ptr(out_off), L.ptr(out), cap, C.byref(ln))
            if st == L.FH_ECAP:
                cap = int(ln.value)
                continue
            L.check(st)
            return out_off, out[:ln.value]
