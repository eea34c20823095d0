"""Seeded synthetic command streams (fh_workload_*, see csrc/workload.cpp).

Mirrors the knobs of fantoch's client Workload + KeyGen
(fantoch/src/client/workload.rs:11-61, key_gen.rs:10-19) for the BASELINE.json
configurations.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L

ZIPF, CONFLICT_RATE, CONFLICT_POOL = 0, 1, 2


@dataclass
class Stream:
    dots: np.ndarray          # u64[n]
    keys: np.ndarray          # u64[n, k]
    fq_proc: np.ndarray       # u8[n, views] (partial replication: [n, k, views]) or None
    fq_time: np.ndarray       # u64, shaped as fq_proc, or None
    key_space: int
    # replica views as per-replica arrival logs (fh_engine_stage_logs layout):
    # log_off u64[nproc+1], log_cmd u32[n*views]; None if not generated
    log_off: np.ndarray = None
    log_cmd: np.ndarray = None
    views_n: int = 0          # fast-quorum size when only the logs are held
    # element logs (FH_STREAM_ELEMENT_LOGS): log_off u64[n_proc*shards+1],
    # log_elem u32[n*k*views] positions (c*views + j)*k + s
    log_elem: np.ndarray = None
    shards: int = 1           # partial replication over `shards` key shards
    nproc: int = 5            # processes per shard

    @property
    def n(self):
        return len(self.dots)

    @property
    def k(self):
        return self.keys.shape[1]

    @property
    def views(self):
        if self.fq_proc is not None:
            return self.fq_proc.shape[-1]
        return self.views_n

    def shard_views(self, shard: int):
        """Partial replication: shard `shard`'s part of the stream -- the
        commands with a key on it (global indices), their keys on it
        (key_off CSR + keys, Command::keys(shard), command.rs:95-100) and the
        views of the shard's collect (fq_proc / fq_time [m, views])."""
        assert self.fq_proc is not None and self.fq_proc.ndim == 3, "needs per-slot views"
        on = self.keys % np.uint64(self.shards) == np.uint64(shard)
        cnt = on.sum(axis=1)
        cmds = np.nonzero(cnt)[0]
        key_off = np.zeros(len(cmds) + 1, dtype=np.uint32)
        np.cumsum(cnt[cmds], out=key_off[1:])
        slot = np.argmax(on[cmds], axis=1)  # first slot on the shard: its views
        return (cmds, key_off, self.keys[cmds][on[cmds]], self.fq_proc[cmds, slot],
                self.fq_time[cmds, slot])

    def key_off(self):
        return (np.arange(self.n + 1, dtype=np.uint64) * self.k).astype(np.uint32)


@dataclass
class Workload:
    seed: int = 0xFA170C4000000000
    n: int = 5                  # processes (dot sources 1..n)
    keys_per_cmd: int = 1
    kind: int = ZIPF
    conflict_rate: int = 0
    pool_size: int = 0
    clients: int = 1024
    zipf_s: float = 0.7
    key_count: int = 1 << 20
    views: int = 0              # fast quorum size (0 = single view)
    window: int = 64            # reorder window W
    shards: int = 1             # >= 2: partial replication (include/fantoch_hip.h fh_workload)

    @classmethod
    def zipf(cls, s, key_count, k=1, **kw):
        return cls(kind=ZIPF, zipf_s=s, key_count=key_count, keys_per_cmd=k, **kw)

    @classmethod
    def conflict_rate_(cls, rate, k=1, **kw):
        return cls(kind=CONFLICT_RATE, conflict_rate=rate, keys_per_cmd=k, **kw)

    @classmethod
    def conflict_pool(cls, rate, pool, k=2, **kw):
        return cls(kind=CONFLICT_POOL, conflict_rate=rate, pool_size=pool, keys_per_cmd=k, **kw)

    def _c(self) -> L.fh_workload:
        return L.fh_workload(seed=self.seed, n=self.n, keys_per_cmd=self.keys_per_cmd,
                             kind=self.kind, conflict_rate=self.conflict_rate,
                             pool_size=self.pool_size, clients=self.clients, zipf_s=self.zipf_s,
                             key_count=self.key_count, views=self.views, window=self.window,
                             shards=self.shards)

    def key_space(self) -> int:
        w = self._c()
        return int(L.load().fh_workload_key_space(C.byref(w)))

    def generate(self, count: int, first: int = 0, logs: bool = False,
                 times: bool = True, element_logs: bool = None) -> Stream:
        """Commands [first, first + count).  With views: fq_proc / fq_time if
        `times` (per key slot under partial replication), the per-replica
        arrival logs if `logs` (the same arrivals): command logs, or element
        logs (fh_workload_generate_element_logs) for a partially replicated
        stream or with `element_logs`."""
        lib = L.load()
        w = self._c()
        sh = max(1, self.shards)
        dots = np.zeros(count, dtype=np.uint64)
        keys = np.zeros((count, self.keys_per_cmd), dtype=np.uint64)
        fq_proc = fq_time = None
        if self.views and times:
            shape = (count, self.views) if sh == 1 else (count, self.keys_per_cmd, self.views)
            fq_proc = np.zeros(shape, dtype=np.uint8)
            fq_time = np.zeros(shape, dtype=np.uint64)
        L.check(lib.fh_workload_generate(C.byref(w), first, count, L.ptr(dots), L.ptr(keys),
                                         L.ptr(fq_proc), L.ptr(fq_time)))
        s = Stream(dots, keys, fq_proc, fq_time, self.key_space(), views_n=self.views, shards=sh,
                   nproc=self.n)
        if self.views and logs:
            if element_logs is None:
                element_logs = sh > 1
            if element_logs:
                s.log_off = np.zeros(self.n * sh + 1, dtype=np.uint64)
                s.log_elem = np.zeros(max(1, count * self.keys_per_cmd * self.views),
                                      dtype=np.uint32)
                L.check(lib.fh_workload_generate_element_logs(C.byref(w), first, count,
                                                              L.ptr(s.log_off), L.ptr(s.log_elem)))
                s.log_elem = s.log_elem[:count * self.keys_per_cmd * self.views]
            else:
                s.log_off = np.zeros(self.n + 1, dtype=np.uint64)
                s.log_cmd = np.zeros(count * self.views, dtype=np.uint32)
                L.check(lib.fh_workload_generate_logs(C.byref(w), first, count, L.ptr(s.log_off),
                                                      L.ptr(s.log_cmd)))
        return s

    def key_histogram(self, count: int, first: int = 0) -> np.ndarray:
        """u64[key_space]: commands of [first, first + count) per first key
        (fh_workload_key_histogram)."""
        lib = L.load()
        w = self._c()
        h = np.zeros(self.key_space(), dtype=np.uint64)
        L.check(lib.fh_workload_key_histogram(C.byref(w), first, count, L.ptr(h)))
        return h

    def generate_shard(self, count: int, nshards: int, shard: int, first: int = 0,
                       logs: bool = True, owner: np.ndarray = None) -> Stream:
        """Key shard `shard` of `nshards` of commands [first, first + count):
        the commands whose first key k0 has owner[k0] == shard (`owner` from
        key_owners_balanced; None = k0 % nshards), global dots, with the
        replicas' logs restricted to it (fh_workload_generate_shard_owned)."""
        lib = L.load()
        w = self._c()
        n = C.c_size_t(0)
        if owner is not None:
            owner = np.ascontiguousarray(owner, dtype=np.uint32)
            assert len(owner) == self.key_space()
        L.check(lib.fh_workload_generate_shard_owned(C.byref(w), first, count, L.ptr(owner),
                                                     nshards, shard, C.byref(n), None, None,
                                                     None, None))
        m = n.value
        dots = np.zeros(m, dtype=np.uint64)
        keys = np.zeros((m, self.keys_per_cmd), dtype=np.uint64)
        lo = lc = None
        if self.views and logs:
            lo = np.zeros(self.n + 1, dtype=np.uint64)
            lc = np.zeros(max(1, m * self.views), dtype=np.uint32)
        L.check(lib.fh_workload_generate_shard_owned(C.byref(w), first, count, L.ptr(owner),
                                                     nshards, shard, C.byref(n), L.ptr(dots),
                                                     L.ptr(keys), L.ptr(lo), L.ptr(lc)))
        s = Stream(dots, keys, None, None, self.key_space(), views_n=self.views)
        if lo is not None:
            s.log_off, s.log_cmd = lo, lc[:m * self.views]
        return s


# Per-command cost of a key relative to a cold one, as a function of the
# key's share of the stream: a hot key's commands scan more same-key
# neighbours in the KeyDeps search and form larger ready groups in the tile
# kernel.  Measured on the C4 stream's 8 balanced shards (12.5M commands
# each, tools/shard_probe.py, profiles/r06_shards_balanced.jsonl): shards
# whose hottest key holds 0.8-2.2M commands run 1.62-1.70 ms, 3.3M 1.78 ms,
# 6.5M (the stream's hottest key, 6.5 % of it) 2.25 ms -- about 1.7x per
# command for that key, 1.35x for the 3.3 % one: 1 + 10.8 x share.
HOT_KEY_COST = 14.0


def key_weights(hist: np.ndarray) -> np.ndarray:
    """Per-key work estimates for the key map: the command count times
    1 + HOT_KEY_COST x the key's share of the stream (x16, integral)."""
    h = np.asarray(hist, dtype=np.float64)
    tot = max(1.0, h.sum())
    return np.rint(16.0 * h * (1.0 + HOT_KEY_COST * h / tot)).astype(np.uint64)


def key_owners_weighted(hist: np.ndarray, nshards: int) -> np.ndarray:
    """key_owners_balanced over key_weights(hist): balances the estimated
    work per shard instead of the command count (the shard holding the
    hottest key gets fewer commands)."""
    return key_owners_balanced(key_weights(hist), nshards)


def key_owners_balanced(hist: np.ndarray, nshards: int) -> np.ndarray:
    """u32[key_space] key -> shard map balancing the per-key command counts
    `hist` over `nshards` (fh_key_owners_balanced: greedy largest-first
    packing; deterministic, so every rank computes the same map)."""
    hist = np.ascontiguousarray(hist, dtype=np.uint64)
    owner = np.zeros(len(hist), dtype=np.uint32)
    L.check(L.load().fh_key_owners_balanced(L.ptr(hist), len(hist), nshards, L.ptr(owner)))
    return owner
