"""HipKeyClocks -- Caesar's KeyClocks trait on the HIP engine (fh_keyclocks_*).

Mirrors fantoch_ps/src/protocol/common/pred/clocks/keys/mod.rs:13-45
(SequentialKeyClocks, keys/sequential.rs:14-152): new(process_id, shard_id),
clock_next, clock_join, add, remove, predecessors(dot, cmd, clock, higher).
Keys are interned to dense ids (Key = String); clocks are packed
(seq << 8) | process_id.  Batch entry points take many commands per call.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .keydeps import KeyInterner, make_config


def clock(seq: int, pid: int) -> int:
    return (seq << 8) | pid


class HipKeyClocks:
    def __init__(self, process_id: int, shard_id: int = 0, key_space: int = 1 << 20,
                 device: int = -1):
        self._lib = L.load()
        self.shard_id = shard_id
        self.cfg = make_config(n=0, f=0, device=device, key_space=key_space)
        h = C.c_void_p()
        L.check(self._lib.fh_keyclocks_create(process_id, shard_id, C.byref(self.cfg), C.byref(h)))
        self._h = h
        self.keys = KeyInterner(key_space)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fh_keyclocks_destroy(self._h)
            self._h = None

    __del__ = close

    @staticmethod
    def parallel() -> bool:
        return False  # SequentialKeyClocks::parallel

    def clock_next(self) -> int:
        c = C.c_uint64(0)
        L.check(self._lib.fh_keyclocks_clock_next(self._h, C.byref(c)))
        return c.value

    def clock_join(self, other: int):
        L.check(self._lib.fh_keyclocks_clock_join(self._h, other))

    def _arrays(self, keys_list, ids=False):
        off = np.zeros(len(keys_list) + 1, dtype=np.uint32)
        flat = []
        for i, ks in enumerate(keys_list):
            flat.extend(int(k) if ids else self.keys(k) for k in ks)
            off[i + 1] = len(flat)
        return off, np.asarray(flat, dtype=np.uint64)

    def add_batch(self, dots, keys_list, clocks, ids=False):
        off, k = self._arrays(keys_list, ids)
        d = np.asarray(dots, dtype=np.uint64)
        c = np.asarray(clocks, dtype=np.uint64)
        L.check(self._lib.fh_keyclocks_add(self._h, len(d), L.ptr(d), L.ptr(off),
                                           L.ptr(k) if len(k) else None, L.ptr(c)))

    def remove_batch(self, keys_list, clocks, ids=False):
        off, k = self._arrays(keys_list, ids)
        c = np.asarray(clocks, dtype=np.uint64)
        L.check(self._lib.fh_keyclocks_remove(self._h, len(c), L.ptr(off),
                                              L.ptr(k) if len(k) else None, L.ptr(c)))

    def predecessors_batch(self, dots, keys_list, clocks, higher=False, ids=False):
        """-> (pred_off, pred_dots) or ((pred_off, pred_dots), (hi_off, hi_dots));
        each command's dots in ascending clock order."""
        off, k = self._arrays(keys_list, ids)
        d = np.asarray(dots, dtype=np.uint64)
        c = np.asarray(clocks, dtype=np.uint64)
        n = len(d)
        po, ho = np.zeros(n + 1, dtype=np.uint32), np.zeros(n + 1, dtype=np.uint32)
        pl, hl = C.c_size_t(0), C.c_size_t(0)
        args = (self._h, n, L.ptr(d), L.ptr(off), L.ptr(k) if len(k) else None, L.ptr(c))
        hi_args = (L.ptr(ho), None, 0, C.byref(hl)) if higher else (None, None, 0, None)
        st = self._lib.fh_keyclocks_predecessors(*args, L.ptr(po), None, 0, C.byref(pl), *hi_args)
        L.check(st)
        pd = np.zeros(max(1, pl.value), dtype=np.uint64)
        hd = np.zeros(max(1, hl.value), dtype=np.uint64)
        hi_args = (L.ptr(ho), L.ptr(hd), hl.value, C.byref(hl)) if higher else (None, None, 0, None)
        L.check(self._lib.fh_keyclocks_predecessors(*args, L.ptr(po), L.ptr(pd), pl.value,
                                                    C.byref(pl), *hi_args))
        if higher:
            return (po, pd[:pl.value]), (ho, hd[:hl.value])
        return po, pd[:pl.value]

    # KeyClocks trait, one command at a time (keys/mod.rs:13-45)
    def add(self, dot, keys, clk):
        self.add_batch([dot], [list(keys)], [clk])

    def remove(self, keys, clk):
        self.remove_batch([list(keys)], [clk])

    def predecessors(self, dot, keys, clk, higher=None):
        if higher is None:
            po, pd = self.predecessors_batch([dot], [list(keys)], [clk])
            return set(int(x) for x in pd)
        (po, pd), (ho, hd) = self.predecessors_batch([dot], [list(keys)], [clk], higher=True)
        higher.update(int(x) for x in hd)
        return set(int(x) for x in pd)

    def __len__(self):
        n = C.c_size_t(0)
        L.check(self._lib.fh_keyclocks_len(self._h, C.byref(n)))
        return n.value
