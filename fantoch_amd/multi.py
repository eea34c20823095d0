"""MultiEngine -- the fused engine over several GPUs from one process
(fh_multi_*): one engine per device over key shards (owner from
fh_key_owners_balanced over the staged stream's per-key work estimates); see
include/fantoch_hip.h."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .keydeps import make_config


class MultiEngine:
    def __init__(self, key_space: int, devices, n: int = 5, f: int = 1):
        self._lib = L.load()
        self.key_space = key_space
        self.cfg = make_config(n=n, f=f, device=-1, key_space=key_space)
        devs = (C.c_int32 * len(devices))(*devices)
        h = C.c_void_p()
        L.check(self._lib.fh_multi_create(C.byref(self.cfg), len(devices), devs, C.byref(h)))
        self._h = h
        self.ndev = len(devices)
        self.n = 0

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fh_multi_destroy(self._h)
            self._h = None

    __del__ = close

    def stage(self, s, nproc: int = 5):
        """s: a Stream with per-replica logs (Workload.generate(logs=True))."""
        d = L.fh_stream_desc(n=s.n, keys_per_cmd=s.k, views=s.views, nproc=nproc, flags=0)
        dots = np.ascontiguousarray(s.dots, dtype=np.uint64)
        keys = np.ascontiguousarray(s.keys, dtype=np.uint64)
        off = np.ascontiguousarray(s.log_off, dtype=np.uint64)
        cmd = np.ascontiguousarray(s.log_cmd, dtype=np.uint32)
        L.check(self._lib.fh_multi_stage_logs(self._h, C.byref(d), L.ptr(dots), L.ptr(keys),
                                              L.ptr(off), L.ptr(cmd)))
        self.n = s.n

    def rewind(self):
        L.check(self._lib.fh_multi_rewind(self._h))

    def sync(self):
        L.check(self._lib.fh_multi_sync(self._h))

    def run(self, sync: bool = True) -> float:
        ms = C.c_float(0)
        L.check(self._lib.fh_multi_run(self._h, C.byref(ms) if sync else None))
        return float(ms.value)

    def shard_sizes(self):
        out = []
        for g in range(self.ndev):
            n = C.c_size_t(0)
            L.check(self._lib.fh_multi_shard_size(self._h, g, C.byref(n)))
            out.append(n.value)
        return out

    def owners(self) -> np.ndarray:
        """The key -> shard map of the last staging."""
        o = np.zeros(self.key_space, dtype=np.uint32)
        L.check(self._lib.fh_multi_owners(self._h, L.ptr(o)))
        return o

    def results(self):
        n = self.n
        dep_off = np.zeros(n + 1, dtype=np.uint32)
        key_off = np.zeros(self.key_space + 1, dtype=np.uint32)
        ln = C.c_size_t(0)
        L.check(self._lib.fh_multi_results(self._h, L.ptr(dep_off), None, 0, C.byref(ln), None,
                                           None, L.ptr(key_off), None))
        deps = np.zeros(max(1, ln.value), dtype=np.uint64)
        label = np.zeros(n, dtype=np.uint64)
        rank = np.zeros(n, dtype=np.uint32)
        key_seq = np.zeros(max(1, int(key_off[-1])), dtype=np.uint64)
        L.check(self._lib.fh_multi_results(self._h, L.ptr(dep_off), L.ptr(deps), len(deps),
                                           C.byref(ln), L.ptr(label), L.ptr(rank), L.ptr(key_off),
                                           L.ptr(key_seq)))
        return {"dep_off": dep_off, "deps": deps[:ln.value], "scc_label": label,
                "exec_rank": rank, "key_off": key_off, "key_seq": key_seq[:int(key_off[-1])]}
