"""HipPredecessorsExecutor -- Caesar's executor (PredecessorsExecutor) backed
by the HIP engine (fh_pred_*).

Mirrors fantoch/src/executor/mod.rs:27-88 and
fantoch_ps/src/executor/pred/executor.rs + mod.rs:26-352:

    Executor::new(process_id, shard_id, config)  -> HipPredecessorsExecutor(process_id, shard_id)
    handle(PredecessorsExecutionInfo{dot, cmd, clock, deps})
                                                 -> handle(PredecessorsExecutionInfo(dot, cmd, clock, deps))
    to_clients() -> Option<ExecutorResult>       -> to_clients() -> (rifl, key) | None
    monitor()                                    -> monitor() -> {key: [rifl, ...]}

handle_batch() takes a whole arrival-ordered batch in one device pass.  A
command runs once its deps are committed and its lower-clock deps have run
(mod.rs:132-253); ready commands run in clock order.  Clocks are
Clock{seq, process_id} (protocol/common/pred/clocks/mod.rs:27-30), given as
(seq, process_id) tuples or packed (seq << 8) | process_id.
"""
from __future__ import annotations

import ctypes as C
from collections import deque
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .keydeps import make_config


def pack_clock(clock) -> int:
    """Clock{seq, process_id} -> (seq << 8) | process_id (same order as Ord)."""
    if isinstance(clock, tuple):
        seq, pid = clock
        return (int(seq) << 8) | int(pid)
    return int(clock)


@dataclass
class PredecessorsExecutionInfo:
    """PredecessorsExecutionInfo (executor/pred/executor.rs)."""
    dot: int
    cmd: object
    clock: object
    deps: object


class HipPredecessorsExecutor:
    def __init__(self, process_id: int, shard_id: int = 0, n: int = 1, f: int = 0,
                 shard_count: int = 1, device: int = -1, monitor: bool = True):
        self._lib = L.load()
        self.process_id, self.shard_id = process_id, shard_id
        self.cfg = make_config(n=n, f=f, shard_count=shard_count, device=device)
        h = C.c_void_p()
        L.check(self._lib.fh_pred_create(process_id, shard_id, C.byref(self.cfg), C.byref(h)))
        self._h = h
        self._cmds = {}  # dot -> (command, keys), until executed
        self._to_clients = deque()
        self._monitor = {} if monitor else None

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fh_pred_destroy(self._h)
            self._h = None

    __del__ = close

    @staticmethod
    def parallel() -> bool:
        return False  # PredecessorsExecutor::parallel (executor.rs)

    def _keys_of(self, cmd):
        if cmd is None:
            return []
        return list(cmd.keys(self.shard_id)) if hasattr(cmd, "keys") else list(cmd)

    def handle(self, info: PredecessorsExecutionInfo):
        self.handle_batch([info])

    def handle_batch(self, infos):
        n = len(infos)
        dots = np.zeros(n, dtype=np.uint64)
        clocks = np.zeros(n, dtype=np.uint64)
        dep_off = np.zeros(n + 1, dtype=np.uint32)
        deps = []
        for i, info in enumerate(infos):
            dots[i] = info.dot
            clocks[i] = pack_clock(info.clock)
            deps.extend(int(d) for d in info.deps)
            dep_off[i + 1] = len(deps)
        dep_a = np.asarray(deps, dtype=np.uint64)
        L.check(self._lib.fh_pred_add_batch(self._h, n, L.ptr(dots), L.ptr(clocks),
                                            L.ptr(dep_off), L.ptr(dep_a) if len(dep_a) else None))
        for info in infos:
            self._cmds[int(info.dot)] = (info.cmd, self._keys_of(info.cmd))
        self._fetch()

    def _fetch(self):
        """command_to_execute + execute (executor.rs; mod.rs:71-73)."""
        buf = np.zeros(4096, dtype=np.uint64)
        while True:
            ln = C.c_size_t(0)
            L.check(self._lib.fh_pred_drain(self._h, L.ptr(buf), len(buf), C.byref(ln)))
            for i in range(ln.value):
                d = int(buf[i])
                cmd, ks = self._cmds.pop(d)
                rifl = getattr(cmd, "rifl", d)
                for k in ks:
                    self._to_clients.append((rifl, k))
                    if self._monitor is not None:
                        self._monitor.setdefault(k, []).append(rifl)
                self.executed_order = getattr(self, "executed_order", [])
                self.executed_order.append(d)
            if ln.value < len(buf):
                return

    def to_clients(self):
        return self._to_clients.popleft() if self._to_clients else None

    def monitor(self):
        return self._monitor

    def pending(self) -> int:
        c = C.c_size_t(0)
        L.check(self._lib.fh_pred_pending(self._h, C.byref(c)))
        return c.value
