"""HipGraphExecutor -- the Executor trait with GraphExecutor semantics, backed
by the HIP engine (fh_graph_*).

Mirrors fantoch/src/executor/mod.rs:27-88 and
fantoch_ps/src/executor/graph/executor.rs:19-197:

    Executor::new(process_id, shard_id, config)   -> HipGraphExecutor(process_id, shard_id, n, f)
    handle(GraphExecutionInfo::Add{dot,cmd,deps})  -> handle(GraphExecutionInfo.add(dot, cmd, deps))
    to_clients() -> Option<ExecutorResult>         -> to_clients() -> (rifl, key) | None
    monitor() -> Option<&ExecutionOrderMonitor>    -> monitor() -> {key: [rifl, ...]}
    parallel() -> bool                             -> parallel() (True, like GraphExecutor)

handle() processes one Add at a time (batch of one, API-compatible);
handle_batch() takes a whole arrival-ordered batch in one device pass.  The
reference's Request/RequestReply/Executed infos (partial replication) are not
supported yet; handle() raises for them.
"""
from __future__ import annotations

import ctypes as C
from collections import deque
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .keydeps import Dependency, KeyInterner, make_config


@dataclass
class GraphExecutionInfo:
    """GraphExecutionInfo (executor/graph/executor.rs:205-240)."""
    kind: str
    dot: int = 0
    cmd: object = None
    deps: object = None

    @staticmethod
    def add(dot, cmd, deps):
        return GraphExecutionInfo("add", dot, cmd, deps)


class HipGraphExecutor:
    def __init__(self, process_id: int, shard_id: int = 0, n: int = 1, f: int = 0,
                 shard_count: int = 1, key_space: int = 1 << 20, device: int = -1,
                 monitor: bool = True):
        self._lib = L.load()
        self.process_id, self.shard_id = process_id, shard_id
        self.cfg = make_config(n=n, f=f, shard_count=shard_count, device=device,
                               key_space=key_space)
        h = C.c_void_p()
        L.check(self._lib.fh_graph_create(process_id, shard_id, C.byref(self.cfg), C.byref(h)))
        self._h = h
        self.keys = KeyInterner(key_space)
        self._cmds = {}          # dot -> command, until executed
        self._to_clients = deque()
        self._monitor = {} if monitor else None

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fh_graph_destroy(self._h)
            self._h = None

    __del__ = close

    @staticmethod
    def parallel() -> bool:
        return True  # GraphExecutor::parallel (executor.rs:110-112)

    def _keys_of(self, cmd):
        if cmd is None:
            return []
        return list(cmd.keys(self.shard_id)) if hasattr(cmd, "keys") else list(cmd)

    def handle(self, info: GraphExecutionInfo):
        if info.kind != "add":
            raise NotImplementedError("partial-replication executor infos (SURVEY §8f rank 2)")
        self.handle_batch([info])

    def handle_batch(self, infos):
        n = len(infos)
        dots = np.zeros(n, dtype=np.uint64)
        key_off = np.zeros(n + 1, dtype=np.uint32)
        dep_off = np.zeros(n + 1, dtype=np.uint32)
        keys, deps = [], []
        for i, info in enumerate(infos):
            dots[i] = info.dot
            ks = self._keys_of(info.cmd)
            keys.extend(self.keys(k) for k in ks)
            key_off[i + 1] = len(keys)
            deps.extend(d.dot if isinstance(d, Dependency) else int(d) for d in info.deps)
            dep_off[i + 1] = len(deps)
            self._cmds[int(info.dot)] = (info.cmd, ks)
        key_a = np.asarray(keys, dtype=np.uint64)
        dep_a = np.asarray(deps, dtype=np.uint64)
        L.check(self._lib.fh_graph_add_batch(self._h, n, L.ptr(dots), L.ptr(key_off),
                                             L.ptr(key_a) if len(key_a) else None,
                                             L.ptr(dep_off), L.ptr(dep_a) if len(dep_a) else None))
        self._fetch()

    def _fetch(self):
        """fetch_commands_to_execute + execute (executor.rs:133-145, 191-196)."""
        buf = np.zeros(4096, dtype=np.uint64)
        lab = np.zeros(4096, dtype=np.uint64)
        while True:
            ln = C.c_size_t(0)
            L.check(self._lib.fh_graph_drain(self._h, L.ptr(buf), L.ptr(lab), len(buf),
                                             C.byref(ln)))
            for i in range(ln.value):
                d = int(buf[i])
                cmd, ks = self._cmds.pop(d)
                rifl = getattr(cmd, "rifl", d)
                for k in ks:
                    self._to_clients.append((rifl, k))
                    if self._monitor is not None:
                        self._monitor.setdefault(k, []).append(rifl)
                self.last_labels = getattr(self, "last_labels", {})
                self.last_labels[d] = int(lab[i])
            if ln.value < len(buf):
                return

    def to_clients(self):
        return self._to_clients.popleft() if self._to_clients else None

    def monitor(self):
        return self._monitor

    def pending(self) -> int:
        c = C.c_size_t(0)
        L.check(self._lib.fh_graph_pending(self._h, C.byref(c)))
        return c.value

    def missing(self):
        n = C.c_size_t(0)
        L.check(self._lib.fh_graph_missing(self._h, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value), dtype=np.uint64)
        L.check(self._lib.fh_graph_missing(self._h, L.ptr(out), len(out), C.byref(n)))
        return [int(x) for x in out[:n.value]]

    def set_executed_frontier(self, source: int, seq: int):
        L.check(self._lib.fh_graph_set_executed_frontier(self._h, source, seq))

    def mark_executed(self, dots):
        a = np.asarray(list(dots), dtype=np.uint64)
        L.check(self._lib.fh_graph_mark_executed(self._h, len(a), L.ptr(a) if len(a) else None))
