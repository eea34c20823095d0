"""HipGraphExecutor -- the Executor trait with GraphExecutor semantics, backed
by the HIP engine (fh_graph_*).

Mirrors fantoch/src/executor/mod.rs:27-88 and
fantoch_ps/src/executor/graph/executor.rs:19-197:

    Executor::new(process_id, shard_id, config)   -> HipGraphExecutor(process_id, shard_id, n, f)
    handle(GraphExecutionInfo::Add{dot,cmd,deps})  -> handle(GraphExecutionInfo.add(dot, cmd, deps))
    to_clients() -> Option<ExecutorResult>         -> to_clients() -> ExecutorResult(rifl, key, op_result) | None
    monitor() -> Option<&ExecutionOrderMonitor>    -> monitor() -> {key: [rifl, ...]}
    parallel() -> bool                             -> parallel() (True, like GraphExecutor)

    cleanup() / to_executors / fetch_requests / fetch_request_replies
                                                   -> cleanup(), requests(), request_replies()

handle() processes one info at a time (an Add is a batch of one,
API-compatible); handle_batch() takes a whole arrival-ordered batch of Adds
in one device pass.  Partial replication (graph/mod.rs:279-408): Add infos
carry shard sets (Dependency.shards, Command.shards()); a missing dependency
not replicated here becomes a request to its target shard; Request infos are
answered with Info / Executed replies or buffered until cleanup();
RequestReply infos are ingested (Info -> add, Executed -> executed clock +
pending retry).  One handle plays both executor roles of the shard (the
reference routes Add/RequestReply to index 0 and Request/Executed to index 1,
executor.rs:242-262, over a shared VertexIndex).
"""
from __future__ import annotations

import ctypes as C
from collections import deque
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .keydeps import Dependency, KeyInterner, make_config
from .kvs import ExecutorResult, KVStore


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

    @staticmethod
    def request(from_shard, dots):
        """GraphExecutionInfo::Request{from, dots} (executor.rs:215-220)."""
        return GraphExecutionInfo("request", from_shard, None, list(dots))

    @staticmethod
    def request_reply(replies):
        """GraphExecutionInfo::RequestReply{infos} (executor.rs:221-224)."""
        return GraphExecutionInfo("request_reply", 0, None, list(replies))

    @staticmethod
    def executed(dots):
        """GraphExecutionInfo::Executed{dots} (executor.rs:225-227)."""
        return GraphExecutionInfo("executed", 0, None, list(dots))


@dataclass
class RequestReply:
    """RequestReply::{Info{dot, cmd, deps}, Executed{dot}} (graph/mod.rs:33-43)."""
    kind: str          # "info" | "executed"
    dot: int
    cmd: object = None
    deps: object = None  # list[Dependency] for Info


def _mask(shards) -> int:
    m = 0
    for s in shards:
        if s >= 64:
            raise ValueError("shard ids must be < 64")
        m |= 1 << s
    return m


def _unmask(m: int):
    return frozenset(s for s in range(64) if (m >> s) & 1)


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
        self.store = KVStore()  # GraphExecutor's KVStore (executor.rs:29, 191-196)
        # request replies taken from the handle as soon as they are made, with
        # the command attached then (process_requests clones vertex.cmd when
        # it answers, graph/mod.rs:323-330: a later execution must not lose it)
        self._replies = {}

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
        """GraphExecutor::handle (executor.rs:76-100)."""
        if info.kind == "add":
            self.handle_batch([info])
        elif info.kind == "request":
            self.handle_request(info.dot, info.deps)
        elif info.kind == "request_reply":
            self.handle_request_reply(info.deps)
        elif info.kind == "executed":
            pass  # handle_executed: the shard's single handle already holds the clock
        else:
            raise ValueError(f"unknown GraphExecutionInfo kind {info.kind!r}")

    def handle_batch(self, infos):
        n = len(infos)
        dots = np.zeros(n, dtype=np.uint64)
        key_off = np.zeros(n + 1, dtype=np.uint32)
        dep_off = np.zeros(n + 1, dtype=np.uint32)
        cmd_sh = np.zeros(n, dtype=np.uint64)
        keys, deps, dep_sh = [], [], []
        sharded = False
        for i, info in enumerate(infos):
            dots[i] = info.dot
            ks = self._keys_of(info.cmd)
            keys.extend(self.keys(k) for k in ks)
            key_off[i + 1] = len(keys)
            for d in info.deps:
                if isinstance(d, Dependency):
                    deps.append(d.dot)
                    dep_sh.append(_mask(d.shards) if d.shards is not None else 0)
                    sharded |= d.shards is not None
                else:
                    deps.append(int(d))
                    dep_sh.append(0)
            dep_off[i + 1] = len(deps)
            if hasattr(info.cmd, "shards"):
                cmd_sh[i] = _mask(info.cmd.shards())
            self._cmds[int(info.dot)] = (info.cmd, ks)
        key_a = np.asarray(keys, dtype=np.uint64)
        dep_a = np.asarray(deps, dtype=np.uint64)
        dsh_a = np.asarray(dep_sh, dtype=np.uint64)
        if self.cfg.shard_count > 1 and sharded:
            L.check(self._lib.fh_graph_add_batch_sharded(
                self._h, n, L.ptr(dots), L.ptr(key_off), L.ptr(key_a) if len(key_a) else None,
                L.ptr(dep_off), L.ptr(dep_a) if len(dep_a) else None, L.ptr(cmd_sh),
                L.ptr(dsh_a) if len(dsh_a) else None))
        else:
            L.check(self._lib.fh_graph_add_batch(self._h, n, L.ptr(dots), L.ptr(key_off),
                                                 L.ptr(key_a) if len(key_a) else None,
                                                 L.ptr(dep_off),
                                                 L.ptr(dep_a) if len(dep_a) else None))
        self._fetch()

    # -- partial replication (graph/mod.rs:279-408, executor.rs:147-189) -----
    def handle_request(self, from_shard: int, dots):
        a = np.asarray(list(dots), dtype=np.uint64)
        L.check(self._lib.fh_graph_handle_requests(self._h, from_shard, len(a),
                                                   L.ptr(a) if len(a) else None))
        self._take_replies()

    def handle_request_reply(self, replies):
        """In reply order (mod.rs:377-408): each run of consecutive Info
        replies is one add batch (handle_add per reply), each Executed reply
        updates the executed clock and retries the pending vertices."""
        run = []
        for r in replies:
            if r.kind == "info":
                run.append(GraphExecutionInfo.add(r.dot, r.cmd, r.deps))
                continue
            if run:
                self.handle_batch(run)
                run = []
            self.mark_executed([r.dot])
            self.handle_batch([])  # check_pending against the new clock
        if run:
            self.handle_batch(run)

    def set_time(self, now_ms: int):
        """SysTime::millis for the vertices added next (Vertex::new)."""
        L.check(self._lib.fh_graph_set_time(self._h, int(now_ms)))

    def monitor_pending(self, threshold_ms: int = 1000):
        """Executor::monitor_pending (index.rs:53-103): [(dot, pending_ms,
        missing deps)] longest pending first; raises FhError(FH_EINVARIANT)
        for a pending command without missing dependencies."""
        n = C.c_size_t(0)
        L.check(self._lib.fh_graph_monitor_pending(self._h, int(threshold_ms), None, None, None, 0,
                                                   C.byref(n)))
        if n.value == 0:
            return []
        d = np.zeros(n.value, dtype=np.uint64)
        t = np.zeros(n.value, dtype=np.uint64)
        m = np.zeros(n.value, dtype=np.uint64)
        L.check(self._lib.fh_graph_monitor_pending(self._h, int(threshold_ms), L.ptr(d), L.ptr(t),
                                                   L.ptr(m), n.value, C.byref(n)))
        return list(zip(d.tolist(), t.tolist(), m.tolist()))

    def take_metrics(self):
        """ChainSize / ExecutionDelay values collected since the last call
        (ExecutorMetricsKind, executor/mod.rs:120-129)."""
        nc, nd = C.c_size_t(0), C.c_size_t(0)
        st = self._lib.fh_graph_take_metrics(self._h, None, 0, None, 0, C.byref(nc), C.byref(nd))
        if nc.value == 0 and nd.value == 0:
            L.check(st)
            return [], []
        ch = np.zeros(max(1, nc.value), dtype=np.uint64)
        de = np.zeros(max(1, nd.value), dtype=np.uint64)
        L.check(self._lib.fh_graph_take_metrics(self._h, L.ptr(ch), nc.value, L.ptr(de), nd.value,
                                                C.byref(nc), C.byref(nd)))
        return ch[:nc.value].tolist(), de[:nd.value].tolist()

    def passes(self):
        p, k = C.c_uint64(0), C.c_uint64(0)
        L.check(self._lib.fh_graph_passes(self._h, C.byref(p), C.byref(k)))
        return p.value, k.value

    def cleanup(self):
        """Executor::cleanup -> check_pending_requests (mod.rs:168-179)."""
        L.check(self._lib.fh_graph_cleanup(self._h))
        self._take_replies()

    def requests(self):
        """fetch_requests: {target shard: set(dots)} (mod.rs:147-150)."""
        n = C.c_size_t(0)
        st = self._lib.fh_graph_requests(self._h, None, None, 0, C.byref(n))
        if n.value == 0:
            return {}
        if st != L.FH_ECAP:
            L.check(st)
        dot = np.zeros(n.value, dtype=np.uint64)
        sh = np.zeros(n.value, dtype=np.uint64)
        L.check(self._lib.fh_graph_requests(self._h, L.ptr(dot), L.ptr(sh), n.value, C.byref(n)))
        out = {}
        for d, s in zip(dot.tolist(), sh.tolist()):
            out.setdefault(int(s), set()).add(int(d))
        return out

    def request_replies(self):
        """fetch_request_replies: {to shard: [RequestReply]} (mod.rs:152-157),
        taken."""
        self._take_replies()
        out, self._replies = self._replies, {}
        return out

    def _take_replies(self):
        nr, nd = C.c_size_t(0), C.c_size_t(0)
        st = self._lib.fh_graph_request_replies(self._h, 0, None, None, None, None, None, 0,
                                                None, None, C.byref(nr), C.byref(nd))
        if nr.value == 0:
            return
        if st != L.FH_ECAP:
            L.check(st)
        r, d = nr.value, max(1, nd.value)
        to = np.zeros(r, np.uint64)
        kind = np.zeros(r, np.uint8)
        dot = np.zeros(r, np.uint64)
        csh = np.zeros(r, np.uint64)
        off = np.zeros(r + 1, np.uint32)
        ddot = np.zeros(d, np.uint64)
        dsh = np.zeros(d, np.uint64)
        L.check(self._lib.fh_graph_request_replies(
            self._h, r, L.ptr(to), L.ptr(kind), L.ptr(dot), L.ptr(csh), L.ptr(off), d,
            L.ptr(ddot), L.ptr(dsh), C.byref(nr), C.byref(nd)))
        for i in range(r):
            dt = int(dot[i])
            if kind[i] == L.FH_REPLY_INFO:
                deps = [Dependency(int(ddot[e]), _unmask(int(dsh[e])) if dsh[e] else None)
                        for e in range(off[i], off[i + 1])]
                # the handle answered Info: the vertex is pending, so its
                # command is still held here
                rep = RequestReply("info", dt, self._cmds[dt][0], deps)
            else:
                rep = RequestReply("executed", dt)
            self._replies.setdefault(int(to[i]), []).append(rep)

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
                if hasattr(cmd, "execute"):
                    # Command::execute on this executor's KVStore + monitor
                    self._to_clients.extend(cmd.execute(self.shard_id, self.store, self._monitor))
                else:  # a bare key list (tests): the order only
                    rifl = getattr(cmd, "rifl", d)
                    for k in ks:
                        self._to_clients.append(ExecutorResult(rifl, k, None))
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
