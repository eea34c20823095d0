"""ctypes view of the CPU oracle (oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package (fantoch_amd).
Parity status and the reference tests that pin it: see oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")

u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    if not os.path.exists(_SO):
        build()
    lib = C.CDLL(_SO)
    V, S = C.c_void_p, C.c_size_t
    lib.fo_keydeps_new.restype = V
    lib.fo_keydeps_new.argtypes = [C.c_uint64]
    lib.fo_keydeps_free.argtypes = [V]
    lib.fo_keydeps_add_cmd.restype = S
    lib.fo_keydeps_add_cmd.argtypes = [V, C.c_uint64, V, S, V, S, C.c_int, V, S]
    lib.fo_keydeps_add_noop.restype = S
    lib.fo_keydeps_add_noop.argtypes = [V, C.c_uint64, V, S]
    lib.fo_keydeps_cmd_deps.restype = S
    lib.fo_keydeps_cmd_deps.argtypes = [V, V, S, V, S]
    lib.fo_keydeps_noop_deps.restype = S
    lib.fo_keydeps_noop_deps.argtypes = [V, V, S]
    lib.fo_keydeps_run.restype = S
    lib.fo_keydeps_run.argtypes = [C.c_uint64, S, u64p, u32p, u64p, V, u32p, u64p, S]
    lib.fo_quorum_deps.restype = S
    lib.fo_quorum_deps.argtypes = [S, S, u32p, u64p, C.c_int, S, u64p, S, C.POINTER(C.c_int)]
    lib.fo_views_run.restype = S
    lib.fo_views_run.argtypes = [C.c_int, C.c_uint32, S, C.c_uint32, u64p, u32p, u64p,
                                 u8p, u64p, u32p, u64p, S]
    lib.fo_graph_new.restype = V
    lib.fo_graph_new.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.fo_graph_free.argtypes = [V]
    lib.fo_graph_add.restype = S
    lib.fo_graph_add.argtypes = [V, C.c_uint64, V, S, V, S]
    lib.fo_graph_index_only.argtypes = [V, C.c_uint64, V, S, V, S]
    lib.fo_graph_set_executed_frontier.argtypes = [V, C.c_uint32, C.c_uint64]
    lib.fo_graph_find_scc.restype = C.c_int
    lib.fo_graph_find_scc.argtypes = [V, C.c_int, C.c_uint64, C.POINTER(S), C.POINTER(S),
                                      V, S, C.POINTER(S)]
    lib.fo_graph_executed.restype = C.c_int
    lib.fo_graph_executed.argtypes = [V, C.c_uint64]
    lib.fo_graph_drain.restype = S
    lib.fo_graph_drain.argtypes = [V, V, V, S]
    lib.fo_graph_pending_count.restype = S
    lib.fo_graph_pending_count.argtypes = [V]
    lib.fo_lkeydeps_new.restype = V
    lib.fo_lkeydeps_new.argtypes = [C.c_uint64]
    lib.fo_lkeydeps_free.argtypes = [V]
    lib.fo_lkeydeps_add_cmd.restype = S
    lib.fo_lkeydeps_add_cmd.argtypes = [V, C.c_uint64, V, S, C.c_int, V, S, C.c_int, V, S]
    lib.fo_lkeydeps_add_noop.restype = S
    lib.fo_lkeydeps_add_noop.argtypes = [V, C.c_uint64, V, S]
    lib.fo_lkeydeps_cmd_deps.restype = S
    lib.fo_lkeydeps_cmd_deps.argtypes = [V, V, S, V, S]
    lib.fo_lkeydeps_noop_deps.restype = S
    lib.fo_lkeydeps_noop_deps.argtypes = [V, V, S]
    lib.fo_pred_new.restype = V
    lib.fo_pred_new.argtypes = [C.c_uint32]
    lib.fo_pred_free.argtypes = [V]
    lib.fo_pred_add.restype = S
    lib.fo_pred_add.argtypes = [V, C.c_uint64, C.c_uint64, V, S]
    lib.fo_pred_drain.restype = S
    lib.fo_pred_drain.argtypes = [V, V, S]
    lib.fo_pred_pending_count.restype = S
    lib.fo_pred_pending_count.argtypes = [V]
    lib.fo_graph_add_sharded.restype = S
    lib.fo_graph_add_sharded.argtypes = [V, C.c_uint64, V, S, C.c_uint64, V, V, S]
    lib.fo_graph_handle_requests.argtypes = [V, C.c_uint64, V, S]
    lib.fo_graph_cleanup.argtypes = [V]
    lib.fo_graph_requests.restype = S
    lib.fo_graph_requests.argtypes = [V, V, V, S]
    lib.fo_graph_replies_size.argtypes = [V, C.POINTER(S), C.POINTER(S)]
    lib.fo_graph_replies_take.argtypes = [V, V, V, V, V, V, V, V]
    lib.fo_graph_mark_executed.restype = S
    lib.fo_graph_mark_executed.argtypes = [V, C.c_uint64]
    lib.fo_graph_violation.restype = C.c_int
    lib.fo_graph_violation.argtypes = [V]
    lib.fo_graph_run.restype = S
    lib.fo_graph_run.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, S, u64p, u32p, u64p,
                                 u32p, u64p, u64p, u64p, C.c_uint64, u32p, u64p]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def dot(src: int, seq: int) -> int:
    return (int(src) << 56) | int(seq)


def _arr(xs):
    a = np.ascontiguousarray(np.asarray(list(xs), dtype=np.uint64))
    return a


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a.size else None


class KeyDeps:
    """SequentialKeyDeps (deps/keys/sequential.rs:7-144); keys are u64 ids."""

    def __init__(self, shard_id: int = 0):
        self._h = lib().fo_keydeps_new(shard_id)
        self._cap = 1 << 12

    def __del__(self):
        if getattr(self, "_h", None):
            lib().fo_keydeps_free(self._h)
            self._h = None

    def _call(self, fn, *args):
        while True:
            out = np.zeros(self._cap, dtype=np.uint64)
            n = fn(*args, _ptr(out), self._cap)
            if n <= self._cap:
                return set(int(x) for x in out[:n])
            self._cap = n * 2

    def add_cmd(self, dot_, keys, past=None):
        k = _arr(keys)
        p = _arr(past or [])
        # capacity is known up front: |past| + |keys| + 1
        cap = len(p) + len(k) + 1
        out = np.zeros(cap, dtype=np.uint64)
        n = lib().fo_keydeps_add_cmd(self._h, dot_, _ptr(k), len(k), _ptr(p), len(p),
                                     1 if past is not None else 0, _ptr(out), cap)
        return set(int(x) for x in out[:n])

    def add_noop(self, dot_):
        # noop deps can be as large as the key table: query the size first
        n = lib().fo_keydeps_noop_deps(self._h, None, 0) + 1
        out = np.zeros(n, dtype=np.uint64)
        m = lib().fo_keydeps_add_noop(self._h, dot_, _ptr(out), n)
        assert m <= n
        return set(int(x) for x in out[:m])

    def cmd_deps(self, keys):
        k = _arr(keys)
        out = np.zeros(len(k) + 1, dtype=np.uint64)
        n = lib().fo_keydeps_cmd_deps(self._h, _ptr(k), len(k), _ptr(out), len(out))
        return set(int(x) for x in out[:n])

    def noop_deps(self):
        n = lib().fo_keydeps_noop_deps(self._h, None, 0)
        out = np.zeros(max(n, 1), dtype=np.uint64)
        lib().fo_keydeps_noop_deps(self._h, _ptr(out), n)
        return set(int(x) for x in out[:n])


class LockedKeyDeps:
    """LockedKeyDeps (deps/keys/locked.rs:10-186), applied sequentially."""

    def __init__(self, shard_id: int = 0):
        self._h = lib().fo_lkeydeps_new(shard_id)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().fo_lkeydeps_free(self._h)
            self._h = None

    def add_cmd(self, dot_, keys, read_only=False, past=None):
        k = _arr(keys)
        p = _arr(past or [])
        cap = len(p) + 2 * len(k) + 1
        out = np.zeros(cap, dtype=np.uint64)
        n = lib().fo_lkeydeps_add_cmd(self._h, dot_, _ptr(k), len(k), 1 if read_only else 0,
                                      _ptr(p), len(p), 1 if past is not None else 0,
                                      _ptr(out), cap)
        return set(int(x) for x in out[:n])

    def add_noop(self, dot_):
        n = lib().fo_lkeydeps_noop_deps(self._h, None, 0) + 1
        out = np.zeros(n, dtype=np.uint64)
        m = lib().fo_lkeydeps_add_noop(self._h, dot_, _ptr(out), n)
        assert m <= n
        return set(int(x) for x in out[:m])

    def cmd_deps(self, keys):
        k = _arr(keys)
        out = np.zeros(2 * len(k) + 1, dtype=np.uint64)
        n = lib().fo_lkeydeps_cmd_deps(self._h, _ptr(k), len(k), _ptr(out), len(out))
        return set(int(x) for x in out[:n])

    def noop_deps(self):
        n = lib().fo_lkeydeps_noop_deps(self._h, None, 0)
        out = np.zeros(max(n, 1), dtype=np.uint64)
        lib().fo_lkeydeps_noop_deps(self._h, _ptr(out), n)
        return set(int(x) for x in out[:n])


def keydeps_run(dots, key_off, keys, is_noop=None, shard_id=0):
    """Run one SequentialKeyDeps over a whole stream; returns (dep_off, deps)."""
    n = len(dots)
    cap = int(len(keys) + n + 16)
    if is_noop is not None and np.any(is_noop):
        cap += int(np.count_nonzero(is_noop)) * (len(np.unique(keys)) + 1)
    out_off = np.zeros(n + 1, dtype=np.uint32)
    out = np.zeros(cap, dtype=np.uint64)
    noop = None
    if is_noop is not None:
        noop_a = np.ascontiguousarray(is_noop, dtype=np.uint8)
        noop = noop_a.ctypes.data_as(C.c_void_p)
    tot = lib().fo_keydeps_run(shard_id, n, np.ascontiguousarray(dots, np.uint64),
                               np.ascontiguousarray(key_off, np.uint32),
                               np.ascontiguousarray(keys, np.uint64), noop, out_off, out, cap)
    assert tot != (2**64 - 1), "oracle output capacity"
    return out_off, out[:tot]


def quorum_deps(fast_quorum_size, reports, mode, threshold=0):
    """QuorumDeps (deps/quorum.rs): mode 0 = check_threshold_union(threshold),
    mode 1 = check_union.  reports: list of dep-dot iterables."""
    off = np.zeros(len(reports) + 1, dtype=np.uint32)
    flat = []
    for i, r in enumerate(reports):
        flat.extend(r)
        off[i + 1] = len(flat)
    dep = np.asarray(flat if flat else [0], dtype=np.uint64)
    out = np.zeros(len(flat) + 1, dtype=np.uint64)
    flag = C.c_int(0)
    n = lib().fo_quorum_deps(fast_quorum_size, len(reports), off, dep, mode, threshold, out,
                             len(out), C.byref(flag))
    return set(int(x) for x in out[:n]), bool(flag.value)


def views_run(protocol, nproc, dots, key_off, keys, fq_proc, fq_time):
    n = len(dots)
    fq = fq_proc.shape[1]
    cap = int(len(keys) * fq + n + 16)
    out_off = np.zeros(n + 1, dtype=np.uint32)
    out = np.zeros(cap, dtype=np.uint64)
    tot = lib().fo_views_run(protocol, nproc, n, fq, np.ascontiguousarray(dots, np.uint64),
                             np.ascontiguousarray(key_off, np.uint32),
                             np.ascontiguousarray(keys, np.uint64),
                             np.ascontiguousarray(fq_proc, np.uint8).reshape(-1),
                             np.ascontiguousarray(fq_time, np.uint64).reshape(-1), out_off, out,
                             cap)
    assert tot != (2**64 - 1), "oracle output capacity"
    return out_off, out[:tot]


class Graph:
    """DependencyGraph (executor/graph/mod.rs:45-679) with TarjanSCCFinder."""

    def __init__(self, process_id=1, shard_id=0, n=1, f=1, shard_count=1):
        self._h = lib().fo_graph_new(process_id, shard_id, n, f, shard_count)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().fo_graph_free(self._h)
            self._h = None

    def add(self, dot_, keys, deps):
        k = _arr(keys)
        d = _arr(deps)
        return lib().fo_graph_add(self._h, dot_, _ptr(k), len(k), _ptr(d), len(d))

    def index_only(self, dot_, keys, deps):
        k = _arr(keys)
        d = _arr(deps)
        lib().fo_graph_index_only(self._h, dot_, _ptr(k), len(k), _ptr(d), len(d))

    def set_executed_frontier(self, source, seq):
        lib().fo_graph_set_executed_frontier(self._h, source, seq)

    def find_scc(self, first_find, dot_):
        ready = C.c_size_t(0)
        nfound = C.c_size_t(0)
        nmiss = C.c_size_t(0)
        miss = np.zeros(64, dtype=np.uint64)
        kind = lib().fo_graph_find_scc(self._h, 1 if first_find else 0, dot_, C.byref(ready),
                                       C.byref(nfound), _ptr(miss), 64, C.byref(nmiss))
        return kind, ready.value, nfound.value, [int(x) for x in miss[:nmiss.value]]

    def executed(self, dot_):
        return bool(lib().fo_graph_executed(self._h, dot_))

    def drain(self):
        out, lab = [], []
        buf = np.zeros(1024, dtype=np.uint64)
        lbuf = np.zeros(1024, dtype=np.uint64)
        while True:
            n = lib().fo_graph_drain(self._h, _ptr(buf), _ptr(lbuf), 1024)
            out.extend(int(x) for x in buf[:n])
            lab.extend(int(x) for x in lbuf[:n])
            if n < 1024:
                return out, lab

    def pending(self):
        return lib().fo_graph_pending_count(self._h)

    # -- partial replication (graph/mod.rs:139-157, 168-179, 279-408) -----
    def add_sharded(self, dot_, keys, cmd_shards, deps):
        """handle_add with shard sets: deps = [(dot, shards or None)]."""
        k = _arr(keys)
        d = _arr(x for x, _ in deps)
        m = _arr(_mask(s) for _, s in deps)
        return lib().fo_graph_add_sharded(self._h, dot_, _ptr(k), len(k), _mask(cmd_shards),
                                          _ptr(d), _ptr(m), len(d))

    def handle_requests(self, from_shard, dots):
        d = _arr(dots)
        lib().fo_graph_handle_requests(self._h, from_shard, _ptr(d), len(d))

    def cleanup(self):
        lib().fo_graph_cleanup(self._h)

    def requests(self):
        """requests(): {target shard: {dots}} (taken)."""
        n = lib().fo_graph_requests(self._h, None, None, 0)
        sh = np.zeros(max(1, n), dtype=np.uint64)
        dt = np.zeros(max(1, n), dtype=np.uint64)
        m = lib().fo_graph_requests(self._h, _ptr(sh), _ptr(dt), n)
        assert m == n
        out = {}
        for s, d in zip(sh[:n].tolist(), dt[:n].tolist()):
            out.setdefault(s, set()).add(d)
        return out

    def request_replies(self):
        """request_replies(): {to: [("info", dot, cmd_shards, [(dep, shards)]) |
        ("executed", dot)]} in list order (taken)."""
        nr, nd = C.c_size_t(0), C.c_size_t(0)
        lib().fo_graph_replies_size(self._h, C.byref(nr), C.byref(nd))
        nr, nd = nr.value, nd.value
        if nr == 0:
            return {}
        a = [np.zeros(max(1, x), dtype=np.uint64) for x in (nr, nr, nr, nr, nr + 1, nd, nd)]
        lib().fo_graph_replies_take(self._h, *[_ptr(x) for x in a])
        to, kind, dot_, cm, off, dd, dm = [x.tolist() for x in a]
        out = {}
        for i in range(nr):
            if kind[i] == 0:
                deps = [(dd[e], _unmask(dm[e])) for e in range(off[i], off[i + 1])]
                r = ("info", dot_[i], _unmask(cm[i]), deps)
            else:
                r = ("executed", dot_[i])
            out.setdefault(to[i], []).append(r)
        return out

    def mark_executed(self, dot_):
        """RequestReply::Executed{dot} (mod.rs:393-405)."""
        return lib().fo_graph_mark_executed(self._h, dot_)

    def violation(self):
        return bool(lib().fo_graph_violation(self._h))


def _mask(shards):
    if shards is None:
        return 0
    m = 0
    for s in shards:
        m |= 1 << int(s)
    return m


def _unmask(m):
    if m == 0:
        return None
    return frozenset(i for i in range(64) if (m >> i) & 1)


def graph_run(dots, key_off, keys, dep_off, deps, key_space, process_id=1, n=1, f=1):
    """GraphExecutor over a whole arrival stream.  Returns
    (exec_dots, scc_labels, key_seq_off, key_seq)."""
    ncmd = len(dots)
    exec_dot = np.zeros(max(ncmd, 1), dtype=np.uint64)
    scc = np.zeros(max(ncmd, 1), dtype=np.uint64)
    kso = np.zeros(key_space + 1, dtype=np.uint32)
    ks = np.zeros(max(len(keys), 1), dtype=np.uint64)
    deps_a = np.ascontiguousarray(deps, np.uint64)
    if deps_a.size == 0:
        deps_a = np.zeros(1, dtype=np.uint64)
    keys_a = np.ascontiguousarray(keys, np.uint64)
    if keys_a.size == 0:
        keys_a = np.zeros(1, dtype=np.uint64)
    ne = lib().fo_graph_run(process_id, n, f, ncmd, np.ascontiguousarray(dots, np.uint64),
                            np.ascontiguousarray(key_off, np.uint32), keys_a,
                            np.ascontiguousarray(dep_off, np.uint32), deps_a, exec_dot, scc,
                            key_space, kso, ks)
    return exec_dot[:ne], scc[:ne], kso, ks[:kso[-1]]


def clock(seq: int, process_id: int) -> int:
    """Clock{seq, process_id} packed so that integer order == Clock's Ord
    (protocol/common/pred/clocks/mod.rs:15-30)."""
    return (seq << 8) | process_id


class Pred:
    """PredecessorsGraph (Caesar, executor/pred/mod.rs:26-352)."""

    def __init__(self, process_id=1):
        self._h = lib().fo_pred_new(process_id)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().fo_pred_free(self._h)
            self._h = None

    def add(self, dot_, clock_, deps):
        d = _arr(deps)
        return lib().fo_pred_add(self._h, dot_, clock_, _ptr(d), len(d))

    def drain(self):
        out = []
        buf = np.zeros(1024, dtype=np.uint64)
        while True:
            n = lib().fo_pred_drain(self._h, _ptr(buf), 1024)
            out.extend(int(x) for x in buf[:n])
            if n < 1024:
                return out

    def pending(self):
        return lib().fo_pred_pending_count(self._h)


def pred_run(dots, clocks, dep_off, deps, process_id=1):
    """PredecessorsGraph over an arrival stream, draining after every add.
    Returns (execution order as dots, pending count)."""
    p = Pred(process_id)
    out = []
    deps = np.ascontiguousarray(deps, np.uint64)
    for i in range(len(dots)):
        p.add(int(dots[i]), int(clocks[i]), deps[dep_off[i]:dep_off[i + 1]])
        out.extend(p.drain())
    return np.asarray(out, dtype=np.uint64), p.pending()
