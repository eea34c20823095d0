"""Execution logs: fantoch's on-disk stream of GraphExecutionInfo values
(SURVEY §8f rank 4).

The runner's execution logger (fantoch/src/run/task/execution_logger.rs:11-55)
writes every info an executor receives through `Rw` (run/rw/mod.rs:20-100):
tokio's LengthDelimitedCodec (4-byte big-endian length per frame) around
`bincode::serialize` (bincode 1.3 legacy options: little-endian, fixed-width
integers, u32 enum variant, u64 lengths, u8 bool/Option tags).  The replay
binary (fantoch_ps/src/bin/graph_executor_replay.rs:13-38) feeds them back to a
GraphExecutor.

* `ExecLog` -- the native parser (fh_execlog_parse, csrc/execlog.cpp): events
  as arrays, `replay(executor)` through fh_execlog_replay.
* `encode_*` / `frame` -- a writer for the same format, used to produce logs
  from the seeded workloads (tests, tools); bytes only, no protocol logic.
"""
from __future__ import annotations

import ctypes as C
import struct
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

# ---------------------------------------------------------------- writer ----
# Serde layouts: GraphExecutionInfo executor/graph/executor.rs:204-222,
# RequestReply graph/mod.rs:33-43, Command command.rs:11-20, KVOp kvs.rs:12-16,
# Dependency deps/keys/mod.rs:18-22, Id fantoch/src/id.rs:21-27.

GET, PUT, DELETE = 0, 1, 2


def _u8(x):
    return struct.pack("<B", x)


def _u32(x):
    return struct.pack("<I", x)


def _u64(x):
    return struct.pack("<Q", x)


def _str(s: str) -> bytes:
    b = s.encode()
    return _u64(len(b)) + b


def _dot(d: int) -> bytes:
    """Dot = Id<u8>{source, sequence} from a packed u64."""
    return _u8(d >> 56) + _u64(d & ((1 << 56) - 1))


def _kvop(op) -> bytes:
    if op is None or op == GET:
        return _u32(GET)
    if op == DELETE:
        return _u32(DELETE)
    return _u32(PUT) + _str(op[1] if isinstance(op, tuple) else str(op))


def encode_command(rifl: Tuple[int, int], shard_to_ops: Dict[int, Sequence[Tuple[str, object]]],
                   read_only: bool = False) -> bytes:
    """Command{rifl, shard_to_ops: HashMap<ShardId, HashMap<Key, KVOp>>,
    read_only, _empty_keys}; ops are (key, op) with op = GET / DELETE /
    (PUT, value)."""
    out = [_u64(rifl[0]), _u64(rifl[1]), _u64(len(shard_to_ops))]
    for shard, ops in shard_to_ops.items():
        out.append(_u64(shard))
        out.append(_u64(len(ops)))
        for key, op in ops:
            out.append(_str(key))
            out.append(_kvop(op))
    out.append(_u8(1 if read_only else 0))
    out.append(_u64(0))  # _empty_keys
    return b"".join(out)


def encode_dependency(dot: int, shards: Optional[Iterable[int]]) -> bytes:
    if shards is None:
        return _dot(dot) + _u8(0)
    sh = sorted(set(shards))  # BTreeSet: ascending
    return _dot(dot) + _u8(1) + _u64(len(sh)) + b"".join(_u64(s) for s in sh)


def encode_add(dot: int, cmd: bytes, deps: Sequence[Tuple[int, Optional[Iterable[int]]]]) -> bytes:
    """GraphExecutionInfo::Add{dot, cmd, deps: HashSet<Dependency>}."""
    return (_u32(0) + _dot(dot) + cmd + _u64(len(deps)) +
            b"".join(encode_dependency(d, s) for d, s in deps))


def encode_request(from_shard: int, dots: Sequence[int]) -> bytes:
    return _u32(1) + _u64(from_shard) + _u64(len(dots)) + b"".join(_dot(d) for d in dots)


def encode_request_reply(infos: Sequence[tuple]) -> bytes:
    """infos: ("info", dot, cmd_bytes, deps) | ("executed", dot)."""
    out = [_u32(2), _u64(len(infos))]
    for inf in infos:
        if inf[0] == "info":
            _, dot, cmd, deps = inf
            out.append(_u32(0) + _dot(dot) + cmd + _u64(len(deps)) +
                       b"".join(encode_dependency(d, s) for d, s in deps))
        else:
            out.append(_u32(1) + _dot(inf[1]))
    return b"".join(out)


def encode_executed(dots: Sequence[int]) -> bytes:
    return _u32(3) + _u64(len(dots)) + b"".join(_dot(d) for d in dots)


def frame(payload: bytes) -> bytes:
    """LengthDelimitedCodec default framing: u32 big-endian length."""
    return struct.pack(">I", len(payload)) + payload


# ---------------------------------------------------------------- reader ----
@dataclass
class Events:
    kind: np.ndarray
    dot: np.ndarray
    rifl_client: np.ndarray
    rifl_seq: np.ndarray
    shards: np.ndarray
    read_only: np.ndarray
    key_off: np.ndarray
    key_id: np.ndarray
    dep_off: np.ndarray
    dep_dot: np.ndarray
    dep_shards: np.ndarray


class ExecLog:
    """A parsed execution log (fh_execlog_*); keys of `shard_id` only."""

    def __init__(self, data: bytes, shard_id: int = 0):
        self._lib = L.load()
        self._buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
        h = C.c_void_p()
        L.check(self._lib.fh_execlog_parse(L.ptr(self._buf), len(data), shard_id, C.byref(h)))
        self._h = h

    @classmethod
    def read(cls, path: str, shard_id: int = 0) -> "ExecLog":
        with open(path, "rb") as fh:
            return cls(fh.read(), shard_id)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fh_execlog_destroy(self._h)
            self._h = None

    __del__ = close

    def sizes(self):
        v = [C.c_size_t(0) for _ in range(5)]
        L.check(self._lib.fh_execlog_sizes(self._h, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)  # frames, events, keys, deps, distinct keys

    def events(self) -> Events:
        _, e, k, d, _ = self.sizes()
        ev = Events(np.zeros(e, np.uint8), np.zeros(e, np.uint64), np.zeros(e, np.uint64),
                    np.zeros(e, np.uint64), np.zeros(e, np.uint64), np.zeros(e, np.uint8),
                    np.zeros(e + 1, np.uint32), np.zeros(max(k, 1), np.uint64),
                    np.zeros(e + 1, np.uint32), np.zeros(max(d, 1), np.uint64),
                    np.zeros(max(d, 1), np.uint64))
        L.check(self._lib.fh_execlog_events(self._h, *[L.ptr(a) for a in (
            ev.kind, ev.dot, ev.rifl_client, ev.rifl_seq, ev.shards, ev.read_only, ev.key_off,
            ev.key_id, ev.dep_off, ev.dep_dot, ev.dep_shards)]))
        ev.key_id, ev.dep_dot, ev.dep_shards = ev.key_id[:k], ev.dep_dot[:d], ev.dep_shards[:d]
        return ev

    def key(self, i: int) -> str:
        n = C.c_size_t(0)
        st = self._lib.fh_execlog_key(self._h, i, None, 0, C.byref(n))
        if st not in (L.FH_OK, L.FH_ECAP):
            L.check(st)
        buf = C.create_string_buffer(max(1, n.value))
        L.check(self._lib.fh_execlog_key(self._h, i, buf, n.value, C.byref(n)))
        return buf.raw[:n.value].decode()

    def keys(self) -> List[str]:
        return [self.key(i) for i in range(self.sizes()[4])]

    def replay(self, executor, batch: int = 0) -> int:
        """graph_executor_replay.rs:30-37 through fh_execlog_replay into a
        HipGraphExecutor's handle; returns the commands that became ready
        (drained into the executor's to_clients / monitor)."""
        ev = self.events()
        names = self.keys()
        for e in np.nonzero((ev.kind == L.FH_LOG_ADD) | (ev.kind == L.FH_LOG_REPLY_INFO))[0]:
            ks = [names[int(k)] for k in ev.key_id[ev.key_off[e]:ev.key_off[e + 1]]]
            executor._cmds[int(ev.dot[e])] = (
                _Logged((int(ev.rifl_client[e]), int(ev.rifl_seq[e]))), ks)
        n = C.c_size_t(0)
        L.check(self._lib.fh_execlog_replay(self._h, executor._h, batch, C.byref(n)))
        executor._fetch()
        return n.value


@dataclass
class _Logged:
    """The payload side of a logged command: its rifl (ExecutorResult)."""
    rifl: Tuple[int, int]
