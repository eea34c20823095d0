"""KV execution on the host: the last step of the executor path, after the
engine's per-key order (Command / KV execution stays
host-side; the device output stops at the execution order).

Restates, with the reference's semantics:
  KVOp / KVStore::{execute, execute_with_monitor, do_execute}
      fantoch/src/kvs.rs:9-69
  ExecutorResult                        fantoch/src/executor/mod.rs:168-183
  CommandResult::{new, add_partial, increment_key_count}
      fantoch/src/command.rs:171-216
  AggregatePending::{wait_for, wait_for_rifl, add_executor_result}
      fantoch/src/executor/aggregate.rs:9-99
  ExecutionOrderMonitor::add (the per-key order)  executor/monitor.rs:20-28
Keys and values are strings, as Key = Value = String (kvs.rs:6-7).
"""
from __future__ import annotations

from typing import NamedTuple, Optional


class KVOp(NamedTuple):
    """KVOp::{Get, Put(Value), Delete} (kvs.rs:12-16)."""
    kind: str                    # "get" | "put" | "delete"
    value: Optional[str] = None  # Put's value

    @staticmethod
    def get():
        return KVOp("get")

    @staticmethod
    def put(value: str):
        return KVOp("put", value)

    @staticmethod
    def delete():
        return KVOp("delete")


class ExecutorResult(NamedTuple):
    """ExecutorResult{rifl, key, op_result} (executor/mod.rs:168-183)."""
    rifl: object
    key: str
    op_result: Optional[str]


class KVStore:
    """KVStore (kvs.rs:20-69): a map Key -> Value."""

    def __init__(self):
        self._store = {}

    def execute(self, key: str, op: KVOp) -> Optional[str]:
        """KVStore::execute (test-only in the reference, kvs.rs:31-35)."""
        return self._do_execute(key, op)

    def execute_with_monitor(self, key: str, op: KVOp, rifl, monitor) -> Optional[str]:
        """kvs.rs:37-49: the monitor records (key, rifl) first."""
        if monitor is not None:
            monitor.setdefault(key, []).append(rifl)
        return self._do_execute(key, op)

    def _do_execute(self, key: str, op: KVOp) -> Optional[str]:
        """kvs.rs:52-68: Get returns the value, Put and Delete the previous one."""
        if op.kind == "get":
            return self._store.get(key)
        if op.kind == "put":
            prev = self._store.get(key)
            self._store[key] = op.value
            return prev
        if op.kind == "delete":
            return self._store.pop(key, None)
        raise ValueError(f"unknown KVOp {op!r}")

    def __len__(self):
        return len(self._store)


class CommandResult:
    """CommandResult (command.rs:171-216): the partial results of a
    multi-key command, ready once every key reported."""

    def __init__(self, rifl, key_count: int):
        self.rifl = rifl
        self.key_count = key_count
        self.results = {}

    def add_partial(self, key: str, result) -> bool:
        assert key not in self.results, "a key reported twice (command.rs:196-197)"
        self.results[key] = result
        return len(self.results) == self.key_count

    def increment_key_count(self):
        self.key_count += 1


class AggregatePending:
    """AggregatePending (executor/aggregate.rs:9-99): joins the executors'
    per-key results into whole-command results for the clients."""

    def __init__(self, process_id: int, shard_id: int = 0):
        self.process_id, self.shard_id = process_id, shard_id
        self.pending = {}

    def wait_for(self, cmd) -> bool:
        """aggregate.rs:31-46: expect key_count(shard) partial results."""
        fresh = cmd.rifl not in self.pending
        self.pending[cmd.rifl] = CommandResult(cmd.rifl, cmd.key_count(self.shard_id))
        return fresh

    def wait_for_rifl(self, rifl):
        """aggregate.rs:49-61."""
        self.pending.setdefault(rifl, CommandResult(rifl, 0)).increment_key_count()

    def add_executor_result(self, r: ExecutorResult):
        """aggregate.rs:64-98: the whole result once the last key reports;
        results of commands nobody waits for are ignored."""
        cr = self.pending.get(r.rifl)
        if cr is None:
            return None
        if cr.add_partial(r.key, r.op_result):
            return self.pending.pop(r.rifl)
        return None
