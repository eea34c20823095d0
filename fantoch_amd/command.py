"""Command (fantoch/src/command.rs:11-156) for the host mirror.

The rifl, the keys per shard (Command::keys, :95-100; shards, :108-110) and
each key's KVOp (shard_to_ops).  Keys are strings as in fantoch and are
interned to dense ids by the KeyDeps / executor mirrors; execute() applies
the shard's ops to a KVStore (command.rs:114-127, fantoch_amd/kvs.py).
"""
from __future__ import annotations

from .kvs import ExecutorResult, KVOp


class Command:
    """keys: the command's keys; ops: {key: KVOp} (default: Put(str(rifl))
    on every key, or Get on every key when read_only).  read_only: every op
    is a Get (Command::new, command.rs:23-51, which also rejects commands
    that mix Gets with writes)."""
    __slots__ = ("rifl", "shard_to_keys", "read_only", "ops")

    def __init__(self, rifl, keys, shard_of=None, read_only: bool = False, ops=None):
        self.rifl = rifl
        self.shard_to_keys = {}
        for k in keys:
            s = shard_of(k) if shard_of else 0
            self.shard_to_keys.setdefault(s, [])
            if k not in self.shard_to_keys[s]:
                self.shard_to_keys[s].append(k)
        if ops is None:
            op = KVOp.get() if read_only else KVOp.put(str(rifl))
            ops = {k: op for ks in self.shard_to_keys.values() for k in ks}
        self.ops = dict(ops)
        gets = [op.kind == "get" for op in self.ops.values()]
        self.read_only = all(gets)
        if not self.read_only and any(gets):
            raise ValueError("non-read-only commands cannot contain Get operations "
                             "(command.rs:35-43)")

    @classmethod
    def from_ops(cls, rifl, key_ops, shard_of=None):
        """Command::from (command.rs:53-62): [(key, KVOp)]."""
        key_ops = list(key_ops)
        return cls(rifl, [k for k, _ in key_ops], shard_of, ops=dict(key_ops))

    def key_count(self, shard_id: int = 0) -> int:
        """command.rs:81-87."""
        return len(self.shard_to_keys.get(shard_id, []))

    def execute(self, shard_id: int, store, monitor):
        """Command::execute (command.rs:114-127): this shard's ops on the
        store, in key order, each recorded by the monitor; one
        ExecutorResult per key."""
        return [ExecutorResult(self.rifl, k,
                               store.execute_with_monitor(k, self.ops[k], self.rifl, monitor))
                for k in self.keys(shard_id)]

    def keys(self, shard_id: int = 0):
        return list(self.shard_to_keys.get(shard_id, []))

    def shards(self):
        return sorted(self.shard_to_keys)

    def replicated_by(self, shard_id: int) -> bool:
        return shard_id in self.shard_to_keys

    def conflicts(self, other: "Command") -> bool:
        return any(k in other.shard_to_keys.get(s, []) for s, ks in self.shard_to_keys.items()
                   for k in ks)

    def __repr__(self):
        return f"Command({self.rifl!r}, {self.shard_to_keys!r})"
