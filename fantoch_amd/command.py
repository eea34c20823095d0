"""Minimal Command (fantoch/src/command.rs:11-156) for the host mirror.

Only what the dependency path reads: the rifl, and the keys per shard
(Command::keys, :95-100; shards, :108-110).  Keys are strings as in fantoch
and are interned to dense ids by the KeyDeps / executor mirrors.
"""
from __future__ import annotations


class Command:
    """read_only: every op is a read (Command::read_only, command.rs:65-67)."""
    __slots__ = ("rifl", "shard_to_keys", "read_only")

    def __init__(self, rifl, keys, shard_of=None, read_only: bool = False):
        self.rifl = rifl
        self.read_only = read_only
        self.shard_to_keys = {}
        for k in keys:
            s = shard_of(k) if shard_of else 0
            self.shard_to_keys.setdefault(s, [])
            if k not in self.shard_to_keys[s]:
                self.shard_to_keys[s].append(k)

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
