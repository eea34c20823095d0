"""CPU restatement of SequentialKeyClocks -- TEST INFRASTRUCTURE ONLY.

Only tests/ import this (the checker for fh_keyclocks_*); the product path is
the HIP library.  Pure Python, for small cases.  Follows
fantoch_ps/src/protocol/common/pred/clocks/keys/sequential.rs line by line:
per key a map clock -> dot (CommandsPerKey, :11-12); clocks packed
(seq << 8) | process_id so integer order is Clock's Ord (clocks/mod.rs:15-30).
Pinned by the reference's clock_test / predecessors_test
(tests/golden/key_clocks.json, tests/test_oracle_keyclocks.py).
"""
from __future__ import annotations


def clock(seq: int, pid: int) -> int:
    return (seq << 8) | pid


class KeyClocks:
    def __init__(self, process_id: int, shard_id: int = 0):
        self.process_id = process_id      # :22-30
        self.shard_id = shard_id
        self.seq = 0
        self.clocks = {}                   # key -> {clock: dot}

    def clock_next(self) -> int:          # :33-37
        self.seq += 1
        return clock(self.seq, self.process_id)

    def clock_join(self, other: int):     # :39-42
        self.seq = max(self.seq, other >> 8)

    def add(self, dot: int, keys, c: int):  # :43-56
        for k in keys:
            cmds = self.clocks.setdefault(k, {})
            assert c not in cmds, "can't add a timestamp belonging to a command already added"
            cmds[c] = dot

    def remove(self, keys, c: int):       # :58-75
        for k in keys:
            cmds = self.clocks.setdefault(k, {})
            assert cmds.pop(c, None) is not None, \
                "can't remove a timestamp belonging to a command never added"

    def predecessors(self, dot: int, keys, c: int, higher=None):  # :77-119
        preds = set()
        for k in keys:
            for cc, d in self.clocks.get(k, {}).items():
                if cc < c:
                    preds.add(d)
                elif cc > c:
                    if higher is not None:
                        higher.add(d)
                elif d != dot:
                    raise AssertionError("found different command with the same timestamp")
        return preds
