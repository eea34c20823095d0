"""Caesar-shaped inputs for the predecessors executor (test data generator).

Follows the shape the reference's test_add_random builds
(fantoch_ps/src/executor/pred/mod.rs:503-610) and what
KeyClocks::predecessors reports (protocol/common/pred/clocks/keys/
sequential.rs:74-119): unique clocks; for every conflicting pair (a shared
key) the lower-clock command is a dependency of the higher-clock one, and the
higher-clock one is a dependency of the lower one with probability
`higher_p`.  Commands are committed in clock order perturbed by a window
(commit order != clock order); `drop` commands are never committed, so their
dependents stay pending.
"""
from __future__ import annotations

import numpy as np


def dot(src: int, seq: int) -> int:
    return (src << 56) | seq


def caesar_stream(n: int, n_keys: int, k: int, seed: int, nproc: int = 5, window: int = 32,
                  higher_p: float = 0.5, drop: int = 0):
    """-> dict(dots, clocks, keys [n, k], dep_off, deps) in commit (arrival)
    order, plus the dropped dots."""
    rng = np.random.default_rng(seed)
    pid = 1 + np.arange(n) % nproc
    seq = 1 + np.arange(n) // nproc
    dots = (pid.astype(np.uint64) << np.uint64(56)) | seq.astype(np.uint64)
    clocks = (np.arange(1, n + 1, dtype=np.uint64) << np.uint64(8)) | pid.astype(np.uint64)
    keys = np.stack([rng.choice(n_keys, size=k, replace=False) for _ in range(n)]).astype(np.uint64)
    deps = [set() for _ in range(n)]
    for key in range(n_keys):
        members = np.nonzero((keys == key).any(axis=1))[0]  # ascending = clock order
        for a in range(len(members)):
            i = members[a]
            deps[i].update(int(dots[j]) for j in members[:a])  # every lower clock
            hi = members[a + 1:]
            if len(hi):
                pick = hi[rng.random(len(hi)) < higher_p]
                deps[i].update(int(dots[j]) for j in pick)
    arrival = np.argsort(np.arange(n) + rng.uniform(0, window, n), kind="stable")
    dropped = set(rng.choice(n, size=drop, replace=False).tolist()) if drop else set()
    arrival = np.asarray([i for i in arrival if i not in dropped], dtype=np.int64)
    dep_off = np.zeros(len(arrival) + 1, dtype=np.uint32)
    flat = []
    for j, i in enumerate(arrival):
        flat.extend(sorted(deps[i]))
        dep_off[j + 1] = len(flat)
    return dict(dots=dots[arrival], clocks=clocks[arrival], keys=keys[arrival], dep_off=dep_off,
                deps=np.asarray(flat, dtype=np.uint64),
                dropped=[int(dots[i]) for i in sorted(dropped)])


def per_key(order, dots, keys):
    """Per-key execution sequences from an execution order of dots."""
    kmap = {int(d): [int(x) for x in ks] for d, ks in zip(dots, keys)}
    out = {}
    for d in order:
        for key in kmap[int(d)]:
            out.setdefault(key, []).append(int(d))
    return out
