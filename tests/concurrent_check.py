"""Shared by tests/test_keydeps_concurrent_gpu.py (HipKeyDeps on the GPU) and
tests/test_concurrent_check.py (the same checker against the oracle's
LockedKeyDeps on the CPU): the concurrent_test worker and its invariant
(fantoch_ps/src/protocol/common/graph/deps/keys/mod.rs:331-471)."""
import random

from fantoch_amd.command import Command
from oracle import oracle as O


def worker(kd, process_id, ops, max_keys, keys_number, noop_pct, read_pct, seed, out):
    rng = random.Random(seed)
    res = []
    for seq in range(1, ops + 1):
        dot = O.dot(process_id, seq)
        if rng.randrange(100) < noop_pct:
            res.append((dot, None, kd.add_noop(dot)))
            continue
        nk = rng.randrange(1, max_keys + 1)
        ks = sorted({str(rng.randrange(keys_number)) for _ in range(nk)})
        cmd = Command((process_id, seq), ks, read_only=rng.randrange(100) < read_pct)
        res.append((dot, cmd, kd.add_cmd(dot, cmd, None)))
    out[process_id] = res


def closures(dots, deps):
    """Dependency closure of every dot as a bit set (Python int over dot
    indices): the deps only name earlier calls (one locked instance), so the
    graph is acyclic and a memoised post-order visit suffices."""
    idx = {d: i for i, d in enumerate(dots)}
    clo = {}
    for root in dots:
        if root in clo:
            continue
        st = [(root, iter(deps[root]))]
        while st:
            d, it = st[-1]
            nxt = next((x for x in it if x in idx and x not in clo), None)
            if nxt is not None:
                st.append((nxt, iter(deps[nxt])))
                continue
            st.pop()
            m = 0
            for x in deps[d]:
                if x in idx:
                    m |= clo[x] | (1 << idx[x])
            clo[d] = m
    return idx, clo


def check_conflicts_ordered(cmds, deps):
    """Every two conflicting writes (noops write every key) are connected one
    way: per key, the writers must form one chain under reachability --
    checked on consecutive members after sorting by closure size, which
    transitivity extends to every pair.  That is the reference's pairwise
    check (keys/mod.rs:389-418) in O(n log n) per key, for the commands its
    gen_cmd issues (writes only).  Reads are left out of the pairs:
    LockedKeyDeps orders a write after the key's latest read only
    (locked.rs:83-128), so an earlier read and a later write of one key may
    stay unconnected (write 1, reads 2 and 3, write 4: 4 -> {3, 1},
    2 -> {1}); the reads still must not break the writers' chain."""
    dots = sorted(cmds)
    idx, clo = closures(dots, deps)
    keys = sorted({k for c in cmds.values() if c is not None for k in c.keys()})
    for k in keys:
        writers = [d for d in dots if cmds[d] is None or
                   (k in cmds[d].keys() and not cmds[d].read_only)]
        writers.sort(key=lambda d: bin(clo[d]).count("1"))
        for a, b in zip(writers, writers[1:]):
            assert clo[b] >> idx[a] & 1, f"writers {a:#x} / {b:#x} of key {k} not connected"
