"""The concurrent_test checker (tests/concurrent_check.py) on the CPU: two
threads drive the oracle's LockedKeyDeps (locked.rs:10-186) behind one lock,
as LockedKeyDeps' clones share its locked table; the invariant must hold, and
it must catch a dropped dependency."""
import threading

import pytest

from concurrent_check import check_conflicts_ordered, worker
from oracle import oracle as O


class LockedOracle:
    """The oracle's LockedKeyDeps with the add_cmd(dot, cmd, past) shape."""

    def __init__(self):
        self.kd = O.LockedKeyDeps(0)
        self.lock = threading.Lock()
        self.ids = {}

    def add_cmd(self, dot, cmd, past):
        with self.lock:
            ks = [self.ids.setdefault(k, len(self.ids)) for k in cmd.keys()]
            return self.kd.add_cmd(dot, ks, read_only=cmd.read_only)

    def add_noop(self, dot):
        with self.lock:
            return self.kd.add_noop(dot)


def run(noop_pct, read_pct, seed):
    kd = LockedOracle()
    out = {}
    ts = [threading.Thread(target=worker, args=(kd, p, 3000, 2, 4, noop_pct, read_pct,
                                                seed + p, out)) for p in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    cmds, deps = {}, {}
    for p in (1, 2):
        for dot, cmd, ds in out[p]:
            cmds[dot] = cmd
            deps[dot] = ds
    return cmds, deps


@pytest.mark.parametrize("noop_pct,read_pct", [(0, 0), (20, 40)])
def test_oracle_locked_key_deps_satisfies_invariant(noop_pct, read_pct):
    cmds, deps = run(noop_pct, read_pct, 7)
    check_conflicts_ordered(cmds, deps)


def test_checker_catches_a_dropped_dependency():
    cmds, deps = run(0, 0, 11)
    # drop one dependency of a late command: the pair loses its only path
    victim = max(d for d in deps if deps[d])
    dep = next(iter(deps[victim]))
    deps[victim] = deps[victim] - {dep}
    with pytest.raises(AssertionError):
        check_conflicts_ordered(cmds, deps)
