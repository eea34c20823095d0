"""concurrent_test (fantoch_ps/src/protocol/common/graph/deps/keys/mod.rs:
331-471) against HipKeyDeps(read_write=True), the LockedKeyDeps drop-in: two
threads share one instance (parallel() is true; every call holds the
instance's lock, as LockedKeyDeps' clones share its locked table), each adds
3000 commands of 1-2 keys out of 4 from its own DotGen (process ids 1 and 2,
fantoch/src/id.rs:88-91).  Invariant: every two conflicting commands have a
dependency path one way or the other.

The reference's gen_cmd (fantoch_ps/src/util.rs:28-51) ignores its noop
probability and issues writes only; the first case ports exactly that.  Its
is_dep recursion revisits the same dot, so it passes any command with a
non-empty dependency set; here the path check is a real search over the
gathered dependency sets.  The second case adds what the reference's test
leaves out: noops (which conflict with everything, keys/mod.rs:393-401) and
read-only commands, which LockedKeyDeps does not connect to every later write
(tests/concurrent_check.py), so only the writes' pairs are checked there."""
import threading

import pytest

from concurrent_check import check_conflicts_ordered, worker
from fantoch_amd.keydeps import HipKeyDeps

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("noop_pct,read_pct,rounds", [(0, 0, 10), (20, 40, 4)])
def test_concurrent_locked_key_deps(noop_pct, read_pct, rounds):
    for r in range(rounds):
        kd = HipKeyDeps(0, key_space=16, read_write=True)
        assert kd.parallel()
        out = {}
        ts = [threading.Thread(target=worker,
                               args=(kd, p, 3000, 2, 4, noop_pct, read_pct, 1000 * r + p, out))
              for p in (1, 2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        kd.close()
        cmds, deps = {}, {}
        for p in (1, 2):
            for dot, cmd, ds in out[p]:
                assert dot not in cmds
                cmds[dot] = cmd
                deps[dot] = ds
        check_conflicts_ordered(cmds, deps)


def test_sequential_key_deps_is_not_parallel():
    kd = HipKeyDeps(0, key_space=16)
    assert not kd.parallel()
    kd.close()
