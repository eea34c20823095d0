"""LockedKeyDeps' read/write rules in the oracle (fo_lkeydeps_*,
fantoch_ps/src/protocol/common/graph/deps/keys/locked.rs:83-185).

The reference pins LockedKeyDeps only on write-only commands
(key_deps_flow::<LockedKeyDeps>, keys/mod.rs:86-88) -- checked here against
the same golden flow as SequentialKeyDeps.  The read rules have no
known-answer test in the reference; the cases below are derived by hand from
locked.rs:100-117 (a read depends on the latest write and becomes the latest
read; a write depends on the latest read and the latest write and becomes
the latest write, leaving the latest read in place) and :130-169 (noops)."""
import random

from conftest import D, Interner, UD, load_golden
from oracle import oracle as O


def test_key_deps_flow_write_only():
    g = load_golden("key_deps_flow.json")
    kd = O.LockedKeyDeps(g["shard_id"])
    ik = Interner()
    cmds = {name: ik.many(keys) for name, keys in g["commands"].items()}
    for step in g["steps"]:
        if step["op"] == "add_cmd":
            kd.add_cmd(D(step["dot"]), ik.many(step["keys"]))
        elif step["op"] == "add_noop":
            kd.add_noop(D(step["dot"]))
        for what, want in step["expect"].items():
            want = {D(x) for x in want}
            got = kd.noop_deps() if what == "noop" else kd.cmd_deps(cmds[what])
            assert got == want, (step, what, [UD(x) for x in got])


def test_read_write_rules_by_hand():
    kd = O.LockedKeyDeps(0)
    d = lambda s: O.dot(1, s)  # noqa: E731
    A, B = 0, 1
    assert kd.add_cmd(d(1), [A]) == set()                       # W1(A)
    assert kd.add_cmd(d(2), [A], read_only=True) == {d(1)}      # R2: latest write
    assert kd.add_cmd(d(3), [A], read_only=True) == {d(1)}      # R3: reads don't chain
    assert kd.add_cmd(d(4), [A]) == {d(3), d(1)}                # W4: latest read + write
    assert kd.add_cmd(d(5), [A], read_only=True) == {d(4)}
    assert kd.add_cmd(d(6), [A]) == {d(5), d(4)}
    assert kd.add_cmd(d(7), [A]) == {d(5), d(6)}                # the latest read stays
    assert kd.add_cmd(d(8), [A, B], read_only=True) == {d(7)}   # B has no write
    assert kd.cmd_deps([A]) == {d(8), d(7)}
    assert kd.add_noop(d(9)) == {d(8), d(7)}                    # every latest read/write
    assert kd.add_cmd(d(10), [B]) == {d(8), d(9)}               # read of B + the noop
    assert kd.add_cmd(d(11), [A], read_only=True, past=[O.dot(2, 1)]) == {d(7), d(9),
                                                                          O.dot(2, 1)}
    assert kd.noop_deps() == {d(9), d(11), d(7), d(10), d(8)}


def test_write_only_streams_equal_sequential():
    rng = random.Random(5)
    seq, locked = O.KeyDeps(0), O.LockedKeyDeps(0)
    for i in range(1, 3000):
        dot = O.dot(1 + i % 5, i)
        if rng.random() < 0.01:
            assert seq.add_noop(dot) == locked.add_noop(dot)
        else:
            keys = rng.sample(range(40), rng.randint(1, 3))
            assert seq.add_cmd(dot, keys) == locked.add_cmd(dot, keys)
