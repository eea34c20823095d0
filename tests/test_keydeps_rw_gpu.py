"""LockedKeyDeps' read/write rules on the GPU (fh_keydeps_add_batch_rw,
csrc/keydeps.hip: segmented prefix-max scans over the key-sorted batch)
against the oracle (fo_lkeydeps_*, locked.rs:83-185), bit-exact per
command, across batches, with noops and `past`."""
import numpy as np
import pytest

from conftest import D, Interner, UD, load_golden
from fantoch_amd.command import Command
from fantoch_amd.keydeps import HipKeyDeps
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_key_deps_flow_write_only_golden():
    """key_deps_flow::<LockedKeyDeps> (keys/mod.rs:86-88)"""
    g = load_golden("key_deps_flow.json")
    kd = HipKeyDeps(g["shard_id"], key_space=16, read_write=True)
    for step in g["steps"]:
        if step["op"] == "add_cmd":
            kd.add_cmd(D(step["dot"]), Command(None, step["keys"]), None)
        elif step["op"] == "add_noop":
            kd.add_noop(D(step["dot"]))
        for what, want in step["expect"].items():
            want = {D(x) for x in want}
            got = kd.noop_deps() if what == "noop" else kd.cmd_deps(g["commands"][what])
            assert got == want, (step["dot"], what, [UD(x) for x in got])


def test_read_write_rules_by_hand():
    """the hand-derived cases of tests/test_oracle_rw.py, through add_cmd"""
    kd = HipKeyDeps(0, key_space=16, read_write=True)
    d = lambda s: O.dot(1, s)  # noqa: E731
    R = lambda s, ks: Command(s, ks, read_only=True)  # noqa: E731
    W = lambda s, ks: Command(s, ks)  # noqa: E731
    assert kd.add_cmd(d(1), W(1, ["A"])) == set()
    assert kd.add_cmd(d(2), R(2, ["A"])) == {d(1)}
    assert kd.add_cmd(d(3), R(3, ["A"])) == {d(1)}
    assert kd.add_cmd(d(4), W(4, ["A"])) == {d(3), d(1)}
    assert kd.add_cmd(d(5), R(5, ["A"])) == {d(4)}
    assert kd.add_cmd(d(6), W(6, ["A"])) == {d(5), d(4)}
    assert kd.add_cmd(d(7), W(7, ["A"])) == {d(5), d(6)}
    assert kd.add_cmd(d(8), R(8, ["A", "B"])) == {d(7)}
    assert kd.cmd_deps(["A"]) == {d(8), d(7)}
    assert kd.add_noop(d(9)) == {d(8), d(7)}
    assert kd.add_cmd(d(10), W(10, ["B"])) == {d(8), d(9)}
    assert kd.add_cmd(d(11), R(11, ["A"]), past=[O.dot(2, 1)]) == {d(7), d(9), O.dot(2, 1)}
    assert kd.noop_deps() == {d(9), d(11), d(7), d(10), d(8)}


@pytest.mark.parametrize("n,keys,k,reads,batches", [
    (30_000, 64, 1, 0.5, 4),        # hot keys: long segments, scans across tiles
    (60_000, 4096, 3, 0.3, 3),      # multi-key commands
    (20_000, 512, 2, 0.9, 5),       # mostly reads
])
def test_random_streams_match_oracle(n, keys, k, reads, batches):
    rng = np.random.default_rng(n + keys)
    dots = np.asarray([O.dot(1 + i % 5, 1 + i // 5) for i in range(n)], dtype=np.uint64)
    cmd_keys = [rng.choice(keys, size=k, replace=False).tolist() for _ in range(n)]
    ro = rng.random(n) < reads
    noop = rng.random(n) < 0.002
    with_past = rng.random(n) < 0.05
    past = [[int(dots[max(0, i - 1 - j)]) for j in range(2)] if with_past[i] and i else []
            for i in range(n)]
    ok = O.LockedKeyDeps(0)
    want = []
    for i in range(n):
        if noop[i]:
            want.append(sorted(ok.add_noop(int(dots[i]))))
        else:
            want.append(sorted(ok.add_cmd(int(dots[i]), cmd_keys[i], bool(ro[i]),
                                          past[i] if with_past[i] and i else None)))
    kd = HipKeyDeps(0, key_space=keys, intern=False, read_write=True)
    bounds = np.linspace(0, n, batches + 1).astype(int)
    got = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        has_past = bool(with_past[a:b].any())
        off, deps = kd.add_batch(dots[a:b], [[] if noop[i] else cmd_keys[i] for i in range(a, b)],
                                 noop[a:b], [past[i] if with_past[i] and i else []
                                             for i in range(a, b)] if has_past else None,
                                 read_only=ro[a:b])
        got.extend(deps[off[j]:off[j + 1]].tolist() for j in range(b - a))
    for i in range(n):
        assert got[i] == want[i], (i, bool(ro[i]), bool(noop[i]))
    assert kd.noop_deps() == ok.noop_deps()
    for key in range(min(keys, 64)):
        assert kd.cmd_deps([key]) == ok.cmd_deps([key])
