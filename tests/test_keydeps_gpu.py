"""KeyDeps on the GPU (fh_keydeps_* through the C ABI) against the oracle and
the reference's key_deps_flow known answers.  Bit-exact dep sets."""
import numpy as np
import pytest

from conftest import D, Interner, UD, load_golden
from fantoch_amd.keydeps import Dependency, HipKeyDeps
from fantoch_amd.workload import Workload
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_key_deps_flow_golden():
    """deps/keys/mod.rs:98-329 through the per-call trait mirror."""
    g = load_golden("key_deps_flow.json")
    kd = HipKeyDeps(g["shard_id"], key_space=16)
    cmds = {name: keys for name, keys in g["commands"].items()}
    for step in g["steps"]:
        if step["op"] == "add_cmd":
            kd.add_cmd(D(step["dot"]), step["keys"], None)
        elif step["op"] == "add_noop":
            kd.add_noop(D(step["dot"]))
        for what, want in step["expect"].items():
            want = {D(x) for x in want}
            got = kd.noop_deps() if what == "noop" else kd.cmd_deps(cmds[what])
            assert got == want, (step["dot"], what, [UD(x) for x in got])


def test_add_cmd_returns_sequential_deps_and_past_union():
    kd = HipKeyDeps(0, key_space=64)
    a, b, c = D([1, 1]), D([2, 1]), D([1, 2])
    assert kd.add_cmd(a, ["x"]) == set()
    assert kd.add_cmd(b, ["x", "y"]) == {a}
    past = {D([3, 7]), D([4, 2])}
    assert kd.add_cmd(c, ["y"], past) == past | {b}
    assert kd.add_noop(D([5, 1])) == {b, c}
    assert kd.add_cmd(D([5, 2]), ["z"]) == {D([5, 1])}


class _Cmd:
    """keys(shard) / shards() of a command (fantoch/src/command.rs:95-110)."""

    def __init__(self, keys, shards):
        self._keys, self._shards = keys, shards

    def keys(self, shard_id):
        return self._keys

    def shards(self):
        return self._shards


def test_returned_deps_keep_their_shards():
    """add_cmd(B) returns exactly the dot B displaced from x's slot, so the
    Dependency values of that result still carry A's shards
    (Dependency::from_cmd, keys/mod.rs:25-30), as the Rust shim builds them
    before set_slot (fantoch_hip/src/keydeps.rs)."""
    kd = HipKeyDeps(0, key_space=64)
    a, b, n = D([1, 1]), D([2, 1]), D([3, 1])
    assert kd.add_cmd(a, _Cmd(["x"], [0, 2])) == set()
    deps = kd.add_cmd(b, _Cmd(["x"], [0]))
    assert deps == {a}
    assert kd.dependencies(deps) == {Dependency(a, frozenset({0, 2}))}
    # a noop's deps carry the shards of the key slots it read
    nd = kd.add_noop(n)
    assert kd.dependencies(nd) == {Dependency(b, frozenset({0}))}


def _oracle_csr(dots, key_off, keys, is_noop=None):
    off, deps = O.keydeps_run(dots, key_off, keys, is_noop)
    return off, deps


def _check_same(off_a, dep_a, off_b, dep_b):
    assert np.array_equal(off_a, off_b)
    assert np.array_equal(dep_a, dep_b)


@pytest.mark.parametrize("k,batches", [(1, 1), (1, 4), (2, 3), (3, 1)])
def test_batches_match_oracle_zipf(k, batches):
    w = Workload.zipf(0.99, 5000, k=k, seed=11 + k)
    s = w.generate(40_000)
    key_off = s.key_off()
    keys = s.keys.reshape(-1)
    want_off, want = _oracle_csr(s.dots, key_off, keys)
    kd = HipKeyDeps(0, key_space=s.key_space, intern=False)
    bounds = np.linspace(0, s.n, batches + 1).astype(int)
    got_off = [0]
    got = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        off, deps = kd.add_batch(s.dots[a:b], (key_off[a:b + 1] - key_off[a], keys[key_off[a]:key_off[b]]))
        got.append(deps)
        got_off.extend((off[1:] + got_off[-1]).tolist())
    _check_same(np.asarray(got_off, dtype=np.uint32), np.concatenate(got), want_off, want)


def test_noops_and_variable_keys_match_oracle():
    rng = np.random.default_rng(5)
    n = 3000
    dots = np.array([D([1 + i % 3, 1 + i // 3]) for i in range(n)], dtype=np.uint64)
    nk = rng.integers(1, 4, size=n)
    is_noop = (rng.random(n) < 0.01).astype(np.uint8)
    nk[is_noop == 1] = 0
    key_off = np.zeros(n + 1, dtype=np.uint32)
    key_off[1:] = np.cumsum(nk)
    keys = np.concatenate([rng.choice(50, size=c, replace=False) for c in nk]).astype(np.uint64)
    want_off, want = _oracle_csr(dots, key_off, keys, is_noop)
    kd = HipKeyDeps(0, key_space=50, intern=False)
    off, deps = kd.add_batch(dots, (key_off, keys), is_noop)
    _check_same(off, deps, want_off, want)
    # the state left behind matches too
    ok = O.KeyDeps(0)
    for i in range(n):
        if is_noop[i]:
            ok.add_noop(int(dots[i]))
        else:
            ok.add_cmd(int(dots[i]), keys[key_off[i]:key_off[i + 1]].tolist())
    assert kd.noop_deps() == ok.noop_deps()
    for key in range(50):
        assert kd.cmd_deps([key]) == ok.cmd_deps([key])


def test_past_is_unioned():
    rng = np.random.default_rng(9)
    n = 2000
    dots = np.array([D([2, 1 + i]) for i in range(n)], dtype=np.uint64)
    keys = rng.integers(0, 20, size=n).astype(np.uint64)
    key_off = np.arange(n + 1, dtype=np.uint32)
    past = [[D([7, int(x)]) for x in rng.integers(1, 100, size=rng.integers(0, 4))] for _ in range(n)]
    kd = HipKeyDeps(0, key_space=20, intern=False)
    off, deps = kd.add_batch(dots, (key_off, keys), None, past)
    ok = O.KeyDeps(0)
    for i in range(n):
        want = ok.add_cmd(int(dots[i]), [int(keys[i])], past[i])
        assert set(int(x) for x in deps[off[i]:off[i + 1]]) == want
        assert list(deps[off[i]:off[i + 1]]) == sorted(want)


def test_bad_key_is_rejected_without_state_change():
    from fantoch_amd._lib import FhError
    kd = HipKeyDeps(0, key_space=8, intern=False)
    kd.add_batch([D([1, 1])], [[3]])
    with pytest.raises(FhError):
        kd.add_batch([D([1, 2])], [[8]])
    assert kd.cmd_deps([3]) == {D([1, 1])}


def test_c2_full_size_1m_zipf07_matches_oracle():
    """BASELINE config C2 at full size: 1M cmds, Zipf 0.7 over 1M keys, 1 key."""
    w = Workload.zipf(0.7, 1 << 20, k=1)
    s = w.generate(1_000_000)
    key_off = s.key_off()
    keys = s.keys.reshape(-1)
    want_off, want = _oracle_csr(s.dots, key_off, keys)
    kd = HipKeyDeps(0, key_space=s.key_space, intern=False)
    off, deps = kd.add_batch(s.dots, (key_off, keys))
    _check_same(off, deps, want_off, want)
