"""Caesar's KeyClocks on the device (fh_keyclocks_*) against the reference's
known-answer tests (clock_test, predecessors_test: tests/golden/key_clocks.json)
and against the oracle restatement (oracle/keyclocks.py) on random operation
sequences; then the device's predecessors feed the device's predecessors
executor (fh_pred_*) end to end."""
import numpy as np
import pytest

from conftest import D, load_golden
from fantoch_amd import _lib as L
from fantoch_amd.keyclocks import HipKeyClocks, clock
from fantoch_amd.pred import HipPredecessorsExecutor, PredecessorsExecutionInfo
from oracle import oracle as O
from oracle.keyclocks import KeyClocks
from test_oracle_keyclocks import run_clock, run_golden

pytestmark = pytest.mark.gpu


def test_predecessors_golden():
    g = load_golden("key_clocks.json")
    run_golden(HipKeyClocks(g["process_id"], g["shard_id"]), g)


def test_clock_golden():
    g = load_golden("key_clocks.json")
    run_clock(HipKeyClocks(g["process_id"], g["shard_id"]), g)


def test_invariants_leave_state_unchanged():
    kc = HipKeyClocks(1, key_space=16)
    kc.add(D((1, 1)), ["A", "B"], clock(5, 1))
    assert len(kc) == 2
    with pytest.raises(L.FhError) as e:
        kc.add(D((1, 2)), ["B"], clock(5, 1))   # the same timestamp on B
    assert e.value.status == L.FH_EINVARIANT and len(kc) == 2
    with pytest.raises(L.FhError):
        kc.remove(["A"], clock(6, 1))           # never added
    assert len(kc) == 2
    with pytest.raises(L.FhError):
        kc.predecessors(D((2, 7)), ["A"], clock(5, 1))  # another dot, same timestamp
    assert kc.predecessors(D((1, 1)), ["A"], clock(5, 1)) == set()


def test_two_dots_with_one_clock_on_different_keys():
    """`add` only rejects a repeated timestamp on one key (sequential.rs:43-56),
    so two dots may hold one clock on different keys; predecessors' HashSet<Dot>
    (:77-119) then reports both, and the same dot on several keys once (ADVICE
    r2: the merge used to drop repeats by clock alone).  The oracle agrees."""
    kc, orc = HipKeyClocks(1, key_space=16), KeyClocks(1, 0)
    for obj in (kc, orc):
        obj.add(D((1, 1)), ["A"], clock(3, 1))
        obj.add(D((2, 1)), ["B"], clock(3, 1))       # another dot, same clock, other key
        obj.add(D((3, 1)), ["A", "B"], clock(2, 1))  # one dot on both keys
    want = {D((1, 1)), D((2, 1)), D((3, 1))}
    assert orc.predecessors(D((4, 1)), ["A", "B"], clock(9, 1)) == want
    po, pd = kc.predecessors_batch([D((4, 1))], [["A", "B"]], [clock(9, 1)])
    assert sorted(pd.tolist()) == sorted(want) and len(pd) == 3
    assert pd.tolist()[0] == D((3, 1))  # ascending (clock, dot)


def test_more_than_eight_keys_is_not_implemented():
    kc = HipKeyClocks(1, key_space=64)
    keys = [f"k{i}" for i in range(9)]
    with pytest.raises(L.FhError) as e:
        kc.add(D((1, 1)), keys, clock(1, 1))
    assert e.value.status == L.FH_ENOTIMPL and len(kc) == 0
    with pytest.raises(L.FhError) as e:
        kc.predecessors(D((1, 1)), keys, clock(2, 1))
    assert e.value.status == L.FH_ENOTIMPL


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_batches_match_oracle(seed):
    """Batches of adds, removes and predecessor queries (with `higher`) over
    growing clocks -- the composite key widens on the way -- against the
    oracle applying the same operations one by one; output order = clock."""
    rng = np.random.default_rng(seed)
    kc, orc = HipKeyClocks(3, key_space=64), KeyClocks(3)
    live = {}  # clock -> (dot, keys)
    nxt = 1
    for rnd in range(12):
        n = int(rng.integers(1, 300))
        dots, keys, clocks = [], [], []
        for _ in range(n):
            c = clock(nxt, int(rng.integers(1, 6)))
            nxt += int(rng.integers(1, 1 << min(rnd * 3 + 1, 30)))
            ks = [f"k{x}" for x in rng.choice(40, size=int(rng.integers(1, 5)), replace=False)]
            d = D((int(rng.integers(1, 6)), nxt))
            dots.append(d), keys.append(ks), clocks.append(c)
            live[c] = (d, ks)
        kc.add_batch(dots, keys, clocks)
        for d, ks, c in zip(dots, keys, clocks):
            orc.add(d, ks, c)
        # remove a random subset
        gone = [c for c in live if rng.random() < 0.3]
        kc.remove_batch([live[c][1] for c in gone], gone)
        for c in gone:
            orc.remove(live.pop(c)[1], c)
        assert len(kc) == sum(len(v) for v in orc.clocks.values())
        # queries: live commands and fresh ones
        q = list(live.items())[:200]
        qd = [v[0] for _, v in q] + [D((9, i + 1)) for i in range(50)]
        qk = [v[1] for _, v in q] + [[f"k{x}" for x in rng.choice(40, 2, replace=False)]
                                       for _ in range(50)]
        qc = [c for c, _ in q] + [int(x) for x in rng.integers(0, clock(nxt + 5, 0), 50)
                                  if int(x) not in live][:50]
        qd, qk = qd[:len(qc)], qk[:len(qc)]
        (po, pd), (ho, hd) = kc.predecessors_batch(qd, qk, qc, higher=True)
        for i in range(len(qc)):
            hi = set()
            want = orc.predecessors(qd[i], qk[i], qc[i], hi)
            got = pd[po[i]:po[i + 1]].tolist()
            assert set(got) == want and len(got) == len(want)
            assert set(hd[ho[i]:ho[i + 1]].tolist()) == hi


def test_caesar_predecessors_feed_the_executor():
    """KeyClocks::predecessors -> PredecessorsGraph on the device: every
    command's deps = the lower-clock commands on its keys (all added), then
    the predecessors executor in a perturbed commit order; per-key order and
    the execution order equal the oracle's PredecessorsGraph on the oracle's
    KeyClocks deps."""
    rng = np.random.default_rng(7)
    n, nk = 3000, 200
    pid = 1 + np.arange(n) % 5
    dots = [D((int(p), int(i // 5 + 1))) for i, p in enumerate(pid)]
    clocks = [clock(i + 1, int(p)) for i, p in enumerate(pid)]
    keys = [[f"k{x}" for x in rng.choice(nk, size=2, replace=False)] for _ in range(n)]
    kc, orc = HipKeyClocks(1, key_space=nk), KeyClocks(1)
    kc.add_batch(dots, keys, clocks)
    for d, ks, c in zip(dots, keys, clocks):
        orc.add(d, ks, c)
    po, pd = kc.predecessors_batch(dots, keys, clocks)
    deps = [pd[po[i]:po[i + 1]].tolist() for i in range(n)]
    for i in range(n):
        assert set(deps[i]) == orc.predecessors(dots[i], keys[i], clocks[i])
    order = np.argsort(np.arange(n) + rng.uniform(0, 40, n), kind="stable")
    ex = HipPredecessorsExecutor(1)
    for i in order:
        ex.handle(PredecessorsExecutionInfo(dots[i], keys[i], (clocks[i] >> 8, clocks[i] & 255),
                                            deps[i]))
    assert ex.pending() == 0
    a_dots = np.asarray([dots[i] for i in order], dtype=np.uint64)
    a_clk = np.asarray([clocks[i] for i in order], dtype=np.uint64)
    off = np.zeros(n + 1, dtype=np.uint32)
    flat = []
    for j, i in enumerate(order):
        flat.extend(sorted(deps[i]))
        off[j + 1] = len(flat)
    want, pending = O.pred_run(a_dots, a_clk, off, np.asarray(flat, dtype=np.uint64))
    assert pending == 0
    # parity = each key's execution sequence (the interleaving across keys
    # depends on batching: the reference's is the order commits arrive in)
    keys_of = {d: ks for d, ks in zip(dots, keys)}
    clock_of = {d: c for d, c in zip(dots, clocks)}

    def per_key(seq):
        out = {}
        for d in seq:
            for k in keys_of[int(d)]:
                out.setdefault(k, []).append(int(d))
        return out
    got = per_key(ex.executed_order)
    assert got == per_key(want)
    for k, seq in got.items():  # Caesar: a key's commands run in clock order
        assert [clock_of[d] for d in seq] == sorted(clock_of[d] for d in seq)
