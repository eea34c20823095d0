"""The CPU restatement of Caesar's PredecessorsGraph (oracle/oracle.c,
fo_pred_*) against the reference's own tests (fantoch_ps/src/executor/pred/
mod.rs:386-687), transcribed: `simple`, `already_mutably_borrowed_regression
_test` (exact execution order), and test_add_random's invariant -- every
permutation of the adds gives the same per-key order."""
import itertools
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from caesar_gen import caesar_stream, per_key  # noqa: E402
from oracle import oracle as O  # noqa: E402

D = O.dot
CLK = O.clock


def test_simple():
    """mod.rs:386-426"""
    p = O.Pred(1)
    d0, d1 = D(1, 1), D(2, 1)
    p.add(d0, CLK(2, 1), [d1])
    assert p.drain() == []
    p.add(d1, CLK(1, 2), [d0])
    assert p.drain() == [d1, d0]
    assert p.pending() == 0


def test_already_mutably_borrowed_regression():
    """mod.rs:428-489: commands may depend on themselves"""
    p = O.Pred(1)
    d21, d11, d31 = D(2, 1), D(1, 1), D(3, 1)
    p.add(d21, CLK(2, 3), [d11, d21, d31])
    assert p.drain() == []
    p.add(d11, CLK(2, 2), [d11, d21, d31])
    assert p.drain() == []
    p.add(d31, CLK(1, 3), [d11, d21])
    assert p.drain() == [d31, d11, d21]


def _run(order, s):
    p = O.Pred(1)
    out = []
    for j in order:
        p.add(int(s["dots"][j]), int(s["clocks"][j]), s["deps"][s["dep_off"][j]:s["dep_off"][j + 1]])
        out.extend(p.drain())
    assert p.pending() == 0
    return per_key(out, s["dots"], s["keys"])


def test_add_random_permutations():
    """mod.rs:491-687: n=2 processes x 3 events, two of four keys per command
    (non-transitive conflicts), random unique clocks; all 720 add orders give
    the same per-key order, which is clock order."""
    for seed in range(10):
        s = caesar_stream(6, 4, 2, seed=seed, nproc=2, window=6)
        want = None
        for perm in itertools.permutations(range(6)):
            got = _run(perm, s)
            if want is None:
                want = got
            assert got == want, (seed, perm)
        clock_of = dict(zip(s["dots"].tolist(), s["clocks"].tolist()))
        for key, seq in want.items():
            assert [clock_of[d] for d in seq] == sorted(clock_of[d] for d in seq)


def test_uncommitted_dependency_keeps_dependents_pending():
    s = caesar_stream(300, 16, 2, seed=5, drop=3)
    order, pending = O.pred_run(s["dots"], s["clocks"], s["dep_off"], s["deps"])
    assert pending > 0 and len(order) + pending == len(s["dots"])
    # no executed command has a lower-clock dependency that did not execute
    done = set(order.tolist())
    clock_of = dict(zip(s["dots"].tolist(), s["clocks"].tolist()))
    for j, d in enumerate(s["dots"].tolist()):
        if d not in done:
            continue
        for x in s["deps"][s["dep_off"][j]:s["dep_off"][j + 1]].tolist():
            assert x in clock_of, "an executed command waits for every dep to commit"
            if clock_of[x] < clock_of[d]:
                assert x in done
