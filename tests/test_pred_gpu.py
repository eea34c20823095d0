"""Caesar's predecessors executor on the GPU (fh_pred_*, csrc/pred.hip) against
the oracle restatement of PredecessorsGraph (fantoch_ps/src/executor/pred/
mod.rs:26-352): the reference's known-answer tests, add-order permutations,
and large Caesar-shaped streams in batches (per-key execution sequences, the
executed set and the pending set)."""
import os
import sys

import numpy as np
import pytest

from fantoch_amd import _lib as L
from fantoch_amd.pred import HipPredecessorsExecutor, PredecessorsExecutionInfo
from oracle import oracle as O

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from caesar_gen import caesar_stream, per_key  # noqa: E402

pytestmark = pytest.mark.gpu
D = O.dot


def test_simple():
    """mod.rs:386-426"""
    ex = HipPredecessorsExecutor(1, device=0)
    d0, d1 = D(1, 1), D(2, 1)
    ex.handle(PredecessorsExecutionInfo(d0, ["A"], (2, 1), [d1]))
    assert getattr(ex, "executed_order", []) == []
    ex.handle(PredecessorsExecutionInfo(d1, ["A"], (1, 2), [d0]))
    assert ex.executed_order == [d1, d0]
    assert ex.pending() == 0
    assert ex.monitor() == {"A": [d1, d0]}


def test_already_mutably_borrowed_regression():
    """mod.rs:428-489"""
    ex = HipPredecessorsExecutor(1, device=0)
    d21, d11, d31 = D(2, 1), D(1, 1), D(3, 1)
    ex.handle(PredecessorsExecutionInfo(d21, ["2", "conflict"], (2, 3), [d11, d21, d31]))
    ex.handle(PredecessorsExecutionInfo(d11, ["1", "conflict"], (2, 2), [d11, d21, d31]))
    assert getattr(ex, "executed_order", []) == []
    ex.handle(PredecessorsExecutionInfo(d31, ["3", "conflict"], (1, 3), [d11, d21]))
    assert ex.executed_order == [d31, d11, d21]


def _gpu_run(s, bounds):
    ex = HipPredecessorsExecutor(1, device=0)
    for a, b in zip(bounds[:-1], bounds[1:]):
        ex.handle_batch([PredecessorsExecutionInfo(int(s["dots"][j]), s["keys"][j].tolist(),
                                                   int(s["clocks"][j]),
                                                   s["deps"][s["dep_off"][j]:s["dep_off"][j + 1]])
                         for j in range(a, b)])
    return getattr(ex, "executed_order", []), ex.pending()


def test_add_order_permutations_match_oracle():
    rng = np.random.default_rng(3)
    for seed in range(6):
        s = caesar_stream(6, 4, 2, seed=seed, nproc=2, window=6)
        for _ in range(20):
            perm = rng.permutation(6)
            t = {k: (v[perm] if k in ("dots", "clocks", "keys") else v) for k, v in s.items()}
            off = s["dep_off"]
            t["deps"] = np.concatenate([s["deps"][off[j]:off[j + 1]] for j in perm])
            t["dep_off"] = np.concatenate([[0], np.cumsum([off[j + 1] - off[j] for j in perm])]
                                          ).astype(np.uint32)
            want, _ = O.pred_run(t["dots"], t["clocks"], t["dep_off"], t["deps"])
            got, pend = _gpu_run(t, list(range(7)))
            assert pend == 0
            assert per_key(got, t["dots"], t["keys"]) == per_key(want, t["dots"], t["keys"])


@pytest.mark.parametrize("drop", [0, 25])
def test_caesar_stream_in_batches_matches_oracle(drop):
    s = caesar_stream(20_000, 512, 2, seed=11 + drop, window=64, drop=drop)
    n = len(s["dots"])
    want, want_pending = O.pred_run(s["dots"], s["clocks"], s["dep_off"], s["deps"])
    bounds = [0, 1, 700, 5000, 5001, 12_000, n]
    got, pending = _gpu_run(s, bounds)
    assert pending == want_pending
    assert sorted(got) == sorted(want.tolist())
    assert per_key(got, s["dots"], s["keys"]) == per_key(want, s["dots"], s["keys"])
    if drop:
        assert pending > 0


def test_readded_dot_is_rejected_without_state_change():
    ex = HipPredecessorsExecutor(1, device=0)
    d1, d2 = D(1, 1), D(1, 2)
    ex.handle(PredecessorsExecutionInfo(d1, ["A"], (1, 1), []))
    with pytest.raises(L.FhError):
        ex.handle(PredecessorsExecutionInfo(d1, ["A"], (5, 1), []))
    with pytest.raises(L.FhError):  # duplicate inside one batch
        ex.handle_batch([PredecessorsExecutionInfo(d2, ["A"], (2, 1), [d1]),
                         PredecessorsExecutionInfo(d2, ["A"], (3, 1), [d1])])
    ex.handle(PredecessorsExecutionInfo(d2, ["A"], (2, 1), [d1]))
    assert ex.executed_order == [d1, d2]
