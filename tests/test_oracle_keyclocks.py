"""The KeyClocks oracle (oracle/keyclocks.py) against the reference's own
known-answer tests: clock_test and predecessors_test
(fantoch_ps/src/protocol/common/pred/clocks/keys/sequential.rs:167-),
transcribed in tests/golden/key_clocks.json."""
import pytest

from conftest import D, load_golden
from oracle.keyclocks import KeyClocks, clock


def run_golden(kc, g):
    for op in g["predecessors_test"]:
        c = clock(*op["clock"])
        if op["op"] == "add":
            kc.add(D(op["dot"]), op["keys"], c)
        elif op["op"] == "remove":
            kc.remove(op["keys"], c)
        else:
            blocking = set()
            preds = kc.predecessors(D(op["dot"]), op["keys"], c, blocking)
            assert blocking == {D(x) for x in op["blocking"]}, op
            assert preds == {D(x) for x in op["predecessors"]}, op


def run_clock(kc, g):
    for op in g["clock_test"]:
        if op["op"] == "next":
            assert kc.clock_next() == clock(*op["expect"])
        else:
            kc.clock_join(clock(*op["clock"]))


def test_oracle_predecessors_golden():
    g = load_golden("key_clocks.json")
    run_golden(KeyClocks(g["process_id"], g["shard_id"]), g)


def test_oracle_clock_golden():
    g = load_golden("key_clocks.json")
    run_clock(KeyClocks(g["process_id"], g["shard_id"]), g)


def test_oracle_invariants():
    kc = KeyClocks(1)
    kc.add(D((1, 1)), ["A"], clock(1, 1))
    with pytest.raises(AssertionError):
        kc.add(D((1, 2)), ["A"], clock(1, 1))
    with pytest.raises(AssertionError):
        kc.remove(["B"], clock(1, 1))
    with pytest.raises(AssertionError):
        kc.predecessors(D((2, 9)), ["A"], clock(1, 1))
