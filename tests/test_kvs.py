"""KV execution: the reference's known-answer tests for
KVStore (store_flow, fantoch/src/kvs.rs:71-150) and Command::conflicts
(command.rs:229-262), the executor's per-key results (Command::execute,
command.rs:114-127) and their aggregation for clients (AggregatePending,
executor/aggregate.rs:9-99)."""
import pytest

from fantoch_amd.command import Command
from fantoch_amd.kvs import AggregatePending, ExecutorResult, KVOp, KVStore


def test_store_flow():
    """kvs.rs:75-149, verbatim."""
    a, b, x, y, z = "A", "B", "x", "y", "z"
    s = KVStore()
    assert s.execute(a, KVOp.get()) is None
    assert s.execute(b, KVOp.get()) is None
    assert s.execute(a, KVOp.put(x)) is None
    assert s.execute(a, KVOp.get()) == x
    assert s.execute(b, KVOp.put(y)) is None
    assert s.execute(b, KVOp.get()) == y
    assert s.execute(a, KVOp.put(z)) == x
    assert s.execute(a, KVOp.get()) == z
    assert s.execute(b, KVOp.get()) == y
    assert s.execute(a, KVOp.delete()) == z
    assert s.execute(a, KVOp.get()) is None
    assert s.execute(b, KVOp.get()) == y
    assert s.execute(b, KVOp.delete()) == y
    assert s.execute(b, KVOp.get()) is None
    assert s.execute(a, KVOp.get()) is None
    assert s.execute(a, KVOp.put(x)) is None
    assert s.execute(a, KVOp.get()) == x
    assert s.execute(b, KVOp.get()) is None
    assert s.execute(a, KVOp.delete()) == x
    assert s.execute(a, KVOp.get()) is None


def multi_put(rifl, keys):
    """command.rs:222-227."""
    return Command.from_ops(rifl, [(k, KVOp.put(k)) for k in keys])


def test_conflicts():
    """command.rs:229-262, verbatim."""
    r = (1, 1)
    ca, cb, cc, cab = multi_put(r, ["A"]), multi_put(r, ["B"]), multi_put(r, ["C"]), \
        multi_put(r, ["A", "B"])
    assert ca.conflicts(ca) and not ca.conflicts(cb) and not ca.conflicts(cc) and ca.conflicts(cab)
    assert not cb.conflicts(ca) and cb.conflicts(cb) and not cb.conflicts(cc) and cb.conflicts(cab)
    assert not cc.conflicts(ca) and not cc.conflicts(cb) and cc.conflicts(cc) and not cc.conflicts(cab)
    assert cab.conflicts(ca) and cab.conflicts(cb) and not cab.conflicts(cc) and cab.conflicts(cab)


def test_mixed_gets_and_writes_rejected():
    """command.rs:35-43: a non-read-only command cannot contain a Get."""
    with pytest.raises(ValueError):
        Command.from_ops((1, 1), [("A", KVOp.get()), ("B", KVOp.put("v"))])
    assert Command.from_ops((1, 1), [("A", KVOp.get()), ("B", KVOp.get())]).read_only


def test_execute_results_monitor_and_aggregation():
    """Command::execute on one shard's keys, in the order the executor
    drains; AggregatePending joins the per-key results of each command."""
    store, mon = KVStore(), {}
    shard_of = lambda k: 0 if k in ("A", "B") else 1  # noqa: E731
    c1 = Command.from_ops((1, 1), [("A", KVOp.put("1")), ("B", KVOp.put("1")),
                                   ("C", KVOp.put("1"))], shard_of)
    c2 = Command.from_ops((2, 1), [("A", KVOp.put("2"))], shard_of)
    c3 = Command.from_ops((3, 1), [("A", KVOp.get()), ("B", KVOp.get())], shard_of)
    agg = AggregatePending(process_id=1, shard_id=0)
    for c in (c1, c2, c3):
        agg.wait_for(c)
    out = []
    for c in (c1, c2, c3):
        for r in c.execute(0, store, mon):
            assert isinstance(r, ExecutorResult)
            done = agg.add_executor_result(r)
            if done is not None:
                out.append((done.rifl, dict(done.results)))
    # shard 0 holds A and B only: c1 reports 2 keys, C lives on shard 1
    assert out == [((1, 1), {"A": None, "B": None}), ((2, 1), {"A": "1"}),
                   ((3, 1), {"A": "2", "B": "1"})]
    assert mon == {"A": [(1, 1), (2, 1), (3, 1)], "B": [(1, 1), (3, 1)]}
    # results of commands nobody waits for are ignored
    assert agg.add_executor_result(ExecutorResult((9, 9), "A", None)) is None
