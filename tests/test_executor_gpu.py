"""HipGraphExecutor (fh_graph_*) -- the GraphExecutor drop-in -- against the
reference's known-answer tests (executor/graph/mod.rs:716-1350) and against
the oracle's incremental DependencyGraph on shuffled arrival orders."""
import itertools
import json
import random

import numpy as np
import pytest

from conftest import D, load_golden
from fantoch_amd.command import Command
from fantoch_amd.executor import GraphExecutionInfo, HipGraphExecutor
from fantoch_amd.workload import Workload
from oracle import oracle as O
from test_oracle_golden import random_adds

pytestmark = pytest.mark.gpu


def check_termination(n, args, batch=1):
    """graph/mod.rs:1047-1115 through the HIP executor (per-call handle when
    batch == 1, handle_batch otherwise)."""
    ex = HipGraphExecutor(process_id=1, shard_id=0, n=n, f=1, key_space=64)
    infos = []
    for a in args:
        dot = D(a["dot"])
        keys = a["keys"] if a["keys"] is not None else ["CONF"]
        infos.append(GraphExecutionInfo.add(dot, Command(dot, keys), [D(x) for x in a["deps"]]))
    for i in range(0, len(infos), batch):
        if batch == 1:
            ex.handle(infos[i])
        else:
            ex.handle_batch(infos[i:i + batch])
    assert ex.pending() == 0, "every command executes exactly once"
    out = ex.monitor()
    assert sum(len(v) for v in out.values()) == sum(len(a["keys"] or ["CONF"]) for a in args)
    return out


def test_simple():
    g = load_golden("graph_simple.json")
    ex = HipGraphExecutor(g["process_id"], g["shard_id"], g["n"], g["f"], key_space=8)
    order = []
    for a in g["adds"]:
        dot = D(a["dot"])
        ex.handle(GraphExecutionInfo.add(dot, Command(dot, a["keys"]), [D(x) for x in a["deps"]]))
        got = []
        while (r := ex.to_clients()) is not None:
            got.append(r[0])
        assert got == [D(x) for x in a["expect_executed"]]


@pytest.mark.parametrize("batch", [1, 3])
def test_cycle_all_permutations(batch):
    g = load_golden("graph_cycle.json")
    want = {k: [D(x) for x in v] for k, v in g["expect_order"].items()}
    for perm in itertools.permutations(g["args"]):
        assert check_termination(g["n"], list(perm), batch) == want


@pytest.mark.parametrize("name", ["regression_1.json", "regression_2.json"])
def test_transitive_conflicts_regressions(name):
    g = load_golden(name)
    a = check_termination(g["n"], g["order_a"])
    b = check_termination(g["n"], g["order_b"])
    assert a != b
    assert a == {k: [D(x) for x in v] for k, v in g["derived_order_a"].items()}
    assert b == {k: [D(x) for x in v] for k, v in g["derived_order_b"].items()}


def test_sccs_found_and_missing_dep():
    g = load_golden("sccs_found_and_missing_dep.json")
    ex = HipGraphExecutor(g["process_id"], g["shard_id"], g["n"], g["f"], key_space=8)
    for i, seq in enumerate(g["executed_clock"]):
        ex.set_executed_frontier(i + 1, seq)
    infos = [GraphExecutionInfo.add(D(v["dot"]), Command(D(v["dot"]), g["keys"]),
                                    [D(x) for x in v["deps"]]) for v in g["vertices"]]
    ex.handle_batch(infos)
    got = []
    while (r := ex.to_clients()) is not None:
        got.append(r[0])
    assert got == [D([4, s]) for s in range(31, 41)]  # the SCCs found are executed
    assert ex.pending() == 1                           # the root stays pending
    assert ex.missing() == [D(x) for x in g["expect"]["missing"]]
    # RequestReply::Executed for the missing dependency (mod.rs:397-405) marks
    # it executed; the next batch retries the pending vertex, which executes
    ex.mark_executed([D([5, 61])])
    ex.handle_batch([])
    assert ex.pending() == 0
    assert ex.to_clients()[0] == D([5, 70])


@pytest.mark.parametrize("it", range(10))
@pytest.mark.parametrize("batch", [1, 2, 6])
def test_add_random_all_permutations(it, batch):
    rng = random.Random(0xFA17 + it)
    args = random_adds(rng, 2, 3)
    total = check_termination(2, args, batch)
    perms = list(itertools.permutations(args))
    for perm in (perms if batch == 1 else perms[::37]):
        assert check_termination(2, list(perm), batch) == total


@pytest.mark.parametrize("batch", [1, 7, 500, 4000])
def test_views_stream_shuffled_arrivals_match_oracle(batch):
    """Committed deps from replica views, delivered to the executor in a
    shuffled commit order and in batches: per-key order equals the oracle's
    incremental executor on the same arrival order."""
    s = Workload.zipf(0.99, 512, k=2, views=3, window=64, seed=17).generate(4000)
    key_off = s.key_off()
    keys = s.keys.reshape(-1)
    dep_off, deps = O.views_run(0, 5, s.dots, key_off, keys, s.fq_proc, s.fq_time)
    # commit arrival: stream order perturbed within a window
    rng = np.random.default_rng(3)
    arrival = np.argsort(np.arange(s.n) + rng.integers(0, 200, size=s.n), kind="stable")
    a_dots = s.dots[arrival]
    a_keys = s.keys[arrival]
    a_key_off = (np.arange(s.n + 1) * s.k).astype(np.uint32)
    a_dep_off = np.zeros(s.n + 1, dtype=np.uint32)
    a_deps = []
    for j, i in enumerate(arrival):
        a_deps.extend(deps[dep_off[i]:dep_off[i + 1]])
        a_dep_off[j + 1] = len(a_deps)
    a_deps = np.asarray(a_deps, dtype=np.uint64)
    ex_o, lab_o, kso, ks = O.graph_run(a_dots, a_key_off, a_keys.reshape(-1), a_dep_off, a_deps,
                                       s.key_space)
    want = {int(k): ks[kso[k]:kso[k + 1]].tolist() for k in np.nonzero(np.diff(kso))[0]}
    ex = HipGraphExecutor(1, 0, 5, 1, key_space=s.key_space)
    for b0 in range(0, s.n, batch):
        infos = [GraphExecutionInfo.add(int(a_dots[j]), [int(x) for x in a_keys[j]],
                                        a_deps[a_dep_off[j]:a_dep_off[j + 1]].tolist())
                 for j in range(b0, min(s.n, b0 + batch))]
        ex.handle_batch(infos)
    assert ex.pending() == 0
    got = {k: v for k, v in ex.monitor().items()}
    assert got == want
    # SCC partition equals the oracle's
    assert ex.last_labels == dict(zip(ex_o.tolist(), lab_o.tolist()))


def _ex():
    return HipGraphExecutor(process_id=1, shard_id=0, n=3, f=1, key_space=16)


def _add(ex, dot, deps, keys=("A",)):
    ex.handle(GraphExecutionInfo.add(dot, Command(dot, list(keys)), deps))


def test_monitor_pending_reports_missing_and_ages():
    """VertexIndex::monitor_pending (index.rs:53-103): pending commands older
    than the threshold, longest first, with their missing dependencies (found
    through other pending vertices)."""
    ex = _ex()
    ex.set_time(1000)
    _add(ex, D((1, 1)), [D((2, 1))])            # waits on (2,1), never added
    ex.set_time(1500)
    _add(ex, D((1, 2)), [D((1, 1))])            # waits through (1,1)
    ex.set_time(2600)
    got = ex.monitor_pending(1000)
    assert [(d, t) for d, t, _ in got] == [(D((1, 1)), 1600), (D((1, 2)), 1100)]
    assert all(m == 1 for _, _, m in got)       # (2,1) in both cases
    assert ex.monitor_pending(1500) == [(D((1, 1)), 1600, 1)]


def test_metrics_chain_size_and_execution_delay():
    """save_scc (graph/mod.rs:490-525): one ChainSize per SCC, one
    ExecutionDelay per command (ready time - add time)."""
    ex = _ex()
    ex.set_time(10)
    _add(ex, D((1, 1)), [D((2, 1))])
    ex.set_time(25)
    _add(ex, D((2, 1)), [D((1, 1))])            # closes the 2-cycle
    ex.set_time(30)
    _add(ex, D((3, 1)), [D((1, 1))])            # a singleton after it
    chains, delays = ex.take_metrics()
    assert sorted(chains) == [1, 2]
    assert sorted(delays) == [0, 0, 15]
    assert ex.take_metrics() == ([], [])


def test_pending_retry_skipped_until_a_missing_dep_executes():
    """check_pending retries only when a missing dependency executed: an empty
    retry with nothing resolved runs no graph pass."""
    ex = _ex()
    _add(ex, D((1, 1)), [D((3, 7))])
    p0, s0 = ex.passes()
    ex.handle_batch([])
    ex.mark_executed([D((2, 5))])               # unrelated
    ex.handle_batch([])
    p1, s1 = ex.passes()
    assert (p1, s1) == (p0, s0 + 2) and ex.pending() == 1
    ex.mark_executed([D((3, 7))])
    ex.handle_batch([])
    assert ex.passes()[0] == p0 + 1 and ex.pending() == 0


def test_executed_frontier_never_moves_back_and_folds_exceptions():
    ex = _ex()
    ex.mark_executed([D((2, 3)), D((2, 4)), D((2, 9))])  # exceptions above frontier 0
    from fantoch_amd import _lib as L
    L.check(ex._lib.fh_graph_set_executed_frontier(ex._h, 2, 2))
    # frontier 2 folds 3 and 4 -> 4; (2,9) stays an exception: a dep on (2,5)
    # is missing, (2,9) and (2,4) are executed
    _add(ex, D((1, 1)), [D((2, 4)), D((2, 9))])
    assert ex.pending() == 0
    _add(ex, D((1, 2)), [D((2, 5))])
    assert ex.pending() == 1
    with pytest.raises(L.FhError):
        L.check(ex._lib.fh_graph_set_executed_frontier(ex._h, 2, 1))


def test_many_and_far_clock_exceptions():
    """AEClock with more exceptions than the small pass stages in LDS (1,500,
    so its resolve searches the device list), exceptions beyond the bit ring
    (4,096 above the frontier), and frontier raises folding both."""
    ex = _ex()
    ex.mark_executed([D((2, s)) for s in range(2, 3001, 2)] + [D((2, 10000))] +
                     [D((3, s)) for s in range(5000, 5101)])
    _add(ex, D((1, 1)), [D((2, 2000)), D((2, 10000)), D((3, 5050))])
    assert ex.pending() == 0                      # every dependency executed
    _add(ex, D((1, 2)), [D((2, 2001))])
    assert ex.pending() == 1 and ex.missing() == [D((2, 2001))]
    ex.mark_executed([D((2, 1))])                 # folds 1, 2; 3 is not executed
    _add(ex, D((1, 3)), [D((2, 3))])
    assert ex.pending() == 2
    ex.mark_executed([D((2, 2001))])
    ex.handle_batch([])
    assert ex.pending() == 1                      # (1, 2) went, (1, 3) waits on (2, 3)
    ex.set_executed_frontier(2, 2999)             # folds the even exceptions up to 3000
    ex.handle_batch([])
    assert ex.pending() == 0
    _add(ex, D((1, 4)), [D((2, 3000)), D((3, 5100))])
    _add(ex, D((1, 5)), [D((2, 3001)), D((3, 4999))])
    assert ex.pending() == 1 and ex.missing() == [D((2, 3001)), D((3, 4999))]
    ex.set_executed_frontier(3, 5200)             # far exceptions at or below it go
    ex.mark_executed([D((2, 3001))])
    ex.handle_batch([])
    assert ex.pending() == 0
    got = []
    while (r := ex.to_clients()) is not None:
        got.append(r[0])
    assert got == [D((1, s)) for s in (1, 2, 3, 4, 5)]


def test_device_resident_backlog_then_release_matches_oracle():
    """A command held back until the end leaves most of the stream pending
    behind it (carried on the device from batch to batch); the missing set is
    exactly that dot; re-adding a pending dot is rejected without touching the
    backlog; releasing it executes everything in the oracle's per-key order
    for the same arrival order."""
    s = Workload.zipf(0.99, 256, k=2, views=3, window=64, seed=23).generate(6000)
    key_off = s.key_off()
    keys = s.keys.reshape(-1)
    dep_off, deps = O.views_run(0, 5, s.dots, key_off, keys, s.fq_proc, s.fq_time)
    hold = 40
    arrival = np.array([i for i in range(s.n) if i != hold] + [hold])
    a_dots, a_keys = s.dots[arrival], s.keys[arrival]
    a_key_off = (np.arange(s.n + 1) * s.k).astype(np.uint32)
    a_dep_off = np.zeros(s.n + 1, dtype=np.uint32)
    a_deps = []
    for j, i in enumerate(arrival):
        a_deps.extend(deps[dep_off[i]:dep_off[i + 1]])
        a_dep_off[j + 1] = len(a_deps)
    a_deps = np.asarray(a_deps, dtype=np.uint64)
    ex_o, lab_o, kso, ks = O.graph_run(a_dots, a_key_off, a_keys.reshape(-1), a_dep_off, a_deps,
                                       s.key_space)
    want = {int(k): ks[kso[k]:kso[k + 1]].tolist() for k in np.nonzero(np.diff(kso))[0]}
    ex = HipGraphExecutor(1, 0, 5, 1, key_space=s.key_space)

    def info(j):
        return GraphExecutionInfo.add(int(a_dots[j]), [int(x) for x in a_keys[j]],
                                      a_deps[a_dep_off[j]:a_dep_off[j + 1]].tolist())
    for b0 in range(0, s.n - 1, 333):
        ex.handle_batch([info(j) for j in range(b0, min(s.n - 1, b0 + 333))])
    backlog = ex.pending()
    assert backlog > s.n // 4
    assert ex.missing() == [int(s.dots[hold])]
    from fantoch_amd import _lib as L
    pend = [d for d, _, _ in ex.monitor_pending(0)]
    assert len(pend) == backlog
    j = int(np.nonzero(a_dots == np.uint64(pend[len(pend) // 2]))[0][0])
    with pytest.raises(L.FhError):
        ex.handle_batch([info(j)])                   # already pending
    assert ex.pending() == backlog
    ex.handle_batch([info(s.n - 1)])                 # the held command
    assert ex.pending() == 0 and ex.missing() == []
    assert ex.monitor() == want
    assert ex.last_labels == dict(zip(ex_o.tolist(), lab_o.tolist()))


def test_kv_results_follow_the_oracle_order():
    """Command / KV execution: the HIP executor runs each
    drained command on its KVStore (Command::execute, command.rs:114-127;
    KVStore::do_execute, kvs.rs:52-68).  With every command a Put of its own
    value, each ExecutorResult is the previous Put's value on that key in the
    oracle's per-key execution order (None for the key's first command)."""
    from fantoch_amd.kvs import KVOp
    s = Workload.zipf(0.99, 256, k=2, views=3, window=64, seed=23).generate(3000)
    key_off = s.key_off()
    keys = s.keys.reshape(-1)
    dep_off, deps = O.views_run(0, 5, s.dots, key_off, keys, s.fq_proc, s.fq_time)
    _, _, kso, ks = O.graph_run(s.dots, key_off, keys, dep_off, deps, s.key_space)
    want = {}
    for k in np.nonzero(np.diff(kso))[0]:
        seq = ks[kso[k]:kso[k + 1]].tolist()
        for j, d in enumerate(seq):
            want[(d, str(int(k)))] = str(seq[j - 1]) if j else None
    ex = HipGraphExecutor(1, 0, 5, 1, key_space=s.key_space)
    infos = []
    for i in range(s.n):
        d = int(s.dots[i])
        c = Command.from_ops(d, [(str(int(k)), KVOp.put(str(d))) for k in s.keys[i]])
        infos.append(GraphExecutionInfo.add(d, c, deps[dep_off[i]:dep_off[i + 1]].tolist()))
    for b0 in range(0, s.n, 700):
        ex.handle_batch(infos[b0:b0 + 700])
    assert ex.pending() == 0
    got = {}
    while (r := ex.to_clients()) is not None:
        got[(r.rifl, r.key)] = r.op_result
    assert got == want
    # the store holds each key's last Put
    for k in np.nonzero(np.diff(kso))[0]:
        assert ex.store.execute(str(int(k)), KVOp.get()) == str(int(ks[kso[k + 1] - 1]))


def test_small_pass_equals_general_pass():
    """The one-launch small-graph pass (csrc/graph_small.hip, V <= 2048)
    against the general pass (FH_GRAPH_SMALL=0, read once per process: child
    processes) on shuffled streams in batches of 1, 5 and 300 with a held-back
    backlog: identical drained dots and SCC labels, in the same order, and
    identical pending counts after every batch.  The 2-key stream keeps more
    than 1024 commands pending, so passes with 1024 < V <= 2048 (two vertices
    per thread) run small."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import json, sys
import numpy as np
sys.path.insert(0, {root!r})
from fantoch_amd.engine import Engine
from fantoch_amd.executor import HipGraphExecutor, GraphExecutionInfo
from fantoch_amd.workload import Workload
out = []
for k, seed in ((1, 91), (2, 92)):
    s = Workload.zipf(0.99, 512, k=k, views=3, window=64, seed=seed).generate(6000)
    eng = Engine(s.key_space, n=5)
    eng.stage(s); eng.run()
    r = eng.results()
    rng = np.random.default_rng(5)
    order = [int(i) for i in np.argsort(np.arange(s.n) + rng.integers(0, 200, s.n), kind="stable")]
    order = order[:17] + order[18:] + [order[17]]  # one command held back: a backlog
    for batch in (1, 5, 300):
        ex = HipGraphExecutor(1, 0, 5, 1, key_space=s.key_space)
        pend = []
        for b0 in range(0, len(order), batch):
            ex.handle_batch([GraphExecutionInfo.add(int(s.dots[j]), [int(x) for x in s.keys[j]],
                             [int(x) for x in r["deps"][r["dep_off"][j]:r["dep_off"][j + 1]]])
                             for j in order[b0:b0 + batch]])
            pend.append(ex.pending())
        seq = []
        while True:
            x = ex.to_clients()
            if x is None:
                break
            seq.append([int(x.rifl), int(x.key)])
        out.append([seq, sorted(ex.last_labels.items()), pend, ex.passes()])
print(json.dumps(out))
"""
    res = []
    for env in ({}, {"FH_GRAPH_SMALL": "0"}):
        e = dict(os.environ, **env)
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           timeout=300, env=e)
        assert p.returncode == 0, p.stdout + p.stderr
        res.append(json.loads(p.stdout.strip().splitlines()[-1]))
    assert [r[:3] for r in res[0]] == [r[:3] for r in res[1]]
    # the 2-key stream at batch 1 crosses 1024 pending while below 2048
    pend = res[0][3][2]
    assert any(1024 < x < 2047 for x in pend), max(pend)


def test_small_pass_deadline_returns_ehip():
    """A small pass (graph_small.hip) that does not finish by the host's
    deadline fails the call with FH_EHIP and fh_last_error set instead of
    spinning (graph_small.h poll_completion).  Fault injection: the kernel
    waits 300 ms before it starts, the deadline is 20 ms.  The handle then
    refuses further calls; destroying it waits for the kernel."""
    from fantoch_amd import _lib as L
    ex = HipGraphExecutor(process_id=1, shard_id=0, n=5, f=1, key_space=64)
    a = D([1, 1])
    ex.handle(GraphExecutionInfo.add(a, Command(a, ["x"]), []))
    assert ex.to_clients() is not None
    lib = L.load()
    L.check(lib.fh_graph_inject_small_delay(ex._h, 300_000, 20))
    b = D([2, 1])
    with pytest.raises(L.FhError) as e:
        ex.handle(GraphExecutionInfo.add(b, Command(b, ["x"]), [a]))
    assert e.value.status == L.FH_EHIP
    assert "did not complete within 20 ms" in str(e.value)
    with pytest.raises(L.FhError) as e2:
        ex.pending()
    assert e2.value.status == L.FH_EHIP
    ex.close()
    # a fresh handle is unaffected
    ex2 = HipGraphExecutor(process_id=1, shard_id=0, n=5, f=1, key_space=64)
    ex2.handle(GraphExecutionInfo.add(a, Command(a, ["x"]), []))
    assert ex2.to_clients() is not None
    ex2.close()
