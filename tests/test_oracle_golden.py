"""The CPU oracle against the reference's own known-answer tests.

Pins oracle/ before anything is checked against it (tests/golden/ holds the
transcribed vectors; tests/golden/make_golden.py documents their sources).
"""
import itertools
import random

import pytest

from conftest import D, Interner, UD, load_golden
from oracle import oracle as O


def test_key_deps_flow():
    g = load_golden("key_deps_flow.json")
    kd = O.KeyDeps(g["shard_id"])
    ik = Interner()
    cmds = {name: ik.many(keys) for name, keys in g["commands"].items()}
    for step in g["steps"]:
        if step["op"] == "add_cmd":
            kd.add_cmd(D(step["dot"]), ik.many(step["keys"]), None)
        elif step["op"] == "add_noop":
            kd.add_noop(D(step["dot"]))
        for what, want in step["expect"].items():
            want = {D(x) for x in want}
            got = kd.noop_deps() if what == "noop" else kd.cmd_deps(cmds[what])
            assert got == want, (step, what, [UD(x) for x in got])


def test_add_cmd_with_past_is_union():
    kd = O.KeyDeps(0)
    a = O.dot(1, 1)
    kd.add_cmd(a, [7], None)
    past = {O.dot(3, 9), O.dot(2, 4)}
    got = kd.add_cmd(O.dot(2, 5), [7], past)
    assert got == past | {a}


@pytest.mark.parametrize("case", range(12))
def test_quorum_deps(case):
    g = load_golden("quorum_deps.json")
    c = g["cases"][case]
    reports = [[D(x) for x in r] for r in c["reports"]]
    mode = 0 if c["mode"] == "threshold_union" else 1
    union, flag = O.quorum_deps(c["q"], reports, mode, c.get("threshold", 0))
    assert union == {D(x) for x in c["union"]}
    assert flag == c["flag"]


def check_termination(n, args, key_space_hint=None):
    """graph/mod.rs:1047-1115 via the oracle's DependencyGraph."""
    ik = Interner()
    g = O.Graph(process_id=1, shard_id=0, n=n, f=1)
    order = {}
    pending = set()
    for a in args:
        keys = a["keys"] if a["keys"] is not None else ["CONF"]
        dot = D(a["dot"]) if isinstance(a["dot"], list) else a["dot"]
        deps = [D(x) if isinstance(x, list) else x for x in a["deps"]]
        pending.add(dot)
        g.add(dot, ik.many(keys), deps)
        ex, _ = g.drain()
        keymap = {dot: keys}
        for e in ex:
            pending.discard(e)
            for k in keys_of[e]:
                order.setdefault(k, []).append(e)
    assert not pending, "every command executes exactly once"
    return order


keys_of = {}


def run_args(n, args):
    for a in args:
        dot = D(a["dot"]) if isinstance(a["dot"], list) else a["dot"]
        keys_of[dot] = a["keys"] if a["keys"] is not None else ["CONF"]
    return check_termination(n, args)


def test_graph_simple():
    g = load_golden("graph_simple.json")
    gr = O.Graph(g["process_id"], g["shard_id"], g["n"], g["f"])
    ik = Interner()
    for a in g["adds"]:
        gr.add(D(a["dot"]), ik.many(a["keys"]), [D(x) for x in a["deps"]])
        ex, labels = gr.drain()
        assert ex == [D(x) for x in a["expect_executed"]]
    # both executed as one SCC labelled by its min dot
    assert labels == [D([1, 1])] * 2


def test_graph_cycle_all_permutations():
    g = load_golden("graph_cycle.json")
    want = {k: [D(x) for x in v] for k, v in g["expect_order"].items()}
    for perm in itertools.permutations(g["args"]):
        assert run_args(g["n"], list(perm)) == want


@pytest.mark.parametrize("name", ["regression_1.json", "regression_2.json"])
def test_transitive_conflicts_regressions(name):
    g = load_golden(name)
    a = run_args(g["n"], g["order_a"])
    b = run_args(g["n"], g["order_b"])
    assert a != b  # the reference's assertion
    assert a == {k: [D(x) for x in v] for k, v in g["derived_order_a"].items()}
    assert b == {k: [D(x) for x in v] for k, v in g["derived_order_b"].items()}


def test_sccs_found_and_missing_dep():
    g = load_golden("sccs_found_and_missing_dep.json")
    gr = O.Graph(g["process_id"], g["shard_id"], g["n"], g["f"])
    ik = Interner()
    for v in g["vertices"]:
        gr.index_only(D(v["dot"]), ik.many(g["keys"]), [D(x) for x in v["deps"]])
    for i, seq in enumerate(g["executed_clock"]):
        gr.set_executed_frontier(i + 1, seq)
    kind, ready, nfound, missing = gr.find_scc(g["first_find"], D(g["root"]))
    assert kind == 1  # MissingDependencies
    assert missing == [D(x) for x in g["expect"]["missing"]]
    assert ready == nfound
    assert nfound > 0
    ex, labels = gr.drain()
    # (4,31)..(4,40) each its own SCC, executed in chain order
    assert ex == [D([4, s]) for s in range(31, 41)]
    assert labels == ex


def random_adds(rng, n, events_per_process):
    """graph/mod.rs:934-1033 (random_adds), seeded."""
    possible = ["A", "B", "C", "D"]
    dots = [(p, e) for p in range(1, n + 1) for e in range(1, events_per_process + 1)]
    data = {}
    for dt in dots:
        rng.shuffle(possible)
        data[dt] = (sorted(possible[:2]), set())
    for left, right in itertools.combinations(dots, 2):
        lk, ld = data[left]
        rk, rd = data[right]
        if set(lk) & set(rk):
            if left[0] == right[0]:
                if left[1] < right[1]:
                    rd.add(left)
                else:
                    ld.add(right)
            else:
                r = rng.randrange(3)
                if r == 0:
                    ld.add(right)
                elif r == 1:
                    rd.add(left)
                else:
                    ld.add(right)
                    rd.add(left)
    return [{"dot": list(dt), "keys": data[dt][0], "deps": [list(x) for x in data[dt][1]]}
            for dt in dots]


@pytest.mark.parametrize("it", range(10))
def test_add_random_all_permutations(it):
    """graph/mod.rs:921-932 test_add_random: n=2, 3 events/process, 10 iterations,
    all 6! arrival permutations give the same per-key order."""
    rng = random.Random(0xFA17 + it)
    args = random_adds(rng, 2, 3)
    total = run_args(2, args)
    for perm in itertools.permutations(args):
        assert run_args(2, list(perm)) == total
