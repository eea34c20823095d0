"""Execution-log replay (fh_execlog_replay) into the HIP GraphExecutor --
graph_executor_replay.rs:13-38's loop, batched.  Logs are written with the
bincode writer (fantoch_amd/execlog.py, pinned byte-by-byte in
tests/test_execlog.py) from the reference's known-answer graph inputs and
from a replica-view stream whose per-key order the oracle gives."""
import itertools
import random

import numpy as np
import pytest

from conftest import D, load_golden
from fantoch_amd import execlog as E
from fantoch_amd.executor import HipGraphExecutor
from fantoch_amd.workload import Workload
from oracle import oracle as O
from test_oracle_golden import random_adds

pytestmark = pytest.mark.gpu


def log_of(args):
    """One Add frame per {dot, keys, deps}; rifl = (0, packed dot)."""
    out = []
    for a in args:
        dot = D(a["dot"])
        keys = a["keys"] if a["keys"] is not None else ["CONF"]
        cmd = E.encode_command((0, dot), {0: [(k, (E.PUT, "v")) for k in keys]})
        out.append(E.frame(E.encode_add(dot, cmd, [(D(x), [0]) for x in a["deps"]])))
    return b"".join(out)


def replay(data, n, batch):
    ex = HipGraphExecutor(process_id=1, shard_id=0, n=n, f=1, key_space=4096)
    lg = E.ExecLog(data)
    ready = lg.replay(ex, batch)
    assert ex.pending() == 0
    return ready, {k: [r[1] for r in v] for k, v in ex.monitor().items()}


@pytest.mark.parametrize("batch", [0, 1, 4])
def test_cycle_log_all_permutations(batch):
    g = load_golden("graph_cycle.json")
    want = {k: [D(x) for x in v] for k, v in g["expect_order"].items()}
    for perm in itertools.permutations(g["args"]):
        ready, got = replay(log_of(list(perm)), g["n"], batch)
        assert ready == len(perm)
        assert got == want


@pytest.mark.parametrize("it", range(4))
def test_add_random_log_permutations(it):
    rng = random.Random(0xFA17 + it)
    args = random_adds(rng, 2, 3)
    _, total = replay(log_of(args), 2, 1)
    for perm in list(itertools.permutations(args))[::53]:
        assert replay(log_of(list(perm)), 2, 3)[1] == total


def test_views_stream_log_matches_oracle():
    s = Workload.zipf(0.99, 256, k=2, views=3, window=64, seed=5).generate(3000)
    key_off = s.key_off()
    keys = s.keys.reshape(-1)
    dep_off, deps = O.views_run(0, 5, s.dots, key_off, keys, s.fq_proc, s.fq_time)
    frames = []
    for i in range(s.n):
        dot = int(s.dots[i])
        ks = [str(int(k)) for k in keys[key_off[i]:key_off[i + 1]]]
        cmd = E.encode_command((0, dot), {0: [(k, (E.PUT, "v")) for k in ks]})
        frames.append(E.frame(E.encode_add(
            dot, cmd, [(int(d), [0]) for d in deps[dep_off[i]:dep_off[i + 1]]])))
    ready, got = replay(b"".join(frames), 5, 500)
    assert ready == s.n
    _, _, kso, ks = O.graph_run(s.dots, key_off, keys, dep_off, deps, s.key_space, n=5)
    want = {str(k): [int(d) for d in ks[kso[k]:kso[k + 1]]]
            for k in range(len(kso) - 1) if kso[k + 1] > kso[k]}
    assert got == want


def test_log_with_requests_and_replies():
    """Request -> Executed reply; RequestReply::Executed releases a pending
    command; RequestReply::Info adds the requested command."""
    sh = 0
    c1 = E.encode_command((0, D([1, 1])), {0: [("a", E.DELETE)]})
    c2 = E.encode_command((0, D([1, 2])), {0: [("a", E.DELETE)]})
    c3 = E.encode_command((0, D([3, 1])), {1: [("z", E.DELETE)]})
    data = b"".join(E.frame(f) for f in [
        E.encode_add(D([1, 1]), c1, []),                                 # executes
        E.encode_add(D([1, 2]), c2, [(D([1, 1]), [0]), (D([3, 1]), [1])]),  # waits on (3,1)
        E.encode_request(1, [D([1, 1])]),                                # -> Executed reply
        E.encode_request_reply([("info", D([3, 1]), c3, [(D([3, 0 + 7]), [1])])]),
        E.encode_request_reply([("executed", D([3, 7]))]),               # releases (3,1), (1,2)
        E.encode_executed([D([1, 1])]),
    ])
    ex = HipGraphExecutor(process_id=1, shard_id=sh, n=2, f=0, shard_count=2, key_space=8)
    lg = E.ExecLog(data, shard_id=sh)
    assert lg.replay(ex, 0) == 3
    assert ex.pending() == 0
    assert {k: [r[1] for r in v] for k, v in ex.monitor().items()} == {"a": [D([1, 1]), D([1, 2])]}
    reps = ex.request_replies()
    assert [(r.kind, r.dot) for r in reps[1]] == [("executed", D([1, 1]))]
    # (3,1) was requested from its target shard ((3-1)//n = 1) when (1,2)
    # arrived, and (3,7) when the Info for (3,1) arrived
    assert ex.requests() == {1: {D([3, 1]), D([3, 7])}}
