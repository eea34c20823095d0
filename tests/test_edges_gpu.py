"""Edge cases through the C ABI against the oracle: empty and one-command
inputs, sizes at the radix-sort tile (4096) and reorder-window (64)
boundaries, a one-key stream (every command conflicts: one long chain per
replica), the largest key id, and extreme dots (ProcessId 255, sequence
2^56 - 1: the top of the packed order, fantoch/src/id.rs:24-62)."""
import numpy as np
import pytest

from conftest import D
from fantoch_amd import _lib as L
from fantoch_amd.engine import Engine
from fantoch_amd.executor import GraphExecutionInfo, HipGraphExecutor
from fantoch_amd.keydeps import HipKeyDeps
from fantoch_amd.workload import Workload
from oracle import oracle as O
from test_engine_gpu import check_engine

pytestmark = pytest.mark.gpu

MAX_SEQ = (1 << 56) - 1


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 4095, 4096, 4097])
def test_views_engine_at_tile_and_window_boundaries(n):
    s = Workload.zipf(0.99, 1 << 10, k=1, views=3, window=64, seed=100 + n, n=5).generate(n)
    check_engine(s)


@pytest.mark.parametrize("n", [1, 4095, 4097])
def test_single_view_engine_at_tile_boundaries(n):
    s = Workload.zipf(0.7, 1 << 12, k=1, seed=200 + n).generate(n)
    check_engine(s)


def test_one_key_stream_every_command_conflicts():
    """ConflictRate 100 %: every command on the shared key; each replica's
    KeyDeps is one chain and the reordering makes cycles across it."""
    s = Workload.conflict_rate_(100, k=1, views=3, window=64, seed=7, n=5).generate(20_000)
    assert len(np.unique(s.keys)) == 1
    check_engine(s)


def test_keydeps_empty_batch_and_extreme_dots_and_keys():
    """n = 0 is a no-op; dots at the top of the packed order and the largest
    key id of the space go through unchanged (vs SequentialKeyDeps)."""
    K = 1 << 12
    kd = HipKeyDeps(0, key_space=K)
    off, deps = kd.add_batch([], [])
    assert len(off) == 1 and off[0] == 0 and len(deps) == 0
    dots = [D((255, MAX_SEQ)), D((1, 1)), D((255, MAX_SEQ - 1)), D((2, MAX_SEQ)), D((1, 2))]
    keys = [[K - 1], [K - 1, 0], [0], [K - 1], [5, K - 1, 0]]
    off, deps = kd.add_batch(dots, keys)
    key_off = np.zeros(len(keys) + 1, dtype=np.uint32)
    key_off[1:] = np.cumsum([len(k) for k in keys])
    o_off, o_deps = O.keydeps_run(np.asarray(dots, dtype=np.uint64), key_off,
                                  np.asarray([k for ks in keys for k in ks], dtype=np.uint64))
    assert np.array_equal(off, o_off) and np.array_equal(deps, o_deps)
    with pytest.raises(L.FhError):
        kd.add_batch([D((3, 1))], [[K]])            # key id == key_space


def test_executor_extreme_dots_and_empty_batches():
    """An empty batch on a fresh executor does nothing; a 2-cycle between
    (255, 2^56-1) and (1, 1) executes in dot order; a dependency on an
    executed (255, 2^56-1) is ignored (tarjan.rs:131-148)."""
    ex = HipGraphExecutor(1, 0, 5, 1, key_space=16)
    ex.handle_batch([])
    assert ex.pending() == 0
    hi, lo = D((255, MAX_SEQ)), D((1, 1))
    ex.handle(GraphExecutionInfo.add(hi, [3], [lo]))
    assert ex.pending() == 1 and ex.missing() == [lo]
    ex.handle(GraphExecutionInfo.add(lo, [3], [hi]))
    assert ex.pending() == 0
    assert ex.monitor()[3] == [lo, hi]               # one SCC: members in dot order
    ex.handle(GraphExecutionInfo.add(D((2, 1)), [3], [hi]))
    assert ex.pending() == 0


def test_engine_rejects_key_out_of_space():
    s = Workload.zipf(0.99, 1 << 10, k=1, views=3, window=64, seed=3, n=5).generate(1000)
    eng = Engine(s.key_space // 2, n=5)
    with pytest.raises(L.FhError):
        eng.stage(s)


EMPTY_OVER_BACKLOG = """
import sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import torch; torch.zeros(1, device="cuda")
from conftest import D
from fantoch_amd.executor import GraphExecutionInfo, HipGraphExecutor
ex = HipGraphExecutor(1, 0, 5, 1, key_space=16)
# a backlog: a chain of 40 commands on key 3 waiting on (5, 1), plus a 2-cycle
# waiting on (5, 2); each pass carries them
miss1, miss2 = D((5, 1)), D((5, 2))
chain = [D((1, i)) for i in range(1, 41)]
for i, d in enumerate(chain):
    ex.handle(GraphExecutionInfo.add(d, [3], [miss1] if i == 0 else [chain[i - 1]]))
a, b = D((2, 1)), D((3, 1))
ex.handle_batch([GraphExecutionInfo.add(a, [4], [b, miss2]), GraphExecutionInfo.add(b, [4], [a])])
assert ex.pending() == 42, ex.pending()
for _ in range(5):  # empty batches over the carried set (r04i: k_append)
    ex.handle_batch([])
    assert ex.pending() == 42, ex.pending()
    assert sorted(ex.missing()) == sorted([miss1, miss2]), ex.missing()
ex.handle(GraphExecutionInfo.add(miss1, [3], []))
assert ex.pending() == 2
ex.handle_batch([])
ex.handle(GraphExecutionInfo.add(miss2, [4], []))
assert ex.pending() == 0
assert ex.monitor()[3] == [miss1] + chain
assert ex.monitor()[4] == [miss2, a, b]
print("ok")
"""


@pytest.mark.parametrize("small", ["1", "0"])
def test_executor_empty_batches_over_carried_backlog(small):
    """Empty batches while vertices are carried pending (the round-4 fault:
    k_append rewrote the carried set's end offsets on an empty batch), through
    the one-launch small pass (default) and the general pass
    (FH_GRAPH_SMALL=0, read once per process: a child); then the missing deps
    arrive and everything executes in order."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = EMPTY_OVER_BACKLOG.format(root=os.path.dirname(here), tests=here)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=200, env=dict(os.environ, FH_GRAPH_SMALL=small))
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
