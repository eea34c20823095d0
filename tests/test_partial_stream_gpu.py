"""The fused engine on partially replicated streams (BASELINE config C5's
model, include/fantoch_hip.h fh_workload.shards): shard h holds processes
5h+1..5h+5 (fantoch/src/util.rs:115-122), a command's dot comes from its
target shard (id.rs:59-61), and every shard it touches collects it with its
own fast quorum and arrival order (atlas.rs:214-328).  The engine stages the
replicas' element logs (FH_STREAM_ELEMENT_LOGS: each replica sees only the
command's keys on its shard, Command::keys(shard), command.rs:95-100) and
must equal the oracle's shard-by-shard computation unioned across shards
(MShardCommit, atlas.rs:559-639; tests/fullsize.py shard_union) followed by
one GraphExecutor: bit-exact deps, SCC partition and per-key sequences."""
import numpy as np
import pytest

from fantoch_amd.engine import Engine
from fantoch_amd.workload import Stream, Workload
from fullsize import shard_union
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def oracle_partial(s):
    off, deps = shard_union(s)
    ex, lab, kso, ks = O.graph_run(s.dots, s.key_off(), s.keys.reshape(-1), off, deps,
                                   s.key_space)
    assert len(ex) == s.n, "the oracle executes every command"
    return off, deps, ex, lab, kso, ks


def run_engine(s):
    eng = Engine(s.key_space, n=5)
    eng.stage(s)
    eng.run()
    r = eng.results()
    eng.close()
    return r


@pytest.mark.parametrize("shards,keys,k,n,seed", [
    (8, 4096, 4, 6000, 51),       # C5's shape, small
    (8, 1 << 20, 4, 6000, 52),    # C5's key space
    (2, 256, 2, 4000, 53),        # two shards, hot keys
    (4, 64, 3, 3000, 54),         # very hot keys: long same-key segments per replica
])
def test_partial_stream_matches_oracle(shards, keys, k, n, seed):
    w = Workload.zipf(0.99, keys, k=k, views=3, window=64, seed=seed, n=5, shards=shards)
    s = w.generate(n, logs=True)
    assert s.log_elem is not None and len(s.log_off) == 5 * shards + 1
    off, deps, ex, lab, kso, ks = oracle_partial(s)
    r = run_engine(s)
    assert np.array_equal(r["dep_off"], off) and np.array_equal(r["deps"], deps), "deps"
    want = dict(zip(ex.tolist(), lab.tolist()))
    assert dict(zip(s.dots.tolist(), r["scc_label"].tolist())) == want, "SCC partition"
    assert np.array_equal(r["key_off"], kso) and np.array_equal(r["key_seq"], ks), "per-key"


@pytest.mark.parametrize("env", [{"FH_VIEW_CHUNK": "30000"},
                                 {"FH_VIEW_CHUNK": "30000", "FH_VIEW_CMD": "0"}])
def test_partial_stream_in_chunks_matches_oracle(env):
    """Element logs through the pair-level search (default), and through the
    chunked element path (FH_VIEW_CMD=0) with small KeyDeps chunks
    (FH_VIEW_CHUNK; both read once per process: a child process), so each of
    the 40 replicas' (replica, key) segments crosses chunks and bucketing
    workgroups."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import numpy as np, sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {os.path.join(root, 'tests')!r})
from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload
from fullsize import shard_union
s = Workload.zipf(1.1, 2048, k=4, views=3, window=64, seed=55, shards=8).generate(40_000, logs=True)
off, deps = shard_union(s)
eng = Engine(s.key_space, n=5)
eng.set_deps_only(True)
eng.stage(s)
eng.run()
got_off, got = eng.deps()
assert np.array_equal(got_off, off) and np.array_equal(got, deps)
print("ok")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=200,
                       env=dict(os.environ, **env))
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_partial_stream_batches_match_oracle():
    """A partially replicated stream staged as three element-log batches:
    the 40 replicas' latest tables carry across batches."""
    w = Workload.zipf(0.99, 1 << 12, k=4, views=3, window=64, seed=56, shards=8)
    parts = [w.generate(3000, first=i * 3000, logs=True) for i in range(3)]
    whole = w.generate(9000)
    assert np.array_equal(np.concatenate([p.dots for p in parts]), whole.dots)
    # the whole stream's arrivals: batch b's commands arrive after batch b-1's
    # (the engine's batches are committed in order)
    t = whole.fq_time.copy()
    for i in range(3):
        t[i * 3000:(i + 1) * 3000] += np.uint64(i) * np.uint64(1 << 40)
    whole.fq_time = t
    off, deps = shard_union(whole)
    eng = Engine(whole.key_space, n=5)
    eng.set_deps_only(True)
    eng.stage_logs(parts)
    got = []
    for _ in range(3):
        eng.run()
        got.append(eng.deps()[1])
    assert np.array_equal(np.concatenate(got), deps)


def test_element_logs_equal_command_logs_unsharded():
    """Element logs of an unsharded stream (every key slot of a command at
    each of its replicas) give exactly the command-log path's results."""
    w = Workload.zipf(0.99, 1 << 12, k=4, views=3, window=64, seed=57)
    a = w.generate(30_000, logs=True)
    b = w.generate(30_000, logs=True, element_logs=True)
    assert a.log_cmd is not None and b.log_elem is not None
    ra, rb = run_engine(a), run_engine(b)
    for key in ("dep_off", "deps", "scc_label", "exec_rank", "key_off", "key_seq"):
        assert np.array_equal(ra[key], rb[key]), key


def test_partial_replication_changes_the_graph():
    """The shards' independent arrival orders matter: on the same commands the
    committed deps differ from one 5-process KeyDeps over all keys (the
    target shard's views for every key), and cross-shard cycles merge SCCs."""
    w = Workload.zipf(0.99, 1 << 20, k=4, views=3, window=64, seed=58, shards=8)
    s = w.generate(8000, logs=True)
    r = run_engine(s)
    # the same commands fully replicated: every slot takes the target
    # shard's views (processes renumbered 1..5)
    t_slot = np.argmax((s.keys % np.uint64(8)) == (s.keys[:, :1] % np.uint64(8)), axis=1)
    idx = np.arange(s.n)
    proc = ((s.fq_proc[idx, t_slot].astype(np.int64) - 1) % 5 + 1).astype(np.uint8)
    full = Stream(s.dots, s.keys, proc, s.fq_time[idx, t_slot], s.key_space)
    r1 = run_engine(full)
    o_off, o_deps = O.views_run(0, 5, full.dots, full.key_off(), full.keys.reshape(-1), full.fq_proc,
                                full.fq_time)
    assert np.array_equal(r1["dep_off"], o_off) and np.array_equal(r1["deps"], o_deps)
    a = np.split(r["deps"], r["dep_off"][1:-1].astype(np.int64))
    b = np.split(r1["deps"], r1["dep_off"][1:-1].astype(np.int64))
    differ = sum(not np.array_equal(x, y) for x, y in zip(a, b))
    assert differ > s.n // 10, f"only {differ} commands' deps differ"
    largest = np.unique(r["scc_label"], return_counts=True)[1].max()
    largest1 = np.unique(r1["scc_label"], return_counts=True)[1].max()
    assert largest > largest1, (largest, largest1)


@pytest.mark.parametrize("shards,keys,n,seed", [(8, 4096, 20_000, 61), (8, 1 << 20, 20_000, 62),
                                                (2, 256, 8000, 63)])
def test_pair_search_equals_chunked_path(shards, keys, n, seed):
    """The pair-level search ((command, key slot) units, engine.hip
    unit_meta) and the chunked element path (FH_VIEW_CMD=0, a child process)
    give identical outputs on partially replicated 4-key streams."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import numpy as np, sys
sys.path.insert(0, {root!r})
from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload
s = Workload.zipf(0.99, {keys}, k=4, views=3, window=64, seed={seed}, n=5,
                  shards={shards}).generate({n}, logs=True)
eng = Engine(s.key_space, n=5)
eng.stage(s)
eng.run()
r = eng.results()
np.savez(sys.argv[1], **r)
"""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        outs = []
        for i, env in enumerate(({}, {"FH_VIEW_CMD": "0"})):
            f = os.path.join(d, f"r{i}.npz")
            p = subprocess.run([sys.executable, "-c", code, f], capture_output=True, text=True,
                               timeout=200, env=dict(os.environ, **env))
            assert p.returncode == 0, p.stdout + p.stderr
            outs.append(np.load(f))
        for key in ("dep_off", "deps", "scc_label", "key_off", "key_seq"):
            assert np.array_equal(outs[0][key], outs[1][key]), key
