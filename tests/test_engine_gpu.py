"""The fused engine (fh_engine_*) against the oracle: bit-exact committed
deps, SCC partition (min-dot labels) and per-key execution sequences."""
import numpy as np
import pytest

from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def oracle_pipeline(s, nproc=5):
    """Reference CPU path on the same stream: SequentialKeyDeps (one view) or
    per-replica KeyDeps + QuorumDeps union (views), then GraphExecutor in
    arrival (= stream) order with the per-key monitor."""
    key_off = s.key_off()
    keys = s.keys.reshape(-1)
    if s.fq_proc is None:
        dep_off, deps = O.keydeps_run(s.dots, key_off, keys)
    else:
        dep_off, deps = O.views_run(0, nproc, s.dots, key_off, keys, s.fq_proc, s.fq_time)
    ex, lab, kso, ks = O.graph_run(s.dots, key_off, keys, dep_off, deps, s.key_space)
    return dep_off, deps, ex, lab, kso, ks


def check_engine(s, nproc=5, batches=1, bounds=None):
    eng = Engine(s.key_space, n=nproc)
    dep_off, deps, ex, lab, kso, ks = oracle_pipeline(s, nproc)
    assert len(ex) == s.n, "oracle must execute every command"
    if batches == 1 and bounds is None:
        eng.stage(s, nproc)
        eng.run()
        r = eng.results()
        assert np.array_equal(r["dep_off"], dep_off)
        assert np.array_equal(r["deps"], deps)
        # SCC partition: label = min dot of the command's SCC
        want_label = dict(zip(ex.tolist(), lab.tolist()))
        got_label = dict(zip(s.dots.tolist(), r["scc_label"].tolist()))
        assert got_label == want_label
        # per-key execution sequence
        assert np.array_equal(r["key_off"], kso)
        assert np.array_equal(r["key_seq"], ks)
        # execution order respects every dependency edge
        rank = dict(zip(s.dots.tolist(), r["exec_rank"].tolist()))
        lab_of = got_label
        for i in range(min(s.n, 20000)):
            for d in deps[dep_off[i]:dep_off[i + 1]]:
                d = int(d)
                if lab_of[d] != lab_of[int(s.dots[i])]:
                    assert rank[d] < rank[int(s.dots[i])]
        return r
    # streaming batches: deps and per-key sequences concatenate
    if bounds is None:
        bounds = np.linspace(0, s.n, batches + 1).astype(int)
    got_off, got_deps, got_seq = [np.zeros(1, dtype=np.int64)], [], {}
    base = 0
    for a, b in zip(bounds[:-1], bounds[1:]):
        sub = type(s)(s.dots[a:b], s.keys[a:b], None, None, s.key_space)
        eng.stage(sub, nproc)
        eng.run()
        r = eng.results()
        got_off.append(r["dep_off"][1:].astype(np.int64) + base)
        got_deps.append(r["deps"])
        base += len(r["deps"])
        ko = r["key_off"]
        for key in np.nonzero(np.diff(ko))[0]:
            got_seq.setdefault(int(key), []).append(r["key_seq"][ko[key]:ko[key + 1]])
    assert np.array_equal(np.concatenate(got_off), dep_off.astype(np.int64))
    assert np.array_equal(np.concatenate(got_deps), deps)
    keys_with = np.nonzero(np.diff(kso))[0]
    assert sorted(got_seq) == keys_with.tolist()
    for key in keys_with:
        assert np.array_equal(np.concatenate(got_seq[int(key)]), ks[kso[key]:kso[key + 1]])


@pytest.mark.parametrize("k", [1, 2])
def test_single_view_zipf(k):
    s = Workload.zipf(0.99, 2000, k=k, seed=3 + k).generate(30_000)
    check_engine(s)


def test_single_view_streaming_batches():
    s = Workload.zipf(0.7, 5000, k=1, seed=21).generate(40_000)
    check_engine(s, batches=4)


def test_single_view_hot_buckets_multichunk():
    """Buckets far larger than the bucket kernel's LDS chunk: 16 keys (one key
    per bucket) under Zipf 0.99, and a ConflictRate hot key (50%)."""
    check_engine(Workload.zipf(0.99, 16, k=1, seed=11).generate(60_000))
    check_engine(Workload.conflict_rate_(50, k=1, clients=64, seed=12).generate(50_000), batches=3)


def test_single_view_pipelined_hot_keys():
    """40 equally sized batches staged at once (each run() orders one batch and
    partitions the next in the same launch): the hot-key table fills after
    the first launch and is rebuilt at launch 32, between a batch's partition
    and its ordering, so the batch must be ordered with the keys it was
    partitioned with.  Zipf 0.9 over 2^14 keys gives dozens of keys above
    the hot threshold per batch (table churn)."""
    nb, m = 40, 30_000
    s = Workload.zipf(0.9, 1 << 14, k=1, seed=17).generate(nb * m)
    dep_off, deps, ex, lab, kso, ks = oracle_pipeline(s)
    eng = Engine(s.key_space)
    eng.stage_many([type(s)(s.dots[i * m:(i + 1) * m], s.keys[i * m:(i + 1) * m], None, None,
                            s.key_space) for i in range(nb)])
    got_off, got_deps, got_seq = [np.zeros(1, dtype=np.int64)], [], {}
    base = 0
    for _ in range(nb):
        eng.run()
        r = eng.results()
        got_off.append(r["dep_off"][1:].astype(np.int64) + base)
        got_deps.append(r["deps"])
        base += len(r["deps"])
        ko = r["key_off"]
        for key in np.nonzero(np.diff(ko))[0]:
            got_seq.setdefault(int(key), []).append(r["key_seq"][ko[key]:ko[key + 1]])
    assert np.array_equal(np.concatenate(got_off), dep_off.astype(np.int64))
    assert np.array_equal(np.concatenate(got_deps), deps)
    for key in np.nonzero(np.diff(kso))[0]:
        assert np.array_equal(np.concatenate(got_seq[int(key)]), ks[kso[key]:kso[key + 1]])


def test_single_view_bucket_then_sort_path():
    """A batch above the bucket plan's size limit (> 1024 tiles) between two
    bucket-path batches: both paths share the mapped latest table."""
    s = Workload.zipf(0.9, 1 << 12, k=1, seed=13).generate(4_250_000)
    check_engine(s, bounds=[0, 20_000, 4_230_000, 4_250_000])


def test_c1_atlas_n5_conflict10_views():
    """C1: Atlas n=5 f=1, ConflictRate 10%, 1 key, 10k cmds, replica views."""
    s = Workload.conflict_rate_(10, k=1, views=3, window=64, seed=1).generate(10_000)
    check_engine(s)


@pytest.mark.parametrize("w", [8, 64])
def test_c3_like_conflict_pool_views_large_sccs(w):
    """C3-like: 100% conflict on key 0 plus a pool key, EPaxos fq=3 views."""
    s = Workload.conflict_pool(100, 16, k=2, views=3, window=w, seed=5).generate(6_000)
    r = check_engine(s)
    # there are large SCCs
    _, counts = np.unique(r["scc_label"], return_counts=True)
    assert counts.max() > 50


def test_c4_like_zipf099_views():
    s = Workload.zipf(0.99, 1 << 14, k=1, views=3, window=64, seed=7).generate(40_000)
    r = check_engine(s)
    _, counts = np.unique(r["scc_label"], return_counts=True)
    assert counts.max() > 1  # non-trivial SCCs exist


def test_c5_like_multikey_views():
    s = Workload.zipf(0.99, 4096, k=4, views=3, window=64, seed=9).generate(8_000)
    check_engine(s)


def test_c2_full_size():
    """C2 at full size: 1M cmds, Zipf 0.7 over 1M keys, 1 key/cmd."""
    s = Workload.zipf(0.7, 1 << 20, k=1).generate(1_000_000)
    eng = Engine(s.key_space)
    eng.stage(s)
    eng.run()
    r = eng.results()
    dep_off, deps, ex, lab, kso, ks = oracle_pipeline(s)
    assert np.array_equal(r["dep_off"], dep_off)
    assert np.array_equal(r["deps"], deps)
    assert np.array_equal(r["key_off"], kso)
    assert np.array_equal(r["key_seq"], ks)


def test_c4_like_views_many_tiles():
    """C4 shape across many 4096-vertex tiles of the tile-local graph path."""
    s = Workload.zipf(0.99, 1 << 20, k=1, views=3, window=64, seed=0xFA170C4000000004).generate(
        150_000)
    check_engine(s)


def test_c1_full_views_conflict_rate():
    """C1 at its full size through the logs API (generator logs, not fq times)."""
    w = Workload.conflict_rate_(10, k=1, views=3, window=64, seed=2)
    s = w.generate(10_000, logs=True)
    eng = Engine(s.key_space, n=5)
    eng.stage_logs([s])
    eng.run()
    r = eng.results()
    dep_off, deps, ex, lab, kso, ks = oracle_pipeline(s)
    assert np.array_equal(r["dep_off"], dep_off) and np.array_equal(r["deps"], deps)
    assert dict(zip(s.dots.tolist(), r["scc_label"].tolist())) == dict(zip(ex.tolist(),
                                                                         lab.tolist()))
    assert np.array_equal(r["key_off"], kso) and np.array_equal(r["key_seq"], ks)


def test_views_wide_window_takes_global_path():
    """A reorder window far beyond the tile certificate (forward spans >= 1024)
    must fall back to the global SCC path and still match the oracle."""
    s = Workload.zipf(0.99, 1 << 12, k=1, views=3, window=3000, seed=8).generate(12_000)
    check_engine(s)


def test_rewind_replays_identically():
    s = Workload.zipf(0.99, 1 << 14, k=1, views=3, window=64, seed=4).generate(30_000, logs=True)
    eng = Engine(s.key_space, n=5)
    eng.stage(s)
    eng.run()
    r1 = eng.results()
    for _ in range(2):
        eng.rewind()
        eng.run()
    r2 = eng.results()
    for k in r1:
        assert np.array_equal(r1[k], r2[k]), k


@pytest.mark.parametrize("k,chunk", [(1, None), (1, "7000"), (2, "5000")])
def test_views_streaming_batches_and_chunks(k, chunk, monkeypatch):
    """Replica views fed as several batches of per-replica logs (each
    replica's batch b precedes its batch b + 1), state carried across batches;
    FH_VIEW_CHUNK splits each batch's logs into many KeyDeps chunks.  The
    oracle sees the same arrivals (times offset per batch)."""
    if chunk:
        monkeypatch.setenv("FH_VIEW_CHUNK", chunk)
    import subprocess, sys, json, os
    # the chunk size is read once per process: run in a child
    code = f"""
import numpy as np, sys
sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload, Stream
from oracle import oracle as O
w = Workload.zipf(0.99, 1 << 12, k={k}, views=3, window=64, seed=31)
nb, m = 4, 9000
parts = [w.generate(m, first=i * m, logs=True) for i in range(nb)]
eng = Engine(w.key_space(), n=5)
eng.stage_logs(parts)
dots = np.concatenate([p.dots for p in parts]); keys = np.concatenate([p.keys for p in parts])
proc = np.concatenate([p.fq_proc for p in parts])
tim = np.concatenate([p.fq_time + np.uint64(i) * np.uint64(1 << 40) for i, p in enumerate(parts)])
s = Stream(dots, keys, proc, tim, w.key_space())
key_off = s.key_off(); kk = s.keys.reshape(-1)
off, deps = O.views_run(0, 5, s.dots, key_off, kk, s.fq_proc, s.fq_time)
ex, lab, kso, ks = O.graph_run(s.dots, key_off, kk, off, deps, s.key_space)
lab_of = dict(zip(ex.tolist(), lab.tolist()))
got_off, got_deps, got_seq = [np.zeros(1, dtype=np.int64)], [], {{}}
base = 0
for i in range(nb):
    eng.run()
    r = eng.results()
    got_off.append(r["dep_off"][1:].astype(np.int64) + base); got_deps.append(r["deps"]); base += len(r["deps"])
    for d, l in zip(parts[i].dots.tolist(), r["scc_label"].tolist()):
        assert lab_of[d] == l
    ko = r["key_off"]
    for key in np.nonzero(np.diff(ko))[0]:
        got_seq.setdefault(int(key), []).append(r["key_seq"][ko[key]:ko[key + 1]])
assert np.array_equal(np.concatenate(got_off), off.astype(np.int64))
assert np.array_equal(np.concatenate(got_deps), deps)
for key in np.nonzero(np.diff(kso))[0]:
    assert np.array_equal(np.concatenate(got_seq[int(key)]), ks[kso[key]:kso[key + 1]])
print("ok")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("delay", [False, True])
def test_views_placement_strays_match_oracle(delay):
    """Dependency-code placement (engine.hip place_codes) when the base hint
    is wrong, so elements are placed directly as strays: a zero slack
    (FH_PLACE_SLACK=0) makes every arrival ahead of the replicas' first
    entries a stray, and with `delay` replica 1 receives its member events
    after all of its coordinator events (its slices then span the whole
    stream).  Small chunks (FH_VIEW_CHUNK); both are read once per process,
    so the run is a child process.  Deps-only against the oracle's KeyDeps +
    union."""
    import subprocess, sys, os
    code = f"""
import numpy as np, sys
sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload
from oracle import oracle as O
s = Workload.zipf(0.99, 4096, k=1, views=3, window=64, seed=5).generate(60_000)
if {delay}:
    t = s.fq_time.copy()
    m = s.fq_proc == 1
    m[:, 0] = False  # member events only: the coordinator's stay first
    t[m] += np.uint64(1 << 39)
    s.fq_time = t
eng = Engine(s.key_space, n=5)
eng.set_deps_only(True)
eng.stage(s)
eng.run()
off, deps = eng.deps()
o_off, o_deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc, s.fq_time)
assert np.array_equal(off, o_off) and np.array_equal(deps, o_deps)
print("ok")
"""
    env = dict(os.environ, FH_VIEW_CHUNK="20000", FH_PLACE_SLACK="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=200,
                       env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_views_command_level_path_matches_oracle():
    """The command-level KeyDeps path (engine.hip k_cmd_pack / k_cmd_search,
    the default for one key per command; a child process, as the knob is
    read once): a C4-shaped stream, and a streamed multi-batch one whose
    reorder window (200) leaves the packed arrival positions fewer spare
    bits, against the oracle."""
    import subprocess, sys, os
    code = f"""
import numpy as np, sys
sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload, Stream
from oracle import oracle as O
s = Workload.zipf(0.99, 1 << 16, k=1, views=3, window=64, seed=12).generate(120_000, logs=True)
eng = Engine(s.key_space, n=5)
eng.stage_logs([s])
eng.run()
r = eng.results()
off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc, s.fq_time)
ex, lab, kso, ks = O.graph_run(s.dots, s.key_off(), s.keys.reshape(-1), off, deps, s.key_space)
assert np.array_equal(r["dep_off"], off) and np.array_equal(r["deps"], deps)
assert np.array_equal(r["key_off"], kso) and np.array_equal(r["key_seq"], ks)
w = Workload.zipf(0.99, 1 << 10, k=1, views=3, window=200, seed=13)
parts = [w.generate(8000, first=i * 8000, logs=True) for i in range(3)]
eng = Engine(w.key_space(), n=5)
eng.stage_logs(parts)
dots = np.concatenate([p.dots for p in parts]); keys = np.concatenate([p.keys for p in parts])
proc = np.concatenate([p.fq_proc for p in parts])
tim = np.concatenate([p.fq_time + np.uint64(i) * np.uint64(1 << 40) for i, p in enumerate(parts)])
st = Stream(dots, keys, proc, tim, w.key_space())
off, deps = O.views_run(0, 5, st.dots, st.key_off(), st.keys.reshape(-1), st.fq_proc, st.fq_time)
got = []
for i in range(3):
    eng.run()
    got.append(eng.results()["deps"])
assert np.array_equal(np.concatenate(got), deps)
print("ok")
"""
    env = dict(os.environ, FH_VIEW_CMD="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=200,
                       env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("env", [
    {},
    {"FH_KO_SIDE": "0"},
    {"FH_KEYORDER": "0"},
    {"FH_VIEW_CMD": "0"},
    {"FH_VIEW_CMD": "0", "FH_PLACE_SLACK": "0"},
])
def test_views_kernel_variants_match_oracle(env):
    """The replica-view paths (read once per process: a child process): the
    command-level path (default) and the chunked one (FH_VIEW_CMD=0), each
    against the oracle on a hot-key stream cut into chunks of 20,000
    elements, so that segments cross the bucketing workgroups and chunks: the
    segment tails written by k_bucket_codes in place or, for a segment begun
    in an earlier workgroup, deferred to k_place; with a zero placement
    slack every reordered arrival is a stray."""
    import subprocess, sys, os
    code = f"""
import numpy as np, sys
sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload
from oracle import oracle as O
s = Workload.zipf(1.2, 1 << 12, k=1, views=3, window=64, seed=31).generate(90_000, logs=True)
eng = Engine(s.key_space, n=5)
eng.stage_logs([s])
for _ in range(2):
    eng.rewind()
    eng.run()
    r = eng.results()
off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc, s.fq_time)
ex, lab, kso, ks = O.graph_run(s.dots, s.key_off(), s.keys.reshape(-1), off, deps, s.key_space)
assert np.array_equal(r["dep_off"], off) and np.array_equal(r["deps"], deps)
assert np.array_equal(r["key_off"], kso) and np.array_equal(r["key_seq"], ks)
m = dict(zip(ex.tolist(), lab.tolist()))
assert np.array_equal(r["scc_label"], np.asarray([m[int(d)] for d in s.dots], np.uint64))
print("ok")
"""
    e = dict(os.environ, FH_VIEW_CHUNK="20000", **env)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=200,
                       env=e)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("window,seed", [(64, 21), (80, 22)])
def test_views_mixed_tile_bounds_match_oracle(window, seed):
    """The tile kernel's mixed reach bounds (graph_tile.hip tiles_mixed):
    wider reorder windows raise the maximum excess, so more pass-1 tiles fail
    at R0 = 512 and pass 2 reruns them (and their neighbours) at a larger
    bound.  Twice on one engine: the first run starts from the default bound,
    the second from the one the first run measured."""
    s = Workload.zipf(0.99, 1 << 16, k=1, views=3, window=window, seed=seed).generate(200_000)
    dep_off, deps, ex, lab, kso, ks = oracle_pipeline(s)
    eng = Engine(s.key_space, n=5)
    eng.stage(s)
    want_label = dict(zip(ex.tolist(), lab.tolist()))
    for _ in range(2):
        eng.rewind()
        eng.run()
        r = eng.results()
        assert np.array_equal(r["dep_off"], dep_off) and np.array_equal(r["deps"], deps)
        assert dict(zip(s.dots.tolist(), r["scc_label"].tolist())) == want_label
        assert np.array_equal(r["key_off"], kso) and np.array_equal(r["key_seq"], ks)


@pytest.mark.parametrize("views,nproc,n,keys", [(1, 1, 30_000, 1 << 12), (2, 3, 30_000, 1 << 12),
                                                (4, 5, 30_000, 1 << 12),
                                                (3, 5, 4_500_000, 1 << 20)])
def test_views_command_level_quorum_sizes(views, nproc, n, keys):
    """The command-level KeyDeps path (k_cmd_search) at every fast-quorum size
    it takes (1-3: codes through region records and k_code_scatter; 4: direct
    stores), with the tails found from predecessor marks (in-tile and across
    tiles); the 4.5M-command case spans two 4M-command code regions.  Each
    fast quorum intersects every other (views > nproc / 2), as Atlas/EPaxos
    require: with disjoint quorums two commands on one key need not be
    connected, and the reference's per-key order then follows its hash-set
    iteration (oracle.c check_pending)."""
    s = Workload.zipf(0.99, keys, k=1, views=views, window=64, seed=40 + views,
                      n=nproc).generate(n)
    check_engine(s, nproc=nproc)


@pytest.mark.parametrize("window,keys,seed", [(1024, 16, 21), (2048, 64, 22), (300, 8, 23),
                                             (1024, 256, 24), (600, 1024, 25)])
def test_keyorder_long_edges(window, keys, seed):
    """Hot keys under a wide reorder window: key-order edges far longer than
    the 8-bit distances the search writes (the -128 escapes to full
    positions), and tile reach bounds well above the key-order floor; the
    batch is ordered by the key-order path, or handed to the command-order
    path if the tile certificate fails -- either way equal to the oracle."""
    s = Workload.zipf(1.2, keys, k=1, views=3, window=window, seed=seed).generate(40_000,
                                                                                  logs=True)
    eng = Engine(s.key_space, n=5)
    eng.stage(s)
    for _ in range(2):  # a second run on the learned reach bound
        eng.rewind()
        eng.run()
        r = eng.results()
        off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc,
                                s.fq_time)
        ex, lab, kso, ks = O.graph_run(s.dots, s.key_off(), s.keys.reshape(-1), off, deps,
                                       s.key_space)
        assert np.array_equal(r["dep_off"], off) and np.array_equal(r["deps"], deps)
        assert dict(zip(s.dots.tolist(), r["scc_label"].tolist())) == dict(
            zip(ex.tolist(), lab.tolist()))
        assert np.array_equal(r["key_off"], kso) and np.array_equal(r["key_seq"], ks)
