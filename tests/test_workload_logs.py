"""Host-side: the generator's per-replica arrival logs (fh_workload_generate_logs)
are the replicas' (time, index) orders of the same stream's fq_proc / fq_time
(no GPU needed)."""
import numpy as np
import pytest

from fantoch_amd.workload import Workload


def logs_from_times(s, nproc):
    out = []
    for r in range(1, nproc + 1):
        c, j = np.nonzero(s.fq_proc == r)
        t = s.fq_time[c, j]
        out.append(c[np.lexsort((c, t))].astype(np.uint32))
    return out


@pytest.mark.parametrize("kind,first", [("zipf", 0), ("zipf", 12345), ("rate", 7), ("pool", 0)])
def test_logs_match_times(kind, first):
    kw = dict(views=3, window=64, seed=99, n=5)
    w = {"zipf": lambda: Workload.zipf(0.99, 1 << 12, k=1, **kw),
         "rate": lambda: Workload.conflict_rate_(10, k=1, **kw),
         "pool": lambda: Workload.conflict_pool(100, 16, k=2, **kw)}[kind]()
    s = w.generate(20_000, first=first, logs=True)
    want = logs_from_times(s, 5)
    assert s.log_off[0] == 0 and s.log_off[-1] == s.n * 3
    for r in range(5):
        got = s.log_cmd[s.log_off[r]:s.log_off[r + 1]]
        assert np.array_equal(got, want[r])


def test_logs_small_window_and_other_n():
    w = Workload.zipf(0.9, 100, k=2, views=4, window=8, seed=3, n=7)
    s = w.generate(5_000, first=3, logs=True)
    want = logs_from_times(s, 7)
    for r in range(7):
        assert np.array_equal(s.log_cmd[s.log_off[r]:s.log_off[r + 1]], want[r])


def test_shard_generator_partitions_the_stream():
    """fh_workload_generate_shard: the key shards partition the stream (global
    dots, stream order) and each shard's logs are the replicas' logs of the
    whole stream restricted to the shard."""
    w = Workload.zipf(0.99, 1 << 10, k=1, views=3, window=64, seed=5)
    full = w.generate(30_000, first=11, logs=True)
    parts = [w.generate_shard(30_000, 3, s, first=11) for s in range(3)]
    assert sum(p.n for p in parts) == full.n
    for s, p in enumerate(parts):
        mine = np.nonzero(full.keys[:, 0] % 3 == s)[0]
        assert np.array_equal(p.dots, full.dots[mine])
        assert np.array_equal(p.keys, full.keys[mine])
        local = np.full(full.n, -1, dtype=np.int64)
        local[mine] = np.arange(len(mine))
        for r in range(5):
            fl = full.log_cmd[full.log_off[r]:full.log_off[r + 1]].astype(np.int64)
            want = local[fl][local[fl] >= 0]
            assert np.array_equal(p.log_cmd[p.log_off[r]:p.log_off[r + 1]], want)


# ---- partial replication (fh_workload.shards, BASELINE config C5) ----------

@pytest.mark.parametrize("shards,k,first", [(8, 4, 0), (8, 4, 31_337), (3, 2, 5), (1, 3, 0)])
def test_partial_stream_dots_views_and_element_logs(shards, k, first):
    """Shard h holds processes 5h+1..5h+5 (fantoch/src/util.rs:115-122); a
    command's dot is the next id of its target shard's coordinator (first
    key's shard, client/workload.rs:172-176; id.rs:59-61, 88-91); each key
    slot's views are its shard's collect; the element logs are each
    process's (time, command, slot) order of exactly those views."""
    w = Workload.zipf(0.99, 1 << 12, k=k, views=3, window=64, seed=77, n=5, shards=shards)
    whole = w.generate(first + 20_000)
    s = w.generate(20_000, first=first, logs=True, element_logs=True)
    assert np.array_equal(s.dots, whole.dots[first:]) and np.array_equal(s.keys, whole.keys[first:])
    src = (whole.dots >> np.uint64(56)).astype(np.int64)
    seq = (whole.dots & np.uint64((1 << 56) - 1)).astype(np.int64)
    i = np.arange(whole.n)
    if shards > 1:
        t = (whole.keys[:, 0] % np.uint64(shards)).astype(np.int64)
        assert np.array_equal(src, 5 * t + 1 + i % 5), "coordinator of the target shard"
        for p in np.unique(src):
            assert np.array_equal(seq[src == p], np.arange(1, (src == p).sum() + 1)), "DotGen"
        h = (s.keys % np.uint64(shards)).astype(np.int64)
        assert np.array_equal((s.fq_proc[:, :, 0].astype(np.int64) - 1) // 5, h), "slot's shard"
        fp = s.fq_proc.reshape(s.n, k, 3)
        ft = s.fq_time.reshape(s.n, k, 3)
    else:
        assert np.array_equal(src, 1 + i % 5) and np.array_equal(seq, i // 5 + 1)
        fp = np.repeat(s.fq_proc[:, None, :], k, axis=1)
        ft = np.repeat(s.fq_time[:, None, :], k, axis=1)
    assert len(s.log_off) == 5 * shards + 1 and s.log_off[-1] == s.n * k * 3
    pos = s.log_elem.astype(np.int64)
    assert np.array_equal(np.sort(pos), np.arange(s.n * k * 3)), "every element once"
    for r in range(5 * shards):
        e = pos[s.log_off[r]:s.log_off[r + 1]]
        c, j, sl = e // (3 * k), (e // k) % 3, e % k
        assert np.all(fp[c, sl, j] == r + 1), "element of this process"
        tt = ft[c, sl, j].astype(np.int64)
        order = np.lexsort((e, tt))
        assert np.array_equal(order, np.arange(len(e))), "(time, position) order"
    want = sum(int(((fp == r + 1)).sum()) for r in range(5 * shards))
    assert want == s.n * k * 3


def test_partial_union_differs_from_one_shard():
    """The oracle's partial-replication union (every shard's own collect,
    unioned) is not what one fully replicated KeyDeps gives on the same
    commands: independent per-shard arrival orders create cross-shard
    cycles (SCCs grow)."""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fullsize import shard_union
    from oracle import oracle as O
    s = Workload.zipf(0.99, 1 << 20, k=4, views=3, window=64, seed=58, shards=8).generate(3000)
    off, deps = shard_union(s)
    t_slot = np.argmax((s.keys % np.uint64(8)) == (s.keys[:, :1] % np.uint64(8)), axis=1)
    idx = np.arange(s.n)
    proc = ((s.fq_proc[idx, t_slot].astype(np.int64) - 1) % 5 + 1).astype(np.uint8)
    off1, deps1 = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), proc,
                              s.fq_time[idx, t_slot])
    a = np.split(deps, off[1:-1].astype(np.int64))
    b = np.split(deps1, off1[1:-1].astype(np.int64))
    assert sum(not np.array_equal(x, y) for x, y in zip(a, b)) > s.n // 10
    ko, kk = s.key_off(), s.keys.reshape(-1)
    _, lab, _, _ = O.graph_run(s.dots, ko, kk, off, deps, s.key_space)
    _, lab1, _, _ = O.graph_run(s.dots, ko, kk, off1, deps1, s.key_space)
    assert np.unique(lab, return_counts=True)[1].max() > np.unique(lab1, return_counts=True)[1].max()
