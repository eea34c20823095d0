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
