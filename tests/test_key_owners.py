"""The balanced key -> shard map of the multi-GPU C4 path
(fh_key_owners_balanced, include/fantoch_hip.h): deterministic greedy
largest-first packing of the per-key command counts.  The reference assigns
key shards by hash (fantoch/src/client/workload.rs:203-205); key % N left the
largest of 8 shards of the C4 stream at 1.37x the mean under Zipf 0.99."""
import numpy as np

from fantoch_amd.workload import Workload, key_owners_balanced

C4_SEED = 0xFA170C4000000004


def c4():
    return Workload.zipf(0.99, 1 << 20, k=1, views=3, window=64, seed=C4_SEED, n=5)


def test_c4_100m_shards_balanced_at_2_4_8():
    w = c4()
    h = w.key_histogram(100_000_000)
    assert int(h.sum()) == 100_000_000
    for n in (2, 4, 8):
        o = key_owners_balanced(h, n)
        loads = np.bincount(o, weights=h.astype(np.float64), minlength=n)
        assert loads.max() <= 1.05 * loads.mean(), (n, loads)
        mod = np.bincount(np.arange(len(h)) % n, weights=h.astype(np.float64), minlength=n)
        assert loads.max() < mod.max()  # better than key mod N on Zipf


def test_greedy_rule_and_determinism():
    h = np.array([5, 9, 0, 9, 3, 1, 7], dtype=np.uint64)
    o = key_owners_balanced(h, 3)
    # descending counts, ties by key: 1 (9) -> 0, 3 (9) -> 1, 6 (7) -> 2,
    # 0 (5) -> 2 (load 7), 4 (3) -> 0 (9 vs 9 vs 12: lowest shard), 5 (1) -> 1,
    # 2 (0) -> 1 (loads 12, 10, 12)
    assert o.tolist() == [2, 0, 1, 1, 0, 1, 2]
    assert np.array_equal(key_owners_balanced(h, 3), o)
    assert np.array_equal(key_owners_balanced(h, 1), np.zeros(len(h), dtype=np.uint32))


def test_owned_shards_partition_the_stream():
    w = c4()
    total = 200_000
    o = key_owners_balanced(w.key_histogram(total), 4)
    full = w.generate(total)
    seen = []
    for q in range(4):
        g = w.generate_shard(total, 4, q, owner=o)
        assert np.all(o[g.keys[:, 0]] == q)
        assert int(g.log_off[-1]) == g.n * 3
        seen.append(g.dots)
    allv = np.sort(np.concatenate(seen))
    assert np.array_equal(allv, np.sort(full.dots))


def test_c4_100m_work_weighted_map():
    """key_owners_weighted: the same packing over key_weights (count x (1 +
    HOT_KEY_COST x share)); the shard holding the hottest key gets fewer
    commands, every shard's estimated work stays within 5 % of the mean, and
    the map is a function of the counts alone (every rank computes it)."""
    from fantoch_amd.workload import HOT_KEY_COST, key_owners_weighted, key_weights
    w = c4()
    h = w.key_histogram(100_000_000)
    wt = key_weights(h)
    hot = int(np.argmax(h))
    share = float(h[hot]) / float(h.sum())
    assert abs(float(wt[hot]) / (16.0 * float(h[hot])) - (1 + HOT_KEY_COST * share)) < 1e-6
    for n in (2, 4, 8):
        o = key_owners_weighted(h, n)
        assert np.array_equal(o, key_owners_weighted(h.copy(), n))
        work = np.bincount(o, weights=wt.astype(np.float64), minlength=n)
        assert work.max() <= 1.05 * work.mean(), (n, work)
        cmds = np.bincount(o, weights=h.astype(np.float64), minlength=n)
        assert cmds[o[hot]] == cmds.min()
