"""Shared definitions of the full-size parity fixtures (tests/golden/digests.json,
written by tests/golden/make_digests.py from the oracle, checked on the GPU by
tests/test_fullsize_gpu.py): the configurations, the canonical output digests
and the full-size property checks."""
from __future__ import annotations

import hashlib

import numpy as np

from fantoch_amd.workload import Workload

SEED = 0xFA170C4000000000
KW = dict(views=3, window=64, n=5)

CONFIGS = {
    "c1": dict(desc="C1 Atlas n=5 f=1, ConflictRate 10%, 1 key, 10k commands (full)", n=10_000,
               workload=lambda: Workload.conflict_rate_(10, k=1, seed=SEED + 1, **KW)),
    "c4": dict(desc="C4 Zipf 0.99 over 2^20 keys, 1 key, 100M commands (full, bench.py stream)",
               n=100_000_000,
               workload=lambda: Workload.zipf(0.99, 1 << 20, k=1, seed=SEED + 4, **KW)),
    "c4shard": dict(desc="C4 key shard 0 of 8 of a 20M-command stream (global dots)",
                    total=20_000_000, nshards=8, shard=0,
                    workload=lambda: Workload.zipf(0.99, 1 << 20, k=1, seed=SEED + 4, **KW)),
    "c3": dict(desc="C3 EPaxos ConflictPool 100% (key 0 + 16-key pool), 2 keys: deps at 10M, "
                    "everything on the first 50k", n=10_000_000, prefix=50_000,
               workload=lambda: Workload.conflict_pool(100, 16, k=2, seed=SEED + 3, **KW)),
    "c5": dict(desc="C5 Zipf 0.99 over 2^20 keys, 4 keys: deps at 12.5M, everything on the "
                    "first 30k", n=12_500_000, prefix=30_000,
               workload=lambda: Workload.zipf(0.99, 1 << 20, k=4, seed=SEED + 5, **KW)),
}


def _sha(*arrays):
    h = hashlib.sha256()
    for a, dt in arrays:
        h.update(np.ascontiguousarray(a, dtype=dt).tobytes())
    return h.hexdigest()


def digest_deps(dep_off, deps):
    return _sha((dep_off, "<u4"), (deps, "<u8"))


def digest_labels(labels):
    return _sha((labels, "<u8"))


def digest_perkey(key_off, key_seq):
    return _sha((key_off, "<u4"), (key_seq, "<u8"))


def cmd_index(dots, n, first=0):
    """Generator dots -> command index (DotGen: command i is process 1 + i % n
    with sequence i / n + 1, fantoch/src/id.rs:88-91)."""
    d = np.asarray(dots, dtype=np.uint64)
    p = (d >> np.uint64(56)).astype(np.int64)
    q = (d & np.uint64((1 << 56) - 1)).astype(np.int64)
    return (q - 1) * n + (p - 1) - first


def check_properties(s, r):
    """Full-size properties of an engine result on stream s (no oracle):
    * execution order respects every dependency edge across SCCs;
    * inside an SCC the execution order is dot order;
    * per-key sequences hold exactly each key's commands;
    * the SCC partition equals an independent SCC computation (scipy) over
      the committed deps, and every SCC's label is its minimum dot."""
    n = s.n
    dep_off = r["dep_off"].astype(np.int64)
    deps = r["deps"]
    lab = r["scc_label"]
    rank = r["exec_rank"].astype(np.int64)
    assert np.array_equal(np.sort(rank), np.arange(n)), "exec ranks are a permutation"
    first = 0
    idx = cmd_index(deps, 5, first)
    src = np.repeat(np.arange(n), np.diff(dep_off))
    inb = (idx >= 0) & (idx < n)
    src_i, dst_i = src[inb], idx[inb]
    assert np.array_equal(s.dots[dst_i], deps[inb]), "dep dots resolve to stream commands"
    cross = lab[src_i] != lab[dst_i]
    assert np.all(rank[dst_i[cross]] < rank[src_i[cross]]), "deps across SCCs execute first"
    # dot order inside SCCs along the execution order
    order = np.argsort(rank)
    lo, do = lab[order], s.dots[order]
    same = lo[1:] == lo[:-1]
    assert np.all(do[1:][same] > do[:-1][same]), "SCC members run in dot order"
    # SCC members contiguous in execution order
    starts = np.concatenate([[True], lo[1:] != lo[:-1]])
    assert len(np.unique(lo)) == int(starts.sum()), "SCC members contiguous"
    # labels are the min dot
    u, inv = np.unique(lab, return_inverse=True)
    mn = np.full(len(u), np.iinfo(np.uint64).max, dtype=np.uint64)
    np.minimum.at(mn, inv, s.dots)
    assert np.array_equal(mn, u), "label = min dot of the SCC"
    # per-key sequences: each key's commands, in execution order
    keys = s.keys.reshape(-1)
    cnt = np.bincount(keys.astype(np.int64), minlength=s.key_space)
    assert np.array_equal(np.diff(r["key_off"].astype(np.int64)), cnt), "per-key lengths"
    kcmd = np.repeat(np.arange(n), s.k)
    want = np.lexsort((rank[kcmd], keys))
    assert np.array_equal(r["key_seq"], s.dots[kcmd[want]]), "per-key sequence = exec order"
    # the SCC partition itself, recomputed independently over the committed
    # deps (scipy's strongly connected components, Pearce's algorithm)
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import connected_components
    g = csr_matrix((np.ones(len(src_i), dtype=np.int8), (src_i, dst_i)), shape=(n, n))
    ncomp, comp = connected_components(g, directed=True, connection="strong")
    assert ncomp == len(u), "number of SCCs"
    pairs = np.unique(comp.astype(np.int64) * len(u) + inv)
    assert len(pairs) == ncomp, "SCC partition equals an independent SCC computation"
