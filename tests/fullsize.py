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
    # the same stream's shard 0 of 8 under the balanced key map the multi-GPU
    # bench uses (fh_key_owners_balanced over the stream's key counts)
    "c4shard_bal": dict(desc="C4 balanced key shard 0 of 8 of a 20M-command stream (global dots; "
                             "owner = fh_key_owners_balanced over the stream's key counts)",
                        total=20_000_000, nshards=8, shard=0, balanced=True,
                        workload=lambda: Workload.zipf(0.99, 1 << 20, k=1, seed=SEED + 4, **KW)),
    # the shard holding the hottest key under the work-weighted key map
    # bench.py --gpus N uses (key_owners_weighted: the hot key's commands
    # weighted by their cost, so this shard holds fewer commands)
    "c4shard_w": dict(desc="C4 work-weighted key shard 0 of 8 of a 20M-command stream (global "
                           "dots; owner = key_owners_weighted over the stream's key counts)",
                      total=20_000_000, nshards=8, shard=0, weighted=True,
                      workload=lambda: Workload.zipf(0.99, 1 << 20, k=1, seed=SEED + 4, **KW)),
    "c3": dict(desc="C3 EPaxos ConflictPool 100% (key 0 + 16-key pool), 2 keys: deps at 10M, "
                    "everything on the first 50k", n=10_000_000, prefix=50_000,
               workload=lambda: Workload.conflict_pool(100, 16, k=2, seed=SEED + 3, **KW)),
    # the 4-key stream's first 12.5M commands, unsharded (one KeyDeps per
    # replica over all keys): deps at 12.5M, everything on the first 30k
    "c5_12m": dict(desc="Zipf 0.99 over 2^20 keys, 4 keys, unsharded: deps at 12.5M, everything "
                        "on the first 30k", n=12_500_000, prefix=30_000,
                   workload=lambda: Workload.zipf(0.99, 1 << 20, k=4, seed=SEED + 5, **KW)),
    # C5 as BASELINE.json states it: Atlas partial replication over 8 key
    # shards (shard = key mod 8), 4 keys/cmd, 100M commands.  Shard h holds
    # processes 5h+1..5h+5 (fantoch/src/util.rs:115-122); a command's dot
    # comes from its target shard (its first key's, id.rs:59-61) and every
    # shard it touches collects it with its own fast quorum and arrival
    # delays (atlas.rs:214-328); committed deps = the union of the shards'
    # reports (MShardCommit, atlas.rs:559-639).  Deps at 100M, everything on
    # the first 20k (one SCC holds ~90% of a prefix: the incremental Tarjan
    # is quadratic).
    "c5": dict(desc="C5 Atlas partial replication, 8 key shards (key mod 8, processes 5h+1..5h+5), "
                    "Zipf 0.99 over 2^20 keys, 4 keys/cmd, 100M commands: committed deps = union "
                    "over the shards' own collects; everything on the first 20k",
               n=100_000_000, shards=8, prefix=20_000,
               workload=lambda: Workload.zipf(0.99, 1 << 20, k=4, seed=SEED + 5, shards=8, **KW)),
}


def shard_union(s, log=None, lean=False):
    """The oracle's committed deps of a partially replicated stream: every
    shard's replicas run per-replica SequentialKeyDeps + the fast-quorum
    union over the commands' keys on that shard, in that shard's own arrival
    orders (oracle fo_views_run on Stream.shard_views), and a command's deps
    are the union over its shards (MShardCommit, atlas.rs:559-639, union
    :580-583).  Records are packed command << 32 | source << 26 | sequence,
    so one u64 sort + unique is the union and leaves each row in ascending
    dot order.  `s` may be a function returning the stream; with `lean` it is
    regenerated per shard (the 100M digest's memory).  Test infrastructure
    (the oracle)."""
    from oracle import oracle as O
    make = s if callable(s) else (lambda: s)
    st = make()
    n, shards, nproc = st.n, st.shards, st.nproc * st.shards
    assert n < (1 << 31) and int((st.dots >> np.uint64(56)).max()) < 64
    assert int((st.dots & np.uint64((1 << 56) - 1)).max()) < (1 << 26)
    recs = []
    for sh in range(shards):
        if st is None:
            st = make()
        cmds, ko, kk, fp, ft = st.shard_views(sh)
        dots = st.dots[cmds]
        if lean:
            st = None
        off, deps = O.views_run(0, nproc, dots, ko, kk, fp, ft)
        del dots, ko, kk, fp, ft
        per = np.diff(off.astype(np.int64))
        r = np.repeat(cmds.astype(np.uint64), per) << np.uint64(32)
        r |= (deps >> np.uint64(56)) << np.uint64(26)
        r |= deps & np.uint64((1 << 26) - 1)
        recs.append(r)
        del off, deps, per, cmds
        if log:
            log(f"shard {sh}: {len(r)} records")
    del st
    rec = np.concatenate(recs)
    del recs
    rec.sort()
    keep = np.ones(len(rec), dtype=bool)
    keep[1:] = rec[1:] != rec[:-1]
    rec = rec[keep]
    del keep
    cmd = (rec >> np.uint64(32)).astype(np.int64)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(cmd, minlength=n), out=off[1:])
    del cmd
    lo = rec & np.uint64(0xFFFFFFFF)
    del rec
    deps = ((lo >> np.uint64(26)) << np.uint64(56)) | (lo & np.uint64((1 << 26) - 1))
    return off.astype(np.uint32), deps


def shard_stream(s, nshards: int, shard: int):
    """Shard `shard`'s part of a stream with replica views (key = global id):
    (global command indices with a key on the shard, key_off CSR, the keys on
    the shard in the command's key order)."""
    mine = s.keys % np.uint64(nshards) == np.uint64(shard)
    cnt = mine.sum(axis=1)
    cmds = np.nonzero(cnt)[0]
    key_off = np.zeros(len(cmds) + 1, dtype=np.uint32)
    np.cumsum(cnt[cmds], out=key_off[1:])
    return cmds, key_off, s.keys[cmds][mine[cmds]]


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


class DotIndex:
    """dot -> command index for any stream whose per-source sequences are
    1, 2, ... (DotGen, id.rs:88-91): a table over (source, sequence), sized n
    plus the sources.  Under partial replication a dot's source is its
    target shard's coordinator, so the index is not arithmetic."""

    def __init__(self, dots):
        d = np.asarray(dots, dtype=np.uint64)
        src = (d >> np.uint64(56)).astype(np.int64)
        seq = (d & np.uint64((1 << 56) - 1)).astype(np.int64)
        cnt = np.bincount(src, minlength=256)
        self.base = np.zeros(257, dtype=np.int64)
        np.cumsum(cnt + 1, out=self.base[1:])
        assert seq.min(initial=1) >= 1 and np.all(seq <= cnt[src]), "per-source sequences 1.."
        self.table = np.full(int(self.base[-1]), -1, dtype=np.int64)
        self.table[self.base[src] + seq] = np.arange(len(d))
        self.n = len(d)

    def __call__(self, dots):
        d = np.asarray(dots, dtype=np.uint64)
        src = (d >> np.uint64(56)).astype(np.int64)
        seq = (d & np.uint64((1 << 56) - 1)).astype(np.int64)
        at = self.base[src] + seq
        ok = (seq >= 1) & (at < self.base[src + 1])
        return np.where(ok, self.table[np.where(ok, at, 0)], -1)


def check_properties(s, r, chunk=1 << 24, log=None):
    """Full-size properties of an engine result on stream s (no oracle):
    * execution order respects every dependency edge across SCCs;
    * inside an SCC the execution order is dot order, SCC members are
      contiguous in it, and every SCC's label is its minimum dot;
    * per-key sequences hold exactly each key's commands, in execution order;
    * the SCC partition equals an independent SCC computation (scipy's
      strongly connected components, Pearce's algorithm) over the committed
      deps.
    Linear-time and chunked (C5 at 100M: 856M deps, 400M per-key elements)."""
    log = log or (lambda m: None)
    n = s.n
    index = DotIndex(s.dots)
    dep_off = r["dep_off"].astype(np.int64)
    deps = r["deps"]
    lab = r["scc_label"]
    rank = r["exec_rank"].astype(np.int64)
    assert rank.min() >= 0 and rank.max() < n, "exec ranks in range"
    assert np.all(np.bincount(rank, minlength=n) == 1), "exec ranks are a permutation"
    order = np.empty(n, dtype=np.int64)
    order[rank] = np.arange(n)
    # every dependency: a stream command, in the same SCC or executed earlier
    idx = np.empty(len(deps), dtype=np.int32)
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        e0, e1 = int(dep_off[c0]), int(dep_off[c1])
        d = index(deps[e0:e1])
        assert d.min(initial=0) >= 0 and d.max(initial=-1) < n, "deps are stream commands"
        assert np.array_equal(s.dots[d], deps[e0:e1]), "dep dots resolve to stream commands"
        src = np.repeat(np.arange(c0, c1), np.diff(dep_off[c0:c1 + 1]))
        cross = lab[src] != lab[d]
        assert np.all(rank[d[cross]] < rank[src[cross]]), "deps across SCCs execute first"
        idx[e0:e1] = d
    log("properties: dependency edges ok")
    # SCCs along the execution order: contiguous, dot order inside, label =
    # the first (= minimum) member's dot
    lo, do = lab[order], s.dots[order]
    head = np.ones(n, dtype=bool)
    head[1:] = lo[1:] != lo[:-1]
    inner = ~head[1:]
    assert np.all(do[1:][inner] > do[:-1][inner]), "SCC members run in dot order"
    assert np.array_equal(lo[head], do[head]), "label = min dot of the SCC"
    heads = lo[head]
    nscc = len(heads)
    assert len(np.unique(heads)) == nscc, "SCC members contiguous in the execution order"
    del lo, do, head, inner, heads
    log("properties: SCC order and labels ok")
    # per-key sequences: each key's commands in execution order
    keys = s.keys
    cnt = np.bincount(keys.reshape(-1).astype(np.int64), minlength=s.key_space)
    key_off = r["key_off"].astype(np.int64)
    assert np.array_equal(np.diff(key_off), cnt), "per-key lengths"
    seq = r["key_seq"]
    nel = len(seq)
    for j0 in range(0, nel, chunk):
        j1 = min(nel, j0 + chunk)
        c = index(seq[j0:j1])
        assert c.min(initial=0) >= 0 and c.max(initial=-1) < n, "per-key dots are commands"
        kk = np.searchsorted(key_off, np.arange(j0, j1), side="right") - 1
        assert np.all((keys[c] == kk[:, None].astype(np.uint64)).any(axis=1)), \
            "per-key element of a command holding the key"
        rk = rank[c]
        same = kk[1:] == kk[:-1]
        assert np.all(rk[1:][same] > rk[:-1][same]), "per-key sequence in execution order"
        if j1 < nel:  # the seam between chunks
            c2 = index(seq[j1:j1 + 1])
            k2 = np.searchsorted(key_off, j1, side="right") - 1
            assert k2 != kk[-1] or rank[c2[0]] > rk[-1], "per-key sequence in execution order"
    # (every element belongs to a command holding its key, each key's ranks
    # strictly increase and the per-key counts match: exactly the pairs)
    log("properties: per-key sequences ok")
    # the SCC partition itself, recomputed independently (scipy)
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import connected_components
    g = csr_matrix((np.ones(len(idx), dtype=np.int8), idx, dep_off), shape=(n, n))
    ncomp, comp = connected_components(g, directed=True, connection="strong")
    del g, idx
    log(f"properties: scipy SCC done ({ncomp} SCCs)")
    assert ncomp == nscc, "number of SCCs"
    lab_of = np.empty(ncomp, dtype=np.uint64)
    lab_of[comp] = lab
    assert np.array_equal(lab_of[comp], lab), "SCC partition equals an independent SCC computation"
