"""Partial replication, whole pipeline (SURVEY.md §8e, C5 shape) on CPU:
world_size-2 gloo processes, each a key shard, run
fantoch_amd.partial.PartialPipeline over a 4-keys-per-command Zipf stream with
replica views -- per-shard KeyDeps over the owned keys (pseudo commands), the
all-to-all of (command, dep) records, the owner's union, the all-gather of the
committed rows, the graph, the shard's per-key sequences.  The oracle stands in
for the GPU stages (no GPU here; tests/test_partial_pipeline_gpu.py runs the
HIP stages).  Checked against the oracle on the UNSHARDED stream: committed
deps of every command, the SCC partition, and every key's execution sequence
(atlas.rs:559-639 union semantics, executor/graph/mod.rs order)."""
import os
import socket
import sys

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

N_CMD, WORLD = 3000, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def stream():
    from fantoch_amd.workload import Workload
    w = Workload.zipf(0.99, 512, k=4, views=3, window=64, seed=77, n=5)
    return w.generate(N_CMD, logs=True, times=True)


def oracle_keydeps(ps):
    from oracle import oracle as O
    return O.views_run(0, 5, ps.dots, ps.key_off(), ps.keys.reshape(-1), ps.fq_proc, ps.fq_time)


def numpy_union(n_cmd, cmd, dep):
    off, out = [0], []
    for c in range(n_cmd):
        s = sorted(set(int(x) for x in dep[cmd == c]))
        out.extend(s)
        off.append(len(out))
    return np.asarray(off, np.uint32), np.asarray(out, np.uint64)


def oracle_order(dots, dep_off, deps):
    from oracle import oracle as O
    n = len(dots)
    ex, lab, _, _ = O.graph_run(dots, np.zeros(n + 1, np.uint32), np.zeros(0, np.uint64),
                                dep_off, deps, 1)
    m = dict(zip(ex.tolist(), lab.tolist()))
    return ex[:n], np.asarray([m[int(d)] for d in dots], dtype=np.uint64)


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fantoch_amd.partial import PartialPipeline
    p = PartialPipeline(rank, world, keydeps=oracle_keydeps, union=numpy_union,
                        order=oracle_order)
    out = p.run(stream())
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_pseudo_stream_is_the_owned_key_slots():
    sys.path.insert(0, ROOT)
    from fantoch_amd.partial import pseudo_stream
    s = stream()
    for rank in range(WORLD):
        ps, p2c = pseudo_stream(s, rank, WORLD)
        owned = s.keys % WORLD == rank
        assert len(p2c) == int(owned.sum())
        assert np.all(np.diff(p2c) >= 0)
        assert np.array_equal(ps.keys.reshape(-1) * WORLD + rank, s.keys[owned])
        # every replica log lists a command's pseudo commands where (and as
        # often as) it lists the command
        for r in range(5):
            a, b = int(s.log_off[r]), int(s.log_off[r + 1])
            pa, pb = int(ps.log_off[r]), int(ps.log_off[r + 1])
            ent, pent = s.log_cmd[a:b].astype(np.int64), ps.log_cmd[pa:pb].astype(np.int64)
            want = [int(c) for c in ent for _ in range(int(owned[c].sum()))]
            assert p2c[pent].tolist() == want
            assert len(set(pent.tolist())) == len(pent)


def test_two_shards_pipeline_equals_unsharded_oracle():
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    s = stream()
    dep_off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc,
                                s.fq_time)
    ex, lab, kso, ks = O.graph_run(s.dots, s.key_off(), s.keys.reshape(-1), dep_off, deps,
                                   s.key_space)
    want_label = dict(zip(ex.tolist(), lab.tolist()))
    assert len(set(want_label.values())) < N_CMD // 2, "the stream has non-trivial SCCs"
    cross = sum(len(set(int(k) % WORLD for k in row)) > 1 for row in s.keys)
    assert cross > N_CMD // 2
    seen = set()
    for out in gathered:
        # every rank holds the whole committed graph
        assert np.array_equal(out["dep_off"], dep_off)
        assert np.array_equal(out["deps"], deps)
        assert dict(zip(s.dots.tolist(), out["scc_label"].tolist())) == want_label
        for key, seq in out["key_seq"].items():
            assert key not in seen
            seen.add(key)
            assert seq == ks[kso[key]:kso[key + 1]].tolist(), key
    assert seen == set(int(k) for k in np.unique(s.keys))
