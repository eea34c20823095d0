"""Partial replication on CPU (SURVEY.md §8e, C5 shape): world_size-2 gloo
processes, each a key shard, run fantoch_amd.partial.PartialShard over a
4-keys-per-command Zipf stream in three batches -- local KeyDeps over the
owned keys, the all-to-all of (command, dep) records, the owner's union --
with the oracle standing in for the GPU stages (no GPU here).  Rank 0 checks
that the union of the owners' committed deps equals one SequentialKeyDeps
over the unsharded stream (atlas.rs:580-583 semantics)."""
import os
import socket
import sys

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def oracle_keydeps(shard_id):
    """Stateful per-shard SequentialKeyDeps (oracle) in PartialShard's form."""
    from oracle import oracle as O
    kd = O.KeyDeps(shard_id)

    def run(dots, key_off, key_ids):
        off, out = [0], []
        for i, d in enumerate(dots):
            deps = sorted(kd.add_cmd(int(d), [int(k) for k in key_ids[key_off[i]:key_off[i + 1]]]))
            out.extend(deps)
            off.append(len(out))
        return np.asarray(off, np.uint32), np.asarray(out, np.uint64)
    return run


def numpy_union(n_cmd, cmd, dep):
    off, out = [0], []
    for c in range(n_cmd):
        s = sorted(set(int(x) for x in dep[cmd == c]))
        out.extend(s)
        off.append(len(out))
    return np.asarray(off, np.uint32), np.asarray(out, np.uint64)


def _worker(rank, world, port, batch, nb, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fantoch_amd.partial import PartialShard
    from fantoch_amd.workload import Workload
    w = Workload.zipf(0.99, 512, k=4, seed=31, n=5)
    s = w.generate(batch * nb)
    shard = PartialShard(rank, world, w.key_count, keydeps=oracle_keydeps(rank),
                         union=numpy_union)
    got = {}
    for b in range(nb):
        lo, hi = b * batch, (b + 1) * batch
        owned, off, deps = shard.step(s.dots[lo:hi], s.keys[lo:hi])
        for j, c in enumerate(owned):
            got[int(c) + lo] = [int(x) for x in deps[off[j]:off[j + 1]]]
    gathered = [None] * world
    dist.all_gather_object(gathered, got)
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_two_shards_union_equals_unsharded_keydeps():
    sys.path.insert(0, ROOT)
    from fantoch_amd.workload import Workload
    from oracle import oracle as O
    world, batch, nb = 2, 1500, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, nb, q))
             for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    merged = {}
    for g in gathered:
        assert not (set(merged) & set(g)), "a command has exactly one owner"
        merged.update(g)
    assert sorted(merged) == list(range(batch * nb))
    s = Workload.zipf(0.99, 512, k=4, seed=31, n=5).generate(batch * nb)
    dep_off, deps = O.keydeps_run(s.dots, s.key_off(), s.keys.reshape(-1))
    cross = 0
    for i in range(batch * nb):
        assert merged[i] == sorted(int(x) for x in deps[dep_off[i]:dep_off[i + 1]]), i
        cross += len(set(int(k) % world for k in s.keys[i])) > 1
    assert cross > batch  # the stream really has cross-shard commands
