"""The N>1 path on CPU: world_size-2 gloo processes each order their key shard
(through the oracle -- no GPU here), all-gather per-key sequences mapped back
to global command indices, and rank 0 checks the union equals the unsharded
stream's per-key order.  Also checks the partition is complete and disjoint."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_worker(rank, world, port, batch, nb, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fantoch_amd.shard import shard_batches
    from fantoch_amd.workload import Workload
    from oracle import oracle as O
    w = Workload.zipf(0.7, 4096, k=1, seed=99, n=5)
    batches, index = shard_batches(w, rank, world, batch, nb, return_index=True)
    dots = np.concatenate([b.dots for b in batches])
    keys = np.concatenate([b.keys for b in batches]).reshape(-1)
    gidx = np.concatenate(index)
    key_off = np.arange(len(dots) + 1, dtype=np.uint32)
    dep_off, deps = O.keydeps_run(dots, key_off, keys)
    ex, lab, kso, ks = O.graph_run(dots, key_off, keys, dep_off, deps, batches[0].key_space)
    pos = {int(d): int(g) for d, g in zip(dots, gidx)}
    local = {}
    for k in np.nonzero(np.diff(kso))[0]:
        gkey = int(k) * world + rank  # shard-local id -> global key
        local[gkey] = [pos[int(d)] for d in ks[kso[k]:kso[k + 1]]]
    gathered = [None] * world
    dist.all_gather_object(gathered, (local, gidx.tolist()))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_key_shards_compose_to_global_order():
    sys.path.insert(0, ROOT)
    from fantoch_amd.workload import Workload
    from oracle import oracle as O
    world, batch, nb = 2, 3000, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, batch, nb, q))
             for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    merged, all_idx = {}, []
    for local, idx in gathered:
        assert not (set(merged) & set(local)), "a key lives on exactly one shard"
        merged.update(local)
        all_idx.extend(idx)
    assert len(all_idx) == len(set(all_idx)) == world * batch * nb
    # the unsharded stream prefix covering every sharded command
    top = max(all_idx) + 1
    w = Workload.zipf(0.7, 4096, k=1, seed=99, n=5)
    s = w.generate(top)
    take = np.zeros(top, dtype=bool)
    take[all_idx] = True
    # order the commands the shards processed, on the whole stream
    dots, keys = s.dots[take], s.keys[take].reshape(-1)
    g_of = np.nonzero(take)[0]
    key_off = np.arange(len(dots) + 1, dtype=np.uint32)
    dep_off, deps = O.keydeps_run(dots, key_off, keys)
    ex, lab, kso, ks = O.graph_run(dots, key_off, keys, dep_off, deps, s.key_space)
    pos = {int(d): int(g) for d, g in zip(dots, g_of)}
    want = {int(k): [pos[int(d)] for d in ks[kso[k]:kso[k + 1]]]
            for k in np.nonzero(np.diff(kso))[0]}
    assert merged == want
