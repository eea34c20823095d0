"""The C4 multi-GPU path on CPU: world_size-2 gloo processes each order their
key shard of a replica-view stream with global dots (owner = the balanced key
map, fh_key_owners_balanced over the stream's key counts, computed by every
rank independently -- what bench.py --gpus N does with
fh_workload_generate_shard_owned), through the
oracle -- no GPU here -- and all-gather.  Rank 0 checks that the shards
compose to the unsharded stream's outputs: the same committed deps, SCC
labels and per-key sequences.  With one key per command every dependency
joins two commands of one key, so a shard's graph is closed and needs no
exchange."""
import os
import socket
import sys

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOTAL, KEYS, SEED = 24_000, 1 << 12, 0xFA170C4000000004


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle(s):
    from oracle import oracle as O
    ko = s.key_off()
    kk = s.keys.reshape(-1)
    off, deps = O.views_run(0, 5, s.dots, ko, kk, s.fq_proc, s.fq_time)
    ex, lab, kso, ks = O.graph_run(s.dots, ko, kk, off, deps, s.key_space)
    return off, deps, dict(zip(ex.tolist(), lab.tolist())), kso, ks


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fantoch_amd.workload import Stream, Workload, key_owners_balanced
    w = Workload.zipf(0.99, KEYS, k=1, views=3, window=64, seed=SEED, n=5)
    full = w.generate(TOTAL)
    owner = key_owners_balanced(w.key_histogram(TOTAL), world)
    mine = np.nonzero(owner[full.keys[:, 0]] == rank)[0]
    s = Stream(full.dots[mine], full.keys[mine], full.fq_proc[mine], full.fq_time[mine],
               full.key_space)
    # the shard generator (what bench.py stages) holds exactly these commands
    g = w.generate_shard(TOTAL, world, rank, owner=owner)
    assert np.array_equal(g.dots, s.dots) and np.array_equal(g.keys, s.keys)
    # balanced: each rank within 5% of the mean (key mod 2 is not, on Zipf)
    sizes = [None] * world
    dist.all_gather_object(sizes, int(s.n))
    assert max(sizes) <= 1.05 * TOTAL / world, sizes
    off, deps, lab, kso, ks = _oracle(s)
    deps_of = {int(s.dots[i]): deps[off[i]:off[i + 1]].tolist() for i in range(s.n)}
    seqs = {int(k): ks[kso[k]:kso[k + 1]].tolist() for k in np.nonzero(np.diff(kso))[0]}
    gathered = [None] * world
    dist.all_gather_object(gathered, (deps_of, lab, seqs))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_view_shards_compose_to_unsharded_outputs():
    sys.path.insert(0, ROOT)
    from fantoch_amd.workload import Workload
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    deps_m, lab_m, seq_m = {}, {}, {}
    for deps_of, lab, seqs in gathered:
        assert not (set(deps_m) & set(deps_of)), "a command lives on exactly one shard"
        assert not (set(seq_m) & set(seqs)), "a key lives on exactly one shard"
        deps_m.update(deps_of)
        lab_m.update(lab)
        seq_m.update(seqs)
    w = Workload.zipf(0.99, KEYS, k=1, views=3, window=64, seed=SEED, n=5)
    s = w.generate(TOTAL)
    off, deps, lab, kso, ks = _oracle(s)
    assert len(deps_m) == s.n
    for i in range(s.n):
        assert deps_m[int(s.dots[i])] == deps[off[i]:off[i + 1]].tolist()
    assert lab_m == lab
    assert seq_m == {int(k): ks[kso[k]:kso[k + 1]].tolist() for k in np.nonzero(np.diff(kso))[0]}
