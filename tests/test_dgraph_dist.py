"""Partial replication across ranks (fantoch_amd.dgraph, the fh_dgraph_*
steps) on CPU: world-size-2 (and 3) gloo processes run DistPartial's
orchestration and exchanges -- code all-to-all, query / answer all-to-alls,
the condensed graph's all-gather, the per-key elements' all-to-all -- with
the CPU mirror of the HIP stages (tests/dgraph_cpu.py; no GPU here,
tests/test_dgraph_gpu.py runs the HIP ones).  The assembled outputs must
equal the single-process oracle on the same partially replicated stream:
committed deps of every command (every shard's collect, unioned,
atlas.rs:559-639), the SCC partition and every key's execution sequence."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def make_stream(n, seed, keys=4096, k=4, shards=8):
    from fantoch_amd.workload import Workload
    w = Workload.zipf(0.99, keys, k=k, views=3, window=64, seed=seed, n=5, shards=shards)
    return w.generate(n, logs=True)


def _worker(rank, world, port, n, seed, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dgraph_cpu import CpuStages
    from fantoch_amd.dgraph import DistPartial
    s = make_stream(n, seed)
    p = DistPartial(rank, world, s.key_space, backend=CpuStages(rank, world, s.key_space))
    p.stage(s)
    p.run()
    out = p.results()
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,seed", [(2, 3000, 61), (3, 2500, 62)])
def test_dgraph_ranks_match_oracle(world, n, seed):
    sys.path.insert(0, HERE)
    from fantoch_amd.dgraph import assemble
    from fullsize import shard_union
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = make_stream(n, seed)
    esc = sum(p["escaping"] for p in parts)
    assert 0 < esc < s.n and all(p["cross_edges"] for p in parts), "both vertex classes occur"
    got = assemble(parts, s.n, s.key_space)
    off, deps = shard_union(s)
    assert np.array_equal(got["dep_off"], off) and np.array_equal(got["deps"], deps), "deps"
    ex, lab, kso, ks = O.graph_run(s.dots, s.key_off(), s.keys.reshape(-1), off, deps, s.key_space)
    want = dict(zip(ex.tolist(), lab.tolist()))
    assert dict(zip(s.dots.tolist(), got["scc_label"].tolist())) == want, "SCC partition"
    assert np.array_equal(got["key_off"], kso), "per-key lengths"
    assert np.array_equal(got["key_seq"], ks), "per-key sequences"
