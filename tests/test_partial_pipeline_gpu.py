"""Partial replication, whole pipeline with the HIP stages:
two ranks on the box's one GPU (gloo carries the exchange: RCCL refuses two
ranks on one device), each running fantoch_amd.partial.PartialPipeline with
its defaults -- the fused engine in deps-only mode over the shard's pseudo
commands, fh_dep_union, fh_graph over the all-gathered committed graph.
Checked against the oracle on the unsharded stream: committed deps, SCC
partition, every key's execution sequence."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_CMD, WORLD = 20_000, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def stream():
    from fantoch_amd.workload import Workload
    w = Workload.zipf(0.99, 4096, k=4, views=3, window=64, seed=78, n=5)
    return w.generate(N_CMD, logs=True, times=True)


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    torch.cuda.init()  # torch's HIP runtime first
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fantoch_amd.partial import PartialPipeline
        out = PartialPipeline(rank, world, device=0).run(stream())
        gathered = [None] * world
        dist.all_gather_object(gathered, out)
        if rank == 0:
            q.put(gathered)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_shards_hip_pipeline_equals_unsharded_oracle():
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        gathered = q.get(timeout=150)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    s = stream()
    dep_off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc,
                                s.fq_time)
    ex, lab, kso, ks = O.graph_run(s.dots, s.key_off(), s.keys.reshape(-1), dep_off, deps,
                                   s.key_space)
    want_label = dict(zip(ex.tolist(), lab.tolist()))
    assert len(set(want_label.values())) < N_CMD // 2
    seen = set()
    for out in gathered:
        assert np.array_equal(out["dep_off"], dep_off)
        assert np.array_equal(out["deps"], deps)
        assert dict(zip(s.dots.tolist(), out["scc_label"].tolist())) == want_label
        for key, seq in out["key_seq"].items():
            assert key not in seen
            seen.add(key)
            assert seq == ks[kso[key]:kso[key + 1]].tolist(), key
    assert seen == set(int(k) for k in np.unique(s.keys))


@pytest.mark.gpu
def test_deps_only_run_matches_full_run_deps():
    from fantoch_amd.engine import Engine
    from fantoch_amd._lib import FhError
    from fantoch_amd.workload import Workload
    s = Workload.zipf(0.99, 4096, k=4, views=3, window=64, seed=79, n=5).generate(
        30_000, logs=True, times=False)
    eng = Engine(s.key_space, device=0)
    eng.stage(s)
    eng.run()
    full = eng.results()
    eng.rewind()
    eng.set_deps_only(True)
    eng.run()
    off, deps = eng.deps()
    assert np.array_equal(off, full["dep_off"]) and np.array_equal(deps, full["deps"])
    with pytest.raises(FhError):
        eng.results()  # labels / per-key output are not materialised
    eng.close()


@pytest.mark.gpu
def test_pipeline_over_rccl_world_one():
    """PartialPipeline's collectives through a real RCCL group (world size 1 on
    the one-GPU box: the all-to-all and all-gather are identities over RCCL),
    HIP stages, against the oracle."""
    import socket

    import torch
    import torch.distributed as dist

    from fantoch_amd.partial import PartialPipeline
    from oracle import oracle as O

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        s = stream()
        out = PartialPipeline(0, 1, device=0).run(s)
        dep_off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc,
                                    s.fq_time)
        ex, lab, kso, ks = O.graph_run(s.dots, s.key_off(), s.keys.reshape(-1), dep_off, deps,
                                       s.key_space)
        assert np.array_equal(out["dep_off"], dep_off) and np.array_equal(out["deps"], deps)
        assert dict(zip(s.dots.tolist(), out["scc_label"].tolist())) == dict(
            zip(ex.tolist(), lab.tolist()))
        for key, seq in out["key_seq"].items():
            assert seq == ks[kso[key]:kso[key + 1]].tolist(), key
        assert len(out["key_seq"]) == len(np.unique(s.keys))
    finally:
        dist.destroy_process_group()
