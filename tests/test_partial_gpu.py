"""Partial replication on the GPU: the owner's union kernel (fh_dep_union,
csrc/union.hip) against numpy, and four key shards in one process -- each
with its own HipKeyDeps over its keys, records routed to the command's owner,
the owner's HIP union -- against one SequentialKeyDeps (oracle) over the
unsharded 4-keys-per-command stream (atlas.rs:580-583 semantics)."""
import numpy as np
import pytest

from fantoch_amd import _lib as L
from fantoch_amd.keydeps import HipKeyDeps
from fantoch_amd.partial import command_owner, hip_union, local_view
from fantoch_amd.workload import Workload
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def numpy_union(n_cmd, cmd, dep):
    pairs = np.unique(np.stack([cmd.astype(np.uint64), dep.astype(np.uint64)], 1), axis=0)
    off = np.zeros(n_cmd + 1, dtype=np.uint32)
    np.cumsum(np.bincount(pairs[:, 0].astype(np.int64), minlength=n_cmd), out=off[1:])
    return off, pairs[:, 1]


@pytest.mark.parametrize("n_cmd,nrec", [(1, 0), (7, 50), (100_000, 400_000)])
def test_dep_union_matches_numpy(n_cmd, nrec):
    rng = np.random.default_rng(n_cmd + nrec)
    cmd = rng.integers(0, n_cmd, nrec).astype(np.uint32)
    dep = rng.integers(1, 40, nrec).astype(np.uint64) << np.uint64(56) | rng.integers(
        1, 8, nrec).astype(np.uint64)  # few distinct dots: many duplicates
    off, out = hip_union(0)(n_cmd, cmd, dep)
    want_off, want = numpy_union(n_cmd, cmd, dep)
    assert np.array_equal(off, want_off)
    assert np.array_equal(out, want)


def test_dep_union_rejects_out_of_range_command():
    with pytest.raises(L.FhError):
        hip_union(0)(4, np.array([1, 4], np.uint32), np.array([5, 6], np.uint64))


def test_four_shards_compose_to_unsharded_keydeps():
    world, batch, nb = 4, 20_000, 3
    w = Workload.zipf(0.99, 4096, k=4, seed=41, n=5)
    s = w.generate(batch * nb)
    shards = [HipKeyDeps(shard_id=r, key_space=(w.key_count + world - 1) // world, device=0,
                         intern=False) for r in range(world)]
    union = hip_union(0)
    got = {}
    for b in range(nb):
        lo, hi = b * batch, (b + 1) * batch
        dots, keys = s.dots[lo:hi], s.keys[lo:hi]
        owner = command_owner(keys, world)
        rec_cmd, rec_dep = [], []
        for r in range(world):
            cmds, key_off, key_ids = local_view(keys, r, world)
            off, deps = shards[r].add_batch(dots[cmds], (key_off, key_ids))
            rec_cmd.append(np.repeat(cmds, np.diff(off.astype(np.int64))))
            rec_dep.append(deps)
        rec_cmd, rec_dep = np.concatenate(rec_cmd), np.concatenate(rec_dep)
        for r in range(world):  # the all-to-all, in one process
            mine = owner[rec_cmd] == r
            owned = np.nonzero(owner == r)[0]
            off, deps = union(len(owned), np.searchsorted(owned, rec_cmd[mine]), rec_dep[mine])
            for j, c in enumerate(owned):
                got[int(c) + lo] = deps[off[j]:off[j + 1]]
    dep_off, deps = O.keydeps_run(s.dots, s.key_off(), s.keys.reshape(-1))
    cross = 0
    for i in range(batch * nb):
        assert np.array_equal(got[i], deps[dep_off[i]:dep_off[i + 1]]), i
        cross += len(set(int(k) % world for k in s.keys[i])) > 1
    assert cross > batch


def test_four_shards_device_resident_stages():
    """The device-resident stages (fh_keydeps_add_batch_device, the record
    routing, fh_dep_union on device pointers) over four shards in one
    process, the all-to-all done by slicing: same dep sets as the unsharded
    oracle SequentialKeyDeps."""
    import torch

    from fantoch_amd.partial import device_local_deps, device_route, device_union

    world, batch, nb = 4, 20_000, 3
    w = Workload.zipf(0.99, 4096, k=4, seed=43, n=5)
    s = w.generate(batch * nb)
    shards = [HipKeyDeps(shard_id=r, key_space=(w.key_count + world - 1) // world, device=0,
                         intern=False) for r in range(world)]
    dev = torch.device("cuda", 0)
    got = {}
    for b in range(nb):
        lo, hi = b * batch, (b + 1) * batch
        dots = torch.from_numpy(s.dots[lo:hi].view(np.int64)).to(dev)
        keys = torch.from_numpy(s.keys[lo:hi].astype(np.int64)).to(dev)
        parts = [device_local_deps(shards[r], dots, keys, r, world) for r in range(world)]
        rec_cmd = torch.cat([p[0] for p in parts])
        rec_dep = torch.cat([p[1] for p in parts])
        rec_cmd, rec_dep, counts, owner = device_route(keys, rec_cmd, rec_dep, world)
        starts = [0] + torch.cumsum(counts, 0).tolist()
        for r in range(world):
            c, d = rec_cmd[starts[r]:starts[r + 1]], rec_dep[starts[r]:starts[r + 1]]
            owned = torch.nonzero(owner == r, as_tuple=True)[0]
            off, deps = device_union(len(owned), torch.searchsorted(owned, c), d)
            off, deps = off.cpu().numpy(), deps.cpu().numpy().view(np.uint64)
            for j, cmd in enumerate(owned.cpu().tolist()):
                got[cmd + lo] = deps[off[j]:off[j + 1]]
    dep_off, deps = O.keydeps_run(s.dots, s.key_off(), s.keys.reshape(-1))
    for i in range(batch * nb):
        assert np.array_equal(got[i], deps[dep_off[i]:dep_off[i + 1]]), i


def test_step_device_over_rccl_world_one():
    """PartialShard.step_device through a real RCCL group (world size 1 on
    the one-GPU box): the all-to-all is the identity, the result the full
    KeyDeps."""
    import os
    import socket

    import torch
    import torch.distributed as dist

    from fantoch_amd.partial import PartialShard

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        w = Workload.zipf(0.99, 4096, k=4, seed=44, n=5)
        s = w.generate(30_000)
        torch.cuda.set_device(0)
        sh = PartialShard(0, 1, w.key_count, device=0)
        dev = torch.device("cuda", 0)
        owned, off, deps = sh.step_device(torch.from_numpy(s.dots.view(np.int64)).to(dev),
                                          torch.from_numpy(s.keys.astype(np.int64)).to(dev))
        assert owned.cpu().tolist() == list(range(s.n))
        off, deps = off.cpu().numpy(), deps.cpu().numpy().view(np.uint64)
        dep_off, want = O.keydeps_run(s.dots, s.key_off(), s.keys.reshape(-1))
        assert np.array_equal(off.astype(np.int64), dep_off.astype(np.int64))
        assert np.array_equal(deps, want)
    finally:
        dist.destroy_process_group()
