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
