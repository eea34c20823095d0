"""Partial replication across GPUs: key shards with a cross-shard dependency
exchange.

fantoch's partial replication gives every shard its own KeyDeps over the
command's keys on that shard (Command::keys(shard), fantoch/src/command.rs:
95-100; SequentialKeyDeps::do_add_cmd, deps/keys/sequential.rs:72-104), and
commits a multi-shard command with the union of every shard's deps (Atlas
MShardCommit, fantoch_ps/src/protocol/atlas.rs:559-639, union :580-583).
One process per GPU is one shard here:

  1. local KeyDeps -- the shard's commands (those with a key it owns, in
     stream order) through HipKeyDeps over the owned keys only;
  2. exchange      -- (command, dep) records to the command's owner shard,
     one all-to-all (RCCL over xGMI on GPUs, gloo on CPU);
  3. union         -- the owner merges the reports into ascending unique
     dep sets (fh_dep_union, csrc/union.hip).

owner(key) = key mod world, local key id = key // world; a command's owner is
the shard of its first key (the client's target shard, fantoch/src/client/
workload.rs:172-176).  With a single view every dependency is an earlier
arrival, so the union is the complete committed dep set and each shard's
per-key sequences are its keys' commands in stream order.

The stages are injectable (`keydeps`, `union`) so the world-size-2 CPU test
can run the exchange with the oracle standing in for the GPU stages; the
defaults are the HIP ones and fail loudly without the library.

This is the single-view KeyDeps drop-in for partial replication (SURVEY §8
a8).  The C5 pipeline with replica views, SCCs and per-key order across GPUs
is fantoch_amd.dgraph (csrc/dgraph.hip).
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional

import numpy as np

from . import _lib as L


def command_owner(keys: np.ndarray, world: int) -> np.ndarray:
    """Owner shard of every command: the shard of its first key."""
    return (keys[:, 0] % np.uint64(world)).astype(np.int64)


def local_view(keys: np.ndarray, rank: int, world: int):
    """The shard's part of a batch: (command indices with an owned key,
    key_off CSR over them, local key ids in the command's key order)."""
    mine = keys % np.uint64(world) == np.uint64(rank)
    cnt = mine.sum(axis=1)
    cmds = np.nonzero(cnt)[0]
    key_off = np.zeros(len(cmds) + 1, dtype=np.uint32)
    np.cumsum(cnt[cmds], out=key_off[1:])
    key_ids = (keys[cmds][mine[cmds]] // np.uint64(world)).astype(np.uint64)
    return cmds, key_off, key_ids


def hip_union(device: int = -1):
    """records (owner-local command index, dep) -> (dep_off, deps) through
    fh_dep_union on the GPU."""
    import torch

    lib = L.load()

    def run(n_cmd: int, cmd: np.ndarray, dep: np.ndarray):
        dev = torch.device("cuda", device if device >= 0 else torch.cuda.current_device())
        if len(cmd) and int(cmd.max()) >= n_cmd:
            raise L.FhError(L.FH_EINVAL, "dep_union: record names a command out of range")
        c = torch.from_numpy(np.ascontiguousarray(cmd, dtype=np.uint32).view(np.int32)).to(dev)
        d = torch.from_numpy(np.ascontiguousarray(dep, dtype=np.uint64).view(np.int64)).to(dev)
        off = torch.empty(n_cmd + 1, dtype=torch.int32, device=dev)
        out = torch.empty(max(1, len(cmd)), dtype=torch.int64, device=dev)
        ln = C.c_size_t(0)
        stream = torch.cuda.current_stream(dev).cuda_stream
        L.check(lib.fh_dep_union(dev.index, n_cmd, len(cmd), C.c_void_p(c.data_ptr()),
                                 C.c_void_p(d.data_ptr()), C.c_void_p(off.data_ptr()),
                                 C.c_void_p(out.data_ptr()), C.byref(ln), C.c_void_p(stream)))
        return (off.cpu().numpy().view(np.uint32),
                out[:ln.value].cpu().numpy().view(np.uint64))

    return run


# ------------------------------------------------------ device-resident path
# The same three stages with every array in HBM (torch tensors on the rank's
# GPU): local_view with torch ops, fh_keydeps_add_batch_device, the record
# build, all_to_all_single over RCCL and fh_dep_union on device pointers.
# Nothing crosses PCIe but the few scalars the stages size their outputs with.

def _ptr(t):
    return C.c_void_p(t.data_ptr())


def device_local_deps(kd, dots, keys, rank: int, world: int):
    """The shard's KeyDeps over its owned keys of a batch (dots[n] int64,
    keys[n, k] int64 on the GPU) -> (record command index, record dep) on the
    GPU: one record per dependency its KeyDeps reports for an owned-key
    command (fh_keydeps_add_batch_device)."""
    import torch

    lib = L.load()
    mine = keys % world == rank
    cnt = mine.sum(dim=1)
    cmds = torch.nonzero(cnt, as_tuple=True)[0]
    key_off = torch.zeros(len(cmds) + 1, dtype=torch.int32, device=keys.device)
    key_off[1:] = torch.cumsum(cnt[cmds], 0)
    key_ids = torch.div(keys[cmds][mine[cmds]], world, rounding_mode="floor").contiguous()
    sel_dots = dots[cmds].contiguous()
    n, nkeys = len(cmds), len(key_ids)
    out_off = torch.empty(n + 1, dtype=torch.int32, device=keys.device)
    out_dep = torch.empty(max(1, n + nkeys), dtype=torch.int64, device=keys.device)
    ln = C.c_size_t(0)
    stream = torch.cuda.current_stream(keys.device).cuda_stream
    L.check(lib.fh_keydeps_add_batch_device(
        kd._h, n, nkeys, _ptr(sel_dots), _ptr(key_off), _ptr(key_ids) if nkeys else None,
        _ptr(out_off), _ptr(out_dep), len(out_dep), C.byref(ln), C.c_void_p(stream)))
    per = (out_off[1:] - out_off[:-1]).to(torch.int64)
    rec_cmd = torch.repeat_interleave(cmds, per)
    return rec_cmd, out_dep[:ln.value]


def device_union(n_cmd: int, cmd, dep):
    """records (owner-local command index int64, dep int64) on the GPU ->
    (dep_off int32[n_cmd+1], deps int64) through fh_dep_union."""
    import torch

    lib = L.load()
    dev = dep.device
    c32 = cmd.to(torch.int32).contiguous()
    d64 = dep.contiguous()
    off = torch.empty(n_cmd + 1, dtype=torch.int32, device=dev)
    out = torch.empty(max(1, len(d64)), dtype=torch.int64, device=dev)
    ln = C.c_size_t(0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    L.check(lib.fh_dep_union(dev.index, n_cmd, len(d64), _ptr(c32), _ptr(d64), _ptr(off),
                             _ptr(out), C.byref(ln), C.c_void_p(stream)))
    return off, out[:ln.value]


def device_route(keys, rec_cmd, rec_dep, world: int):
    """Records sorted by destination (the owner of their command) and the
    per-destination counts, for all_to_all_single."""
    import torch

    owner = keys[:, 0] % world
    dest = owner[rec_cmd]
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=world)
    return rec_cmd[order], rec_dep[order], counts, owner


def exchange_records(group, world: int, dest: np.ndarray, cmd: np.ndarray, dep: np.ndarray):
    """All-to-all of (command, dep) records by destination shard (RCCL on
    GPUs, gloo on CPU): counts first, then the records."""
    import torch
    import torch.distributed as dist

    order = np.argsort(dest, kind="stable")
    cmd, dep = cmd[order], dep[order]
    send = np.bincount(dest, minlength=world).astype(np.int64)
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    sc = torch.from_numpy(send).to(dev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv = rc.cpu().numpy()
    payload = torch.from_numpy(np.stack([cmd.astype(np.int64),
                                         dep.astype(np.uint64).view(np.int64)], 1)).to(dev)
    out = torch.empty((int(recv.sum()), 2), dtype=torch.int64, device=dev)
    dist.all_to_all_single(out, payload, output_split_sizes=recv.tolist(),
                           input_split_sizes=send.tolist(), group=group)
    out = out.cpu().numpy()
    return out[:, 0], out[:, 1].view(np.uint64)


class PartialShard:
    """One shard (one process, one GPU) of the partial-replication engine.

    keydeps(dots, key_off, key_ids) -> (dep_off, deps): the shard's KeyDeps
    over its owned keys, persistent across batches (default: HipKeyDeps).
    union(n_cmd, cmd, dep) -> (dep_off, deps) (default: fh_dep_union)."""

    def __init__(self, rank: int, world: int, key_space: int, device: int = -1,
                 group=None, keydeps: Optional[Callable] = None,
                 union: Optional[Callable] = None):
        self.rank, self.world, self.group = rank, world, group
        if keydeps is None:
            from .keydeps import HipKeyDeps
            kd = HipKeyDeps(shard_id=rank, key_space=(key_space + world - 1) // world,
                            device=device, intern=False)
            keydeps = lambda dots, off, ids: kd.add_batch(dots, (off, ids))  # noqa: E731
            self._kd = kd
        self.keydeps = keydeps
        self.union = union if union is not None else hip_union(device)
        self.device = device

    def _exchange(self, dest: np.ndarray, cmd: np.ndarray, dep: np.ndarray):
        return exchange_records(self.group, self.world, dest, cmd, dep)

    def step_device(self, dots, keys):
        """step() with the batch and every stage in HBM (dots[n], keys[n, k]:
        int64 tensors on this rank's GPU): the HIP KeyDeps, the records, one
        RCCL all-to-all (counts, then the records), the HIP union.  Returns
        (owned command indices, dep_off, deps) as GPU tensors."""
        import torch
        import torch.distributed as dist

        rec_cmd, rec_dep = device_local_deps(self._kd, dots, keys, self.rank, self.world)
        rec_cmd, rec_dep, send, owner = device_route(keys, rec_cmd, rec_dep, self.world)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        sc, rc = send.tolist(), recv.tolist()
        payload = torch.stack([rec_cmd, rec_dep], 1)
        got = torch.empty((sum(rc), 2), dtype=torch.int64, device=keys.device)
        dist.all_to_all_single(got, payload, output_split_sizes=rc, input_split_sizes=sc,
                               group=self.group)
        owned = torch.nonzero(owner == self.rank, as_tuple=True)[0]
        pos = torch.searchsorted(owned, got[:, 0].contiguous())
        dep_off, deps = device_union(len(owned), pos, got[:, 1])
        return owned, dep_off, deps

    def step(self, dots: np.ndarray, keys: np.ndarray):
        """One batch of the global stream (dots[n], keys[n, k]).  Returns the
        owned commands' batch indices (ascending) and their committed deps as
        (dep_off, deps)."""
        cmds, key_off, key_ids = local_view(keys, self.rank, self.world)
        off, deps = self.keydeps(dots[cmds], key_off, key_ids)
        off = np.asarray(off, dtype=np.int64)
        per = np.diff(off)
        rec_cmd = np.repeat(cmds, per)
        owner = command_owner(keys, self.world)
        # records only for deps; an owned command without any still gets its
        # (empty) row in the owner's union
        g_cmd, g_dep = self._exchange(owner[rec_cmd], rec_cmd, np.asarray(deps, np.uint64))
        owned = np.nonzero(owner == self.rank)[0]
        pos = np.searchsorted(owned, g_cmd)
        dep_off, dep_set = self.union(len(owned), pos, g_dep)
        return owned, dep_off, dep_set
