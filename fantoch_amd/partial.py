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


# ------------------------------------------------- full pipeline over ranks
# Partial replication with replica views (config C5 across GPUs): every rank
# is a key shard and produces the per-key execution sequences of its keys.
#
#   1. KeyDeps      -- the shard's replicas run SequentialKeyDeps over the
#      command's owned keys only (Command::keys(shard), command.rs:95-100),
#      in their arrival order.  Each owned (command, key) pair is staged as a
#      single-key pseudo command (unique pseudo dot, the real command's
#      arrivals), so the fused engine runs unchanged in deps-only mode: the
#      deps of a key do not depend on the command's other keys, and the
#      union over a command's pairs, views and shards is the command's
#      committed dep set (plain union, quorum.rs:28-98 / atlas.rs:580-583).
#   2. exchange     -- (command, dep) records to the command's owner (the
#      shard of its first key): one all-to-all.
#   3. union        -- the owner merges them (fh_dep_union).
#   4. graph        -- the committed dep rows are all-gathered, and every
#      rank orders the whole graph (SCCs, execution order).  With cross-shard
#      commands on every key, a shard's closure is nearly the whole stream
#      (C5: a 1.19M-member SCC spanning all shards), so the graph exchange is
#      the whole edge set; the reference reaches the same vertices one request
#      at a time (executor/graph/mod.rs:279-408).
#   5. per-key      -- each rank cuts the sequences of its own keys out of the
#      execution order.

PSEUDO_SOURCE = 1


def pseudo_stream(s, rank: int, world: int):
    """The shard's KeyDeps input (stage 1) from a Stream with replica logs:
    (pseudo Stream of k = 1 commands over local key ids, pseudo -> command
    index).  Pseudo p has dot (PSEUDO_SOURCE, p + 1); replica r's log lists a
    command's pseudo commands where it lists the command."""
    from .workload import Stream

    if s.log_cmd is None or s.log_off is None:
        raise ValueError("pseudo_stream: the stream needs its replica logs (generate(logs=True))")
    fq = s.views
    mine = s.keys % np.uint64(world) == np.uint64(rank)
    c, t = np.nonzero(mine)  # command order, then key slot order
    p2c = c.astype(np.int64)
    npair = len(p2c)
    pkeys = (s.keys[c, t] // np.uint64(world)).astype(np.uint64).reshape(-1, 1)
    pdots = (np.uint64(PSEUDO_SOURCE) << np.uint64(56)) | np.arange(1, npair + 1, dtype=np.uint64)
    cnt = np.bincount(p2c, minlength=s.n).astype(np.int64)
    first = np.zeros(s.n + 1, dtype=np.int64)
    np.cumsum(cnt, out=first[1:])
    cmd = s.log_cmd.astype(np.int64)  # replica logs list command indices
    reps = cnt[cmd]
    ends = np.cumsum(reps)
    within = np.arange(int(ends[-1]) if len(ends) else 0, dtype=np.int64) - np.repeat(ends - reps, reps)
    plog = (first[np.repeat(cmd, reps)] + within).astype(np.uint32)
    cum = np.concatenate([[0], ends]).astype(np.uint64)
    plo = cum[s.log_off.astype(np.int64)]
    key_space = (s.key_space + world - 1) // world
    fq_proc = None if s.fq_proc is None else s.fq_proc[p2c]
    fq_time = None if s.fq_time is None else s.fq_time[p2c]
    ps = Stream(pdots, pkeys, fq_proc, fq_time, key_space, log_off=plo, log_cmd=plog,
                views_n=fq)
    return ps, p2c


def pseudo_records(p2c, dots, dep_off, deps):
    """Stage-1 output in pseudo dots -> (command index, real dep dot) records."""
    dep_off = np.asarray(dep_off, dtype=np.int64)
    per = np.diff(dep_off)
    rec_cmd = np.repeat(p2c, per)
    p = (np.asarray(deps, dtype=np.uint64) & np.uint64((1 << 56) - 1)).astype(np.int64) - 1
    return rec_cmd, dots[p2c[p]]


def hip_views_keydeps(device: int = -1, nproc: int = 5):
    """Stage 1 on the GPU: the fused engine in deps-only mode over a pseudo
    stream -> (dep_off, deps) in pseudo dots."""
    from .engine import Engine

    def run(ps):
        eng = Engine(ps.key_space, n=nproc, device=device)
        try:
            eng.set_deps_only(True)
            eng.stage_logs([ps], nproc=nproc)
            eng.run()
            return eng.deps()
        finally:
            eng.close()

    return run


def hip_order(device: int = -1):
    """Stage 4 on the GPU: the graph executor (fh_graph) over a whole
    committed graph -> (execution-ordered dots, SCC label per command)."""
    from .keydeps import make_config

    lib = L.load()

    def run(dots, dep_off, deps):
        n = len(dots)
        cfg = make_config(n=1, f=0, device=device, key_space=1)
        h = C.c_void_p()
        L.check(lib.fh_graph_create(1, 0, C.byref(cfg), C.byref(h)))
        try:
            d = np.ascontiguousarray(dots, dtype=np.uint64)
            ko = np.zeros(n + 1, dtype=np.uint32)
            do = np.ascontiguousarray(dep_off, dtype=np.uint32)
            dp = np.ascontiguousarray(deps, dtype=np.uint64)
            L.check(lib.fh_graph_add_batch(h, n, L.ptr(d), L.ptr(ko), None, L.ptr(do),
                                           L.ptr(dp) if len(dp) else None))
            ex = np.zeros(max(1, n), dtype=np.uint64)
            lab = np.zeros(max(1, n), dtype=np.uint64)
            ln = C.c_size_t(0)
            L.check(lib.fh_graph_drain(h, L.ptr(ex), L.ptr(lab), len(ex), C.byref(ln)))
            if ln.value != n:
                raise L.FhError(L.FH_EINVARIANT, f"graph left {n - ln.value} commands pending")
        finally:
            lib.fh_graph_destroy(h)
        pos = np.searchsorted(dots, ex[:n], sorter=np.argsort(dots, kind="stable"))
        order = np.argsort(dots, kind="stable")[pos]
        label = np.zeros(n, dtype=np.uint64)
        label[order] = lab[:n]
        return ex[:n], label

    return run


def _allgather_rows(group, owned, dep_off, deps, n: int):
    """Every rank's owned rows -> the whole committed CSR (command order)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    cnt = np.diff(np.asarray(dep_off, dtype=np.int64))
    mine = np.stack([np.asarray(owned, np.int64), cnt], 1) if len(owned) else np.zeros((0, 2), np.int64)
    payload = [mine.reshape(-1), np.asarray(deps, dtype=np.uint64).view(np.int64)]
    out = []
    for arr in payload:
        sz = torch.tensor([len(arr)], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(sz) for _ in range(world)]
        dist.all_gather(sizes, sz, group=group)
        sizes = [int(x.item()) for x in sizes]
        mx = max(1, max(sizes))
        buf = torch.zeros(mx, dtype=torch.int64, device=dev)
        buf[:len(arr)] = torch.from_numpy(arr).to(dev)
        bufs = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(bufs, buf, group=group)
        out.append([b[:sz_].cpu().numpy() for b, sz_ in zip(bufs, sizes)])
    rows = np.concatenate([r.reshape(-1, 2) for r in out[0]])
    dep_all = np.concatenate(out[1]).view(np.uint64)
    counts = np.zeros(n, dtype=np.int64)
    counts[rows[:, 0]] = rows[:, 1]
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=off[1:])
    # the gathered deps are row blocks in (rank, owned command) order
    starts = np.repeat(off[rows[:, 0]], rows[:, 1])
    within = np.arange(len(dep_all)) - np.repeat(np.cumsum(rows[:, 1]) - rows[:, 1], rows[:, 1])
    full = np.zeros(len(dep_all), dtype=np.uint64)
    full[starts + within] = dep_all
    return off.astype(np.uint32), full


class PartialPipeline:
    """One rank (one GPU) of the partial-replication pipeline above.

    Stages are injectable so the world-size-2 CPU test runs the exchange
    logic with the oracle in place of the GPU stages:
      keydeps(pseudo_stream) -> (dep_off, deps in pseudo dots)
      union(n_cmd, cmd, dep) -> (dep_off, deps)
      order(dots, dep_off, deps) -> (execution-ordered dots, label per command)
    The defaults are the HIP stages and fail loudly without the library."""

    def __init__(self, rank: int, world: int, group=None, device: int = -1,
                 keydeps: Optional[Callable] = None, union: Optional[Callable] = None,
                 order: Optional[Callable] = None, nproc: int = 5):
        self.rank, self.world, self.group = rank, world, group
        self.keydeps = keydeps if keydeps is not None else hip_views_keydeps(device, nproc)
        self.union = union if union is not None else hip_union(device)
        self.order = order if order is not None else hip_order(device)

    def run(self, s):
        """One stream with replica logs (every rank holds the same stream).
        Returns a dict: committed deps of the whole stream (dep_off, deps),
        the SCC label of every command, and this shard's per-key sequences
        {global key: [dots in execution order]}."""
        ps, p2c = pseudo_stream(s, self.rank, self.world)
        pofs, pdeps = self.keydeps(ps)
        rec_cmd, rec_dep = pseudo_records(p2c, s.dots, pofs, pdeps)
        owner = command_owner(s.keys, self.world)
        g_cmd, g_dep = exchange_records(self.group, self.world, owner[rec_cmd], rec_cmd, rec_dep)
        owned = np.nonzero(owner == self.rank)[0]
        pos = np.searchsorted(owned, g_cmd)
        odo, odeps = self.union(len(owned), pos, g_dep)
        dep_off, deps = _allgather_rows(self.group, owned, odo, odeps, s.n)
        ex, label = self.order(s.dots, dep_off, deps)
        # this shard's per-key sequences, cut out of the execution order
        rank_of = np.empty(s.n, dtype=np.int64)
        srt = np.argsort(s.dots, kind="stable")
        rank_of[srt[np.searchsorted(s.dots, ex, sorter=srt)]] = np.arange(s.n)
        mine = s.keys % np.uint64(self.world) == np.uint64(self.rank)
        c, t = np.nonzero(mine)
        key = s.keys[c, t]
        o = np.lexsort((rank_of[c], key))
        seq = {}
        for kk, dd in zip(key[o].tolist(), s.dots[c[o]].tolist()):
            seq.setdefault(kk, []).append(dd)
        return {"dep_off": dep_off, "deps": deps, "scc_label": label, "key_seq": seq}
