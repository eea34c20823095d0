"""Partial replication across GPUs (config C5 at N > 1): one process per GPU,
the fh_dgraph_* steps (csrc/dgraph.hip) with torch.distributed exchanges
between them -- RCCL over xGMI on the GPUs (device tensors throughout), or
gloo (host copies) when several ranks share one GPU in a test.

Per step (DistPartial.run):
  1. KeyDeps by key shard: this rank's processes (those of the shards h with
     h % N == rank) -> the dependency code of each of their elements.
  2. all-to-all of the codes to their command's range owner (4 B each);
     the owner unions each command's keys x views (QuorumDeps +
     MShardCommit, atlas.rs:559-639), cuts the cross-range edges and runs
     the local SCCs; vertices reaching a cross-range edge are contracted.
  3. all-to-all of cross-range queries and the owners' answers.
  4. all-gather of every rank's part of the condensed graph (vertices and
     edges in one exchange); every rank solves it (SCCs, ready times,
     depths of the escaping vertices).
  5. all-to-all of the (key, order) elements to the keys' owners, sorted
     there into the per-key execution sequences.
The reference reaches other shards' vertices one request / reply at a time
(executor/graph/mod.rs:279-408, index.rs:171-205); this is the batch
restatement, with the whole committed stream in HBM.

The stage object is injectable: `backend=HipStages(...)` (default, the HIP
library; fails loudly without it) or a CPU mirror with the same interface
(tests/dgraph_cpu.py) so the world-size-2 gloo test checks the exchanges and
the algorithm on the CPU.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _lib as L


def shard_logs(s, rank: int, world: int):
    """This rank's element logs out of a partially replicated stream's (every
    process's log): the processes of the shards h with h % world == rank, in
    shard order -> (log_off, log_elem)."""
    assert s.log_elem is not None and s.shards >= 1
    n = s.nproc
    offs, parts, base = [0], [], 0
    for h in range(s.shards):
        if h % world != rank:
            continue
        for p in range(n * h, n * h + n):
            a, b = int(s.log_off[p]), int(s.log_off[p + 1])
            parts.append(s.log_elem[a:b])
            base += b - a
            offs.append(base)
    log_off = np.asarray(offs, dtype=np.uint64)
    log_elem = np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint32)
    return log_off, np.ascontiguousarray(log_elem, dtype=np.uint32)


class HipStages:
    """The fh_dgraph_* steps on this rank's GPU (device tensors in and out)."""

    def __init__(self, rank: int, world: int, key_space: int, device: int, n: int = 5):
        import torch
        from .keydeps import make_config
        self.torch = torch
        self.lib = L.load()
        self.dev = torch.device("cuda", device)
        self.cfg = make_config(n=n, f=1, device=device, key_space=key_space)
        h = C.c_void_p()
        L.check(self.lib.fh_dgraph_create(C.byref(self.cfg), rank, world, C.byref(h)))
        self.h = h
        self.world = world

    def close(self):
        if getattr(self, "h", None):
            self.lib.fh_dgraph_destroy(self.h)
            self.h = None

    def _p(self, t):
        return C.c_void_p(t.data_ptr()) if t is not None and t.numel() else None

    def _empty(self, m, dtype):
        return self.torch.empty(max(1, int(m)), dtype=dtype, device=self.dev)

    def stage(self, s, log_off, log_elem):
        d = L.fh_stream_desc(n=s.n, keys_per_cmd=s.k, views=s.views, nproc=len(log_off) - 1,
                             flags=L.FH_STREAM_ELEMENT_LOGS)
        sc = np.zeros(self.world, dtype=np.uint64)
        rc = np.zeros(self.world, dtype=np.uint64)
        rng = np.zeros(2, dtype=np.uint64)
        dots = np.ascontiguousarray(s.dots, dtype=np.uint64)
        keys = np.ascontiguousarray(s.keys, dtype=np.uint64)
        L.check(self.lib.fh_dgraph_stage(self.h, C.byref(d), s.shards, L.ptr(dots), L.ptr(keys),
                                         L.ptr(log_off), L.ptr(log_elem), L.ptr(sc), L.ptr(rc),
                                         L.ptr(rng)))
        return sc.astype(np.int64), rc.astype(np.int64), (int(rng[0]), int(rng[1]))

    def keydeps(self, nsend):
        out = self._empty(nsend, self.torch.int32)
        L.check(self.lib.fh_dgraph_keydeps(self.h, self._p(out)))
        return out[:nsend]

    def local(self, recv):
        qc = np.zeros(self.world, dtype=np.uint64)
        self.torch.cuda.synchronize(self.dev)
        L.check(self.lib.fh_dgraph_local(self.h, self._p(recv), L.ptr(qc)))
        return qc.astype(np.int64)

    def queries(self, nq):
        out = self._empty(nq, self.torch.int32)
        L.check(self.lib.fh_dgraph_queries(self.h, self._p(out)))
        return out[:nq]

    def answer(self, q):
        out = self._empty(len(q), self.torch.int32)
        self.torch.cuda.synchronize(self.dev)
        L.check(self.lib.fh_dgraph_answer(self.h, len(q), self._p(q), self._p(out)))
        return out[:len(q)]

    def condense(self, answers):
        nv, ne = C.c_uint64(0), C.c_uint64(0)
        self.torch.cuda.synchronize(self.dev)
        L.check(self.lib.fh_dgraph_condense(self.h, self._p(answers), C.byref(nv), C.byref(ne)))
        v = self._empty(2 * nv.value, self.torch.int64)
        e = self._empty(ne.value, self.torch.int64)
        L.check(self.lib.fh_dgraph_condensed_part(self.h, self._p(v), self._p(e)))
        return v[:2 * nv.value], e[:ne.value]

    def solve(self, verts, edges):
        ec = np.zeros(self.world, dtype=np.uint64)
        self.torch.cuda.synchronize(self.dev)
        L.check(self.lib.fh_dgraph_solve(self.h, len(verts) // 2, self._p(verts), len(edges),
                                         self._p(edges), L.ptr(ec)))
        ec = ec.astype(np.int64)
        el = self._empty(2 * int(ec.sum()), self.torch.int64)
        L.check(self.lib.fh_dgraph_elements(self.h, self._p(el)))
        return ec, el[:2 * int(ec.sum())]

    def per_key(self, elems):
        self.torch.cuda.synchronize(self.dev)
        L.check(self.lib.fh_dgraph_per_key(self.h, len(elems) // 2, self._p(elems)))

    def results(self, count):
        dep_off = np.zeros(count + 1, dtype=np.uint32)
        ln, pk = C.c_size_t(0), C.c_size_t(0)
        L.check(self.lib.fh_dgraph_results(self.h, L.ptr(dep_off), None, 0, C.byref(ln), None,
                                           None, None, C.byref(pk)))
        deps = np.zeros(max(1, ln.value), dtype=np.uint64)
        label = np.zeros(max(1, count), dtype=np.uint64)
        pk_key = np.zeros(max(1, pk.value), dtype=np.uint32)
        pk_dot = np.zeros(max(1, pk.value), dtype=np.uint64)
        L.check(self.lib.fh_dgraph_results(self.h, L.ptr(dep_off), L.ptr(deps), len(deps),
                                           C.byref(ln), L.ptr(label), L.ptr(pk_key),
                                           L.ptr(pk_dot), C.byref(pk)))
        return {"dep_off": dep_off, "deps": deps[:ln.value], "scc_label": label[:count],
                "pk_key": pk_key[:pk.value], "pk_dot": pk_dot[:pk.value]}

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def set_profiling(self, on):
        L.check(self.lib.fh_dgraph_set_profiling(self.h, 1 if on else 0))

    def stage_times(self):
        n = C.c_size_t(0)
        L.check(self.lib.fh_dgraph_stage_times(self.h, None, None, 0, C.byref(n)))
        names = (C.c_char_p * max(1, n.value))()
        ms = (C.c_float * max(1, n.value))()
        L.check(self.lib.fh_dgraph_stage_times(self.h, names, ms, n.value, C.byref(n)))
        return {names[i].decode(): float(ms[i]) for i in range(n.value)}


class Exchange:
    """all-to-all / all-gather of 1-D tensors with host-known counts: device
    tensors over RCCL, or host copies over gloo."""

    def __init__(self, group, world: int, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group, self.world = torch, dist, group, world
        self.nccl = dist.get_backend(group) == "nccl"
        self.device = device  # where the stages' tensors live (None: CPU arrays)

    def _comm(self, t):
        # gloo: host tensors; nccl: the stage's device tensors
        if self.nccl:
            return t
        if isinstance(t, np.ndarray):
            return self.torch.from_numpy(np.ascontiguousarray(t))
        return t.cpu()

    def _back(self, t, like):
        if isinstance(like, np.ndarray):
            return t.numpy()
        return t.to(like.device) if not self.nccl else t

    def counts(self, send_counts):
        t = self.torch.tensor(np.asarray(send_counts, dtype=np.int64))
        if self.nccl:
            t = t.to(self.device)
        out = self.torch.empty_like(t)
        self.dist.all_to_all_single(out, t, group=self.group)
        return out.cpu().numpy().astype(np.int64)

    def a2a(self, x, send_counts, recv_counts):
        src = self._comm(x)
        out = self.torch.empty(int(np.sum(recv_counts)), dtype=src.dtype, device=src.device)
        self.dist.all_to_all_single(out, src, output_split_sizes=[int(c) for c in recv_counts],
                                    input_split_sizes=[int(c) for c in send_counts],
                                    group=self.group)
        return self._back(out, x)

    def gather(self, *xs):
        """all-gather of several 1-D tensors of one dtype in one exchange:
        one all-gather of the sizes (read back once) and one of the
        concatenated parts -> every rank's parts, concatenated per tensor."""
        srcs = [self._comm(x) for x in xs]
        dev = srcs[0].device
        n = self.torch.tensor([len(t) for t in srcs], dtype=self.torch.int64, device=dev)
        sizes = [self.torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(sizes, n, group=self.group)
        sizes = self.torch.stack(sizes).cpu().tolist()  # [rank][tensor]
        mx = max(1, max(sum(r) for r in sizes))
        buf = self.torch.zeros(mx, dtype=srcs[0].dtype, device=dev)
        o = 0
        for t in srcs:
            buf[o:o + len(t)] = t
            o += len(t)
        bufs = [self.torch.zeros_like(buf) for _ in range(self.world)]
        self.dist.all_gather(bufs, buf, group=self.group)
        outs = []
        for i, x in enumerate(xs):
            parts = []
            for b, r in zip(bufs, sizes):
                o = sum(r[:i])
                parts.append(b[o:o + r[i]])
            outs.append(self._back(self.torch.cat(parts), x))
        return outs[0] if len(xs) == 1 else outs


class DistPartial:
    """One rank of the multi-GPU partial-replication pipeline."""

    def __init__(self, rank: int, world: int, key_space: int, group=None, device: int = 0,
                 backend=None, n: int = 5, solo: bool = False):
        """solo (measurement, for N ranks sharing one GPU): the KeyDeps,
        local, condense and solve stages run one rank at a time between
        barriers, so their stage times are those of a GPU of their own."""
        self.rank, self.world = rank, world
        self.solo = solo
        self.stages = backend if backend is not None else HipStages(rank, world, key_space, device, n)
        dev = None
        if isinstance(self.stages, HipStages):
            dev = self.stages.dev
        self.ex = Exchange(group, world, dev)

    def stage(self, s):
        """s: the whole partially replicated stream with every process's
        element logs (Workload(shards=...).generate(logs=True))."""
        lo, le = shard_logs(s, self.rank, self.world)
        self.send_counts, self.recv_counts, self.range = self.stages.stage(s, lo, le)

    def run(self):
        """One step over the staged stream; returns its wall time (s)."""
        st, ex = self.stages, self.ex
        t0 = time.perf_counter()
        codes = self._solo(lambda: st.keydeps(int(self.send_counts.sum())))
        recv = ex.a2a(codes, self.send_counts, self.recv_counts)
        qc = self._solo(lambda: st.local(recv))
        q = st.queries(int(qc.sum()))
        qin = ex.counts(qc)
        incoming = ex.a2a(q, qc, qin)
        ans = st.answer(incoming)
        answers = ex.a2a(ans, qin, qc)
        verts, edges = self._solo(lambda: st.condense(answers))
        vg, eg = ex.gather(verts, edges)
        # the condensed graph every rank solves (super vertices, edges)
        self.condensed = (len(vg) // 2, len(eg))
        self.condensed_eg = eg if self.solo else None  # (measurement runs)
        ec, elems = self._solo(lambda: st.solve(vg, eg))
        ein = ex.counts(ec)
        mine = ex.a2a(elems, 2 * ec, 2 * ein)
        st.per_key(mine)
        return time.perf_counter() - t0

    def _solo(self, fn):
        if not self.solo:
            return fn()
        out = None
        for q in range(self.world):
            if q == self.rank:
                out = fn()
                sync = getattr(self.stages, "sync", None)
                if sync is not None:
                    sync()  # the stage's kernels end before the next rank's start
            self.ex.dist.barrier(group=self.ex.group)
        return out

    def results(self):
        """(first command, committed deps + SCC labels of the range, per-key
        elements of this rank's keys in execution order)."""
        r = self.stages.results(self.range[1])
        r["first"] = self.range[0]
        return r


def assemble(parts, n: int, key_space: int):
    """Every rank's results -> the stream's committed deps, SCC labels and
    per-key sequences (key_off over the key space, dots)."""
    parts = sorted(parts, key=lambda p: p["first"])
    offs, deps, labels = [np.zeros(1, dtype=np.int64)], [], []
    base = 0
    for p in parts:
        o = p["dep_off"].astype(np.int64)
        offs.append(o[1:] + base)
        base += int(o[-1])
        deps.append(p["deps"])
        labels.append(p["scc_label"])
    dep_off = np.concatenate(offs).astype(np.uint32)
    assert len(dep_off) == n + 1
    kk = np.concatenate([p["pk_key"] for p in parts]).astype(np.int64)
    dd = np.concatenate([p["pk_dot"] for p in parts])
    order = np.argsort(kk, kind="stable")  # ranks own disjoint keys: a stable merge
    kk, dd = kk[order], dd[order]
    key_off = np.zeros(key_space + 1, dtype=np.uint32)
    np.cumsum(np.bincount(kk, minlength=key_space), out=key_off[1:])
    return {"dep_off": dep_off, "deps": np.concatenate(deps), "scc_label": np.concatenate(labels),
            "key_off": key_off, "key_seq": dd}
