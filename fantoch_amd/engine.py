"""Engine -- the fused device-resident dependency engine (fh_engine_*).

deps (KeyDeps per replica view + QuorumDeps union) -> SCC -> execution order
-> per-key execution sequence, for one batch of commands staged in HBM.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .keydeps import make_config


class Engine:
    def __init__(self, key_space: int, n: int = 5, f: int = 1, device: int = -1):
        self._lib = L.load()
        self.key_space = key_space
        self.cfg = make_config(n=n, f=f, device=device, key_space=key_space)
        h = C.c_void_p()
        L.check(self._lib.fh_engine_create(C.byref(self.cfg), C.byref(h)))
        self._h = h
        self.n = 0
        self.k = 0

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fh_engine_destroy(self._h)
            self._h = None

    __del__ = close

    def reset(self):
        L.check(self._lib.fh_engine_reset(self._h))

    def rewind(self):
        """Replay the staged batches from a clean state (on the engine stream,
        no host synchronisation)."""
        L.check(self._lib.fh_engine_rewind(self._h))

    def sync(self):
        """Wait for every run issued on the engine's stream (fh_engine_sync)."""
        L.check(self._lib.fh_engine_sync(self._h))

    def set_profiling(self, on: bool):
        L.check(self._lib.fh_engine_set_profiling(self._h, 1 if on else 0))

    def set_deps_only(self, on: bool):
        """run() stops after the committed deps (fh_engine_set_deps_only)."""
        L.check(self._lib.fh_engine_set_deps_only(self._h, 1 if on else 0))

    def forget_tuning(self):
        """The next run starts from a fresh engine's tuning guesses
        (fh_engine_forget_tuning): the cold-run cost of the graph stage."""
        L.check(self._lib.fh_engine_forget_tuning(self._h))

    def dep_total(self) -> int:
        """Committed deps of the last run (the CSR's length), no copy."""
        ln = C.c_size_t(0)
        L.check(self._lib.fh_engine_results(self._h, None, None, 0, C.byref(ln), None, None,
                                            None, None))
        return int(ln.value)

    def deps(self):
        """The last run's committed deps only: (dep_off u32[n+1], deps u64)."""
        n = self.n
        dep_off = np.zeros(n + 1, dtype=np.uint32)
        ln = C.c_size_t(0)
        L.check(self._lib.fh_engine_results(self._h, L.ptr(dep_off), None, 0, C.byref(ln), None,
                                            None, None, None))
        deps = np.zeros(max(1, ln.value), dtype=np.uint64)
        L.check(self._lib.fh_engine_results(self._h, L.ptr(dep_off), L.ptr(deps), len(deps),
                                            C.byref(ln), None, None, None, None))
        return dep_off, deps[:ln.value]

    def stage(self, stream, nproc: int = 5):
        """stream: fantoch_amd.workload.Stream (views taken from it; its
        per-replica logs if generated, else fq_proc / fq_time)."""
        if stream.log_cmd is not None or stream.log_elem is not None:
            return self.stage_logs([stream], nproc)
        views = 0 if stream.fq_proc is None else stream.fq_proc.shape[1]
        d = L.fh_stream_desc(n=stream.n, keys_per_cmd=stream.k, views=views,
                             nproc=nproc if views else 0, flags=0)
        dots = np.ascontiguousarray(stream.dots, dtype=np.uint64)
        keys = np.ascontiguousarray(stream.keys, dtype=np.uint64)
        proc = None if not views else np.ascontiguousarray(stream.fq_proc, dtype=np.uint8)
        tim = None if not views else np.ascontiguousarray(stream.fq_time, dtype=np.uint64)
        L.check(self._lib.fh_engine_stage(self._h, C.byref(d), L.ptr(dots), L.ptr(keys),
                                          L.ptr(proc), L.ptr(tim)))
        self.n, self.k = stream.n, stream.k

    def stage_many(self, batches, nproc: int = 5):
        """Stage a list of equally sized Streams; each run() processes the next."""
        first = batches[0]
        views = 0 if first.fq_proc is None else first.fq_proc.shape[1]
        d = L.fh_stream_desc(n=first.n, keys_per_cmd=first.k, views=views,
                             nproc=nproc if views else 0, flags=0)
        assert all(b.n == first.n and b.k == first.k for b in batches)
        dots = np.ascontiguousarray(np.concatenate([b.dots for b in batches]), dtype=np.uint64)
        keys = np.ascontiguousarray(np.concatenate([b.keys for b in batches]), dtype=np.uint64)
        proc = tim = None
        if views:
            proc = np.ascontiguousarray(np.concatenate([b.fq_proc for b in batches]), np.uint8)
            tim = np.ascontiguousarray(np.concatenate([b.fq_time for b in batches]), np.uint64)
        L.check(self._lib.fh_engine_stage_many(self._h, C.byref(d), len(batches), L.ptr(dots),
                                               L.ptr(keys), L.ptr(proc), L.ptr(tim)))
        self.n, self.k = first.n, first.k

    def stage_logs(self, batches, nproc: int = 5):
        """Stage Streams that carry per-replica arrival logs (equal sizes);
        each run() processes the next.  Element logs (partial replication)
        carry their own process count, len(log_off) - 1."""
        first = batches[0]
        views = first.views
        elem = first.log_elem is not None
        if elem:
            nproc = len(first.log_off) - 1
        assert views >= 1 and all(b.n == first.n and b.k == first.k for b in batches)
        d = L.fh_stream_desc(n=first.n, keys_per_cmd=first.k, views=views, nproc=nproc,
                             flags=L.FH_STREAM_ELEMENT_LOGS if elem else 0)
        one = len(batches) == 1
        dots = np.ascontiguousarray(first.dots if one else np.concatenate([b.dots for b in batches]),
                                    dtype=np.uint64)
        keys = np.ascontiguousarray(first.keys if one else np.concatenate([b.keys for b in batches]),
                                    dtype=np.uint64)
        offs, base = [np.zeros(1, dtype=np.uint64)], 0
        for b in batches:
            assert len(b.log_off) == nproc + 1 and (b.log_elem is not None) == elem
            offs.append(b.log_off[1:].astype(np.uint64) + np.uint64(base))
            base += int(b.log_off[-1])
        off = np.concatenate(offs)
        ent = [b.log_elem if elem else b.log_cmd for b in batches]
        ent = np.ascontiguousarray(ent[0] if one else np.concatenate(ent), dtype=np.uint32)
        L.check(self._lib.fh_engine_stage_logs(self._h, C.byref(d), len(batches), L.ptr(dots),
                                               L.ptr(keys), L.ptr(off), L.ptr(ent)))
        self.n, self.k = first.n, first.k

    def run(self, sync: bool = True) -> float:
        ms = C.c_float(0)
        L.check(self._lib.fh_engine_run(self._h, C.byref(ms) if sync else None))
        return float(ms.value)

    def set_probe(self, kernel):
        """kernel: a name, a comma-separated list of names, or None (off)."""
        if isinstance(kernel, (list, tuple)):
            kernel = ",".join(kernel)
        L.check(self._lib.fh_engine_set_probe(self._h, kernel.encode() if kernel else None))

    def probe_stats(self, kernel=None):
        """(average device ms per launch, launches, algorithmic bytes per launch)."""
        ms, n, b = C.c_float(0), C.c_size_t(0), C.c_double(0)
        L.check(self._lib.fh_engine_probe_stats_for(self._h, kernel.encode() if kernel else None,
                                                    C.byref(ms), C.byref(n), C.byref(b)))
        return float(ms.value), int(n.value), float(b.value)

    def kernel_times(self):
        n = C.c_size_t(0)
        L.check(self._lib.fh_engine_kernel_times(self._h, None, None, 0, C.byref(n)))
        names = (C.c_char_p * max(1, n.value))()
        ms = (C.c_float * max(1, n.value))()
        L.check(self._lib.fh_engine_kernel_times(self._h, names, ms, n.value, C.byref(n)))
        return [(names[i].decode(), float(ms[i])) for i in range(n.value)]

    def results(self):
        n = self.n
        dep_off = np.zeros(n + 1, dtype=np.uint32)
        ln = C.c_size_t(0)
        L.check(self._lib.fh_engine_results(self._h, L.ptr(dep_off), None, 0, C.byref(ln), None,
                                            None, None, None))
        deps = np.zeros(max(1, ln.value), dtype=np.uint64)
        label = np.zeros(n, dtype=np.uint64)
        rank = np.zeros(n, dtype=np.uint32)
        key_off = np.zeros(self.key_space + 1, dtype=np.uint32)
        L.check(self._lib.fh_engine_results(self._h, None, None, 0, None, None, None,
                                            L.ptr(key_off), None))
        key_seq = np.zeros(max(1, int(key_off[-1])), dtype=np.uint64)
        L.check(self._lib.fh_engine_results(self._h, L.ptr(dep_off), L.ptr(deps), len(deps),
                                            C.byref(ln), L.ptr(label), L.ptr(rank), None,
                                            L.ptr(key_seq)))
        return {"dep_off": dep_off, "deps": deps[:ln.value], "scc_label": label,
                "exec_rank": rank, "key_off": key_off, "key_seq": key_seq[:int(key_off[-1])]}
