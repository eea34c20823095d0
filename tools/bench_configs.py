#!/usr/bin/env python
"""Throughput of the fused engine (fh_engine_*) on BASELINE.json's other
configurations, one GPU, one JSON line per configuration.

bench.py stays the headline (C2).  This script measures the replica-view
configurations on their full per-GPU sizes:

* C1 -- Atlas n=5 f=1, ConflictRate 10 %, 1 key, 10k commands (plumbing size);
* C3 -- EPaxos n=5 (fast quorum 3), ConflictPool 100 % on key 0 + a 16-key
  pool, 2 keys/cmd, 10M commands: one stream-wide SCC;
* C4 -- one GPU's key shard of the 8-GPU Zipf 0.99 stream: 12.5M commands
  (100M / 8), 1 key/cmd, replica views;
* C5 -- one shard's slice of the partial-replication stream: 4 keys/cmd,
  Zipf 0.99, replica views, 12.5M commands.

A step = one engine pass over the whole staged stream (views' KeyDeps +
QuorumDeps union -> SCCs -> execution order -> per-key sequences) from a clean
engine, inputs resident in HBM (reset + stage happen before the clock starts;
replica views reorder commands across any batch cut, so the stream is one
batch).  The CPU column is the oracle (the C restatement of the reference's
per-replica SequentialKeyDeps + QuorumDeps + incremental GraphExecutor) on a
bounded prefix of the same stream, one thread: the reference's incremental
Tarjan re-walks the pending graph on every add, so C3's single SCC makes it
quadratic and the sample is small.

Parity at these shapes is in tests/test_engine_gpu.py; this script only times.
Usage: python tools/bench_configs.py [--only c3,c4] [--steps 3] [--no-cpu]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "c1": dict(desc="C1: Atlas n=5 f=1, ConflictRate 10%, 1 key/cmd, replica views (fq=3)",
               kind="rate", rate=10, k=1, n=10_000, cpu=10_000),
    "c3": dict(desc="C3: EPaxos n=5 fq=3, ConflictPool 100% (key 0 + 16-key pool), "
                    "2 keys/cmd, replica views, one stream-wide SCC",
               kind="pool", rate=100, pool=16, k=2, n=10_000_000, cpu=10_000),
    "c4": dict(desc="C4 shard: Zipf 0.99 over 1M keys, 1 key/cmd, replica views (fq=3), "
                    "100M/8 commands = one GPU's key shard",
               kind="zipf", s=0.99, keys=1 << 20, k=1, n=12_500_000, cpu=400_000),
    "c5": dict(desc="C5 shard: Zipf 0.99 over 1M keys, 4 keys/cmd, replica views (fq=3), "
                    "100M/8 commands",
               kind="zipf", s=0.99, keys=1 << 20, k=4, n=12_500_000, cpu=4_000),
}


def workload(c, seed):
    from fantoch_amd.workload import Workload
    kw = dict(views=3, window=64, seed=seed, n=5)
    if c["kind"] == "rate":
        return Workload.conflict_rate_(c["rate"], k=c["k"], **kw)
    if c["kind"] == "pool":
        return Workload.conflict_pool(c["rate"], c["pool"], k=c["k"], **kw)
    return Workload.zipf(c["s"], c["keys"], k=c["k"], **kw)


def cpu_rate(s, count):
    from oracle import oracle as O
    count = min(count, s.n)
    dots = s.dots[:count]
    keys = s.keys[:count].reshape(-1)
    key_off = (np.arange(count + 1, dtype=np.uint64) * s.k).astype(np.uint32)
    t0 = time.perf_counter()
    off, deps = O.views_run(0, 5, dots, key_off, keys, s.fq_proc[:count], s.fq_time[:count])
    ex, lab, kso, ks = O.graph_run(dots, key_off, keys, off, deps, s.key_space)
    dt = time.perf_counter() - t0
    return count / dt, dt, count


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c1,c3,c4,c5")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--scale", type=float, default=1.0, help="multiply command counts")
    args = ap.parse_args()
    import torch  # noqa: F401  (device context, like bench.py)

    from fantoch_amd.engine import Engine

    for name in [x for x in args.only.split(",") if x]:
        c = CONFIGS[name]
        n = max(1000, int(c["n"] * args.scale))
        w = workload(c, 0xFA170C4000000000 + int(name[1]))
        t0 = time.perf_counter()
        batch = w.generate(n)
        tgen = time.perf_counter() - t0
        eng = Engine(batch.key_space, n=5, device=0)
        dev_ms, wall = [], []
        for i in range(args.warmup + args.steps):
            # each step orders the whole stream from a clean engine (reset +
            # stage are outside the timed region)
            eng.reset()
            eng.stage(batch)
            t = time.perf_counter()
            ms_ = eng.run(sync=True)
            if i >= args.warmup:
                wall.append(time.perf_counter() - t)
                dev_ms.append(ms_)
        r = eng.results()
        _, counts = np.unique(r["scc_label"], return_counts=True)
        # phases of one more step on the same (warm) engine
        eng.reset()
        eng.stage(batch)
        eng.set_profiling(True)
        eng.run(sync=True)
        phases = {}
        for k, v in eng.kernel_times():
            phases[k] = round(phases.get(k, 0.0) + v, 4)
        eng.close()
        ms = float(np.median(wall)) * 1e3
        out = {"config": name, "workload": c["desc"], "cmds_per_step": n, "steps": args.steps,
               "ms_per_step": ms, "device_ms_per_step": float(np.median(dev_ms)),
               "value": n / (ms * 1e-3), "unit": "commands/s", "largest_scc": int(counts.max()),
               "sccs": int(len(counts)), "gen_s": tgen, "phases_ms": phases}
        if not args.no_cpu:
            v, dt, cnt = cpu_rate(batch, c["cpu"])
            out["cpu_baseline"] = {"value": v, "unit": "commands/s", "cores": 1, "kind": "port",
                                   "sample": f"first {cnt} commands of the same stream, oracle "
                                             f"views KeyDeps + QuorumDeps + incremental "
                                             f"GraphExecutor, 1 thread, {dt:.2f}s"}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
