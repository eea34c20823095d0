#!/usr/bin/env python
"""C4 key-shard probe: the largest shard of the 100M-command C4 stream under
the balanced key map at N ranks (what one rank of `bench.py --gpus N`
orders), through the fused engine on this GPU: wall ms per step, the phase
profile, and (with --steps) a loop rocprofv3 can trace.

Usage: python tools/shard_probe.py [--ranks 8] [--steps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fantoch_amd.engine import Engine  # noqa: E402
from fantoch_amd.workload import Workload, key_owners_balanced  # noqa: E402

try:
    from fantoch_amd.workload import key_owners_weighted  # noqa: E402
except ImportError:  # (older trees)
    key_owners_weighted = None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--commands", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--shards", default="", help="comma-separated shard ids (default: the largest)")
    ap.add_argument("--owners", default="balanced", help="balanced | weighted (key map)")
    a = ap.parse_args()
    w = Workload.zipf(0.99, 1 << 20, k=1, views=3, window=64, seed=0xFA170C4000000004, n=5)
    h = w.key_histogram(a.commands)
    owner = key_owners_balanced(h, a.ranks) if a.owners == "balanced" else \
        key_owners_weighted(h, a.ranks)
    loads = np.bincount(owner, weights=h.astype(np.float64), minlength=a.ranks)
    shards = [int(x) for x in a.shards.split(",")] if a.shards else [int(np.argmax(loads))]
    for q in shards:
        probe(w, a, owner, q)


def probe(w, a, owner, q):
    s = w.generate_shard(a.commands, a.ranks, q, owner=owner)
    eng = Engine(s.key_space, n=5, device=0)
    eng.stage(s)
    eng.rewind()
    eng.run(sync=True)  # warmup (the graph stage learns its reach bound)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.rewind()
        eng.run(sync=False)
    eng.sync()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    eng.set_profiling(True)
    eng.rewind()
    eng.run(sync=True)
    phases = {k: round(v, 4) for k, v in eng.kernel_times()}
    eng.set_profiling(False)
    eng.close()
    hot = int(np.bincount(s.keys[:, 0].astype(np.int64)).max())
    print(json.dumps({"ranks": a.ranks, "owners": a.owners, "shard": q, "commands": int(s.n),
                      "hottest_key_commands": hot, "ms_per_step": round(ms, 4),
                      "phases_ms": phases}), flush=True)


if __name__ == "__main__":
    main()
