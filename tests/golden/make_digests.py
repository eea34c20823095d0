#!/usr/bin/env python
"""Full-size parity fixtures: SHA-256 digests of the oracle's canonical outputs
on the BASELINE.json configurations (test infrastructure, run here on the CPU).

The oracle (oracle/oracle.c: per-replica SequentialKeyDeps + QuorumDeps union
+ incremental GraphExecutor, pinned by the reference's known-answer tests in
tests/test_oracle_golden.py) runs on the seeded generator's streams; the GPU
box regenerates the same streams (fh_workload_*, counter-based) and compares
the engine's outputs against these digests (tests/test_fullsize_gpu.py), so no
oracle output has to travel.

Canonical outputs (tests/fullsize.py: digest_*):
  deps    committed deps per command: dep_off u32[n+1] + dep dots u64, ascending
  labels  min dot of each command's SCC, in command order (u64[n])
  perkey  per-key execution sequence: key_off u32[key_space+1] + dots u64

Configurations (seeds as tools/bench_configs.py):
  c1        Atlas n=5 f=1, ConflictRate 10%, 1 key, 10k commands (full size)
  c4        the headline stream: Zipf 0.99 over 2^20 keys, 1 key, 100M commands
            (full size, bench.py's stream)
  c4shard   key shard 0 of 8 of a 20M-command C4 stream (global dots)
  c4shard_bal  the same stream's shard 0 of 8 under the balanced key map
            (fh_key_owners_balanced over its key counts)
  c4shard_w the same stream's shard 0 of 8 under the work-weighted key map
            (key_owners_weighted; bench.py --gpus N)
  c3        EPaxos ConflictPool 100% (key 0 + 16-key pool), 2 keys: deps at the
            full 10M, everything on the first 50k (the incremental Tarjan is
            quadratic on its one stream-wide SCC)
  c5_12m    Zipf 0.99 over 2^20 keys, 4 keys, unsharded: deps at 12.5M,
            everything on the first 30k
  c5        Atlas partial replication over 8 key shards (processes 5h+1..5h+5,
            dots from the target shard, every shard's own collect and arrival
            delays): deps at the full 100M (fullsize.shard_union), everything
            on the first 20k
Usage: python tests/golden/make_digests.py [--only c1,c4] (c4 needs ~30 GB RAM)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from fullsize import (CONFIGS, DotIndex, digest_deps, digest_labels, digest_perkey,  # noqa: E402
                      shard_union)

OUT = os.path.join(HERE, "digests.json")


def oracle_all(s):
    from oracle import oracle as O
    ko = s.key_off()
    kk = s.keys.reshape(-1)
    off, deps = O.views_run(0, 5, s.dots, ko, kk, s.fq_proc, s.fq_time)
    ex, lab, kso, ks = O.graph_run(s.dots, ko, kk, off, deps, s.key_space)
    assert len(ex) == s.n
    return off, deps, ex, lab, kso, ks


def labels_in_command_order(s, ex, lab):
    out = np.zeros(s.n, dtype=np.uint64)
    out[DotIndex(s.dots)(ex)] = lab
    return out


def oracle_sharded(s):
    """Partial replication: the shards' union (fullsize.shard_union), then
    one GraphExecutor over every command with all its keys."""
    from oracle import oracle as O
    off, deps = shard_union(s)
    ko = s.key_off()
    ex, lab, kso, ks = O.graph_run(s.dots, ko, s.keys.reshape(-1), off, deps, s.key_space)
    assert len(ex) == s.n
    return off, deps, ex, lab, kso, ks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=",".join(CONFIGS))
    a = ap.parse_args()
    res = {}
    if os.path.exists(OUT):
        with open(OUT) as fh:
            res = json.load(fh)
    from oracle import oracle as O
    for name in a.only.split(","):
        c = CONFIGS[name]
        w = c["workload"]()
        t0 = time.time()
        entry = {"desc": c["desc"]}
        if name.startswith("c4shard"):
            full = w.generate(c["total"])
            if c.get("balanced") or c.get("weighted"):
                from fantoch_amd.workload import key_owners_balanced, key_owners_weighted
                om = key_owners_weighted if c.get("weighted") else key_owners_balanced
                owner = om(w.key_histogram(c["total"]), c["nshards"])
                mine = np.nonzero(owner[full.keys[:, 0]] == c["shard"])[0]
            else:
                mine = np.nonzero(full.keys[:, 0] % c["nshards"] == c["shard"])[0]
            from fantoch_amd.workload import Stream
            s = Stream(full.dots[mine], full.keys[mine], full.fq_proc[mine], full.fq_time[mine],
                       full.key_space)
            del full
            off, deps, ex, lab, kso, ks = oracle_all(s)
            pos = {int(d): i for i, d in enumerate(s.dots.tolist())}
            labels = np.zeros(s.n, dtype=np.uint64)
            labels[np.array([pos[int(d)] for d in ex.tolist()])] = lab
            entry.update(n=int(s.n), deps=digest_deps(off, deps), labels=digest_labels(labels),
                         perkey=digest_perkey(kso, ks))
        elif "shards" in c:
            off, deps = shard_union(lambda: w.generate(c["n"]), lean=True,
                                    log=lambda m: print(" ", m, flush=True))
            entry.update(n=int(c["n"]), shards=c["shards"], deps=digest_deps(off, deps),
                         ndeps=int(off[-1]))
            del off, deps
            p = c["prefix"]
            sp = w.generate(p)
            off, deps, ex, lab, kso, ks = oracle_sharded(sp)
            entry["prefix"] = {"n": p, "deps": digest_deps(off, deps),
                               "labels": digest_labels(labels_in_command_order(sp, ex, lab)),
                               "perkey": digest_perkey(kso, ks),
                               "sccs": int(len(np.unique(lab))), "ndeps": int(off[-1])}
        elif "prefix" in c:
            s = w.generate(c["n"])
            ko = s.key_off()
            off, deps = O.views_run(0, 5, s.dots, ko, s.keys.reshape(-1), s.fq_proc, s.fq_time)
            entry.update(n=int(s.n), deps=digest_deps(off, deps), ndeps=int(off[-1]))
            p = c["prefix"]
            sp = w.generate(p)
            off, deps, ex, lab, kso, ks = oracle_all(sp)
            entry["prefix"] = {"n": p, "deps": digest_deps(off, deps),
                               "labels": digest_labels(labels_in_command_order(sp, ex, lab)),
                               "perkey": digest_perkey(kso, ks),
                               "sccs": int(len(np.unique(lab)))}
        else:
            s = w.generate(c["n"])
            off, deps, ex, lab, kso, ks = oracle_all(s)
            entry.update(n=int(s.n), deps=digest_deps(off, deps),
                         labels=digest_labels(labels_in_command_order(s, ex, lab)),
                         perkey=digest_perkey(kso, ks), ndeps=int(off[-1]),
                         sccs=int(len(np.unique(lab))))
        entry["oracle_s"] = round(time.time() - t0, 1)
        res[name] = entry
        print(name, json.dumps(entry), flush=True)
        with open(OUT, "w") as fh:
            json.dump(res, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
