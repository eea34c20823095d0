#!/usr/bin/env python
"""C5 probe: the partially replicated 4-key Zipf stream (seed as
tests/fullsize.py, 8 shards) at a given size through the fused engine on one
GPU; wall ms per step and the phase profile (FH_GRAPH_DEBUG=1 adds the graph
stage's rounds on stderr)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fantoch_amd.engine import Engine  # noqa: E402
from fantoch_amd.workload import Workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--shards", type=int, default=8)
    a = ap.parse_args()
    t = time.time()
    s = Workload.zipf(0.99, 1 << 20, k=4, views=3, window=64, seed=0xFA170C4000000005,
                      n=5, shards=a.shards).generate(a.n, logs=True, times=False)
    print(json.dumps({"gen_s": round(time.time() - t, 1)}), flush=True)
    eng = Engine(s.key_space, n=5, device=0)
    t = time.time()
    eng.stage(s)
    print(json.dumps({"stage_s": round(time.time() - t, 1)}), flush=True)
    for i in range(a.steps):
        eng.rewind()
        t = time.time()
        ms = eng.run(sync=True)
        print(json.dumps({"step": i, "device_ms": round(ms, 2),
                          "wall_ms": round((time.time() - t) * 1e3, 2)}), flush=True)
    eng.set_profiling(True)
    eng.rewind()
    eng.run(sync=True)
    print(json.dumps({"phases_ms": {k: round(v, 3) for k, v in eng.kernel_times()}}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
