#!/usr/bin/env python
"""One rank's fh_dgraph KeyDeps stage on its own (no exchange, one process):
the C5 stream (tests/fullsize.py's seed, 8 shards), rank R of N's element
logs staged through fh_dgraph_stage, then fh_dgraph_keydeps timed per step
and the engine's phase profile of the last one -- so rocprofv3 can trace a
rank's KeyDeps without a multi-process launcher.

Usage: python tools/dgraph_keydeps_probe.py [--rank 0 --world 8 --steps 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import torch  # noqa: F401  (torch's HIP runtime first)
    from fantoch_amd.dgraph import HipStages, shard_logs
    from fantoch_amd.workload import Workload
    t = time.time()
    s = Workload.zipf(0.99, 1 << 20, k=4, views=3, window=64, seed=0xFA170C4000000005,
                      n=5, shards=8).generate(a.n, logs=True, times=False)
    print(json.dumps({"gen_s": round(time.time() - t, 1)}), flush=True)
    st = HipStages(a.rank, a.world, s.key_space, 0, 5)
    lo, le = shard_logs(s, a.rank, a.world)
    t = time.time()
    sc, rc, rng = st.stage(s, lo, le)
    print(json.dumps({"stage_s": round(time.time() - t, 1), "elements": int(lo[-1]),
                      "send": int(sc.sum()), "range": list(rng)}), flush=True)
    for i in range(a.steps):
        t = time.time()
        st.keydeps(int(sc.sum()))
        st.sync()
        print(json.dumps({"step": i, "keydeps_wall_ms": round((time.time() - t) * 1e3, 2)}),
              flush=True)
    st.close()


if __name__ == "__main__":
    main()
