"""A/B the radix-sort tile shapes (FH_SORT_CFG) inside one process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24).  Prints per-config median and
min of the probed kernel time and the whole step time."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fantoch_amd.engine import Engine  # noqa: E402


def main():
    cfgs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    probes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["sort_scatter"]
    sys.argv = ["bench.py"]
    args = bench.parse()
    steps = 10
    res = {}
    for r in range(rounds):
        for c in cfgs:
            os.environ["FH_SORT_CFG"] = str(c)
            batches = bench.shard_batches(args, 0, 1, steps + 2) if r == 0 and c == cfgs[0] else batches
            eng = Engine(batches[0].key_space, device=0)
            eng.stage_many(batches)
            eng.run()
            eng.run()
            for pr in probes:
                pass
            eng.set_probe(probes[0])
            t0 = time.perf_counter()
            for _ in range(steps):
                eng.run(sync=False)
            ms, n, b = eng.probe_stats()
            t1 = time.perf_counter()
            res.setdefault(c, {"probe_us": [], "step_us": []})
            res[c]["probe_us"].append(ms * 1e3)
            res[c]["step_us"].append((t1 - t0) / steps * 1e6)
            eng.close()
    out = {c: {k: (float(np.median(v)), float(np.min(v))) for k, v in d.items()} for c, d in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
