#!/usr/bin/env python
"""Per-phase device times of the C2 secondary line (single view, 1M-command
batches of one Zipf 0.7 stream, every output materialised by run())."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (bring torch's HIP runtime up first)
    from fantoch_amd.engine import Engine
    from fantoch_amd.workload import Stream, Workload
    batch, nb = 1_000_000, 12
    w = Workload.zipf(0.7, 1 << 20, k=1, seed=0xFA170C4000000002, n=5)
    s = w.generate(batch * nb)
    eng = Engine(s.key_space, n=5, device=0)
    eng.stage_many([Stream(s.dots[i * batch:(i + 1) * batch], s.keys[i * batch:(i + 1) * batch],
                           None, None, s.key_space) for i in range(nb)])
    for _ in range(4):
        eng.run(sync=True)
    eng.set_profiling(True)
    acc = {}
    for _ in range(nb - 4):
        eng.run(sync=True)
        for k, v in eng.kernel_times():
            acc.setdefault(k, []).append(v)
    for k, v in acc.items():
        print(f"{k:20s} {np.median(v) * 1e3:8.1f} us")
    print(f"{'total':20s} {sum(np.median(v) for v in acc.values()) * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
