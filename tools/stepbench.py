"""Step-time decomposition for the C2 bench: wall time per step with and
without roofline probe events, and the host cost of one fh_engine_run call."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fantoch_amd.engine import Engine  # noqa: E402
from fantoch_amd.shard import shard_batches  # noqa: E402
from fantoch_amd.workload import Workload  # noqa: E402

w = Workload.zipf(0.7, 1 << 20, k=1, seed=0xFA170C4000000002, n=5)
nb = 5 + 3 * 20
batches = shard_batches(w, 0, 1, 1_000_000, nb)
eng = Engine(batches[0].key_space, n=5, device=0)
eng.stage_many(batches)
for _ in range(5):
    eng.run(sync=False)
torch.cuda.synchronize()


def timed(probe, steps=20):
    eng.set_probe(probe)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(steps):
        h0 = time.perf_counter()
        eng.run(sync=False)
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    eng.set_probe(None)
    return (t1 - t0) / steps * 1e6, host / steps * 1e6


for probe in (None, "kb_partition,kb_order", None):
    wall, host = timed(probe)
    print(f"probe={probe}: {wall:.1f} us/step wall, {host:.1f} us/step host enqueue")
