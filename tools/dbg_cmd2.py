"""Debug: command-level KeyDeps across streamed batches vs the oracle."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload, Stream
from oracle import oracle as O
win = int(sys.argv[1]) if len(sys.argv) > 1 else 200
w = Workload.zipf(0.99, 1 << 10, k=1, views=3, window=win, seed=13)
parts = [w.generate(8000, first=i * 8000, logs=True) for i in range(3)]
eng = Engine(w.key_space(), n=5)
eng.stage_logs(parts)
dots = np.concatenate([p.dots for p in parts]); keys = np.concatenate([p.keys for p in parts])
proc = np.concatenate([p.fq_proc for p in parts])
tim = np.concatenate([p.fq_time + np.uint64(i) * np.uint64(1 << 40) for i, p in enumerate(parts)])
st = Stream(dots, keys, proc, tim, w.key_space())
off, deps = O.views_run(0, 5, st.dots, st.key_off(), st.keys.reshape(-1), st.fq_proc, st.fq_time)
dmap = {int(d): i for i, d in enumerate(dots)}
for b in range(3):
    eng.run()
    r = eng.results()
    go, gd = r["dep_off"], r["deps"]
    bad = 0
    for c in range(8000):
        g = b * 8000 + c
        a = gd[go[c]:go[c + 1]]; e = deps[off[g]:off[g + 1]]
        if len(a) != len(e) or not np.array_equal(a, e):
            bad += 1
            if bad <= 4:
                print(b, c, "key", int(keys[g, 0]), "got", [dmap.get(int(x)) for x in a], "exp", [dmap.get(int(x)) for x in e])
    print("batch", b, "bad", bad)
