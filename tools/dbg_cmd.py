"""Debug: command-level KeyDeps vs the oracle on a small C4-shaped stream."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fantoch_amd.engine import Engine
from fantoch_amd.workload import Workload
from oracle import oracle as O
n = int(sys.argv[1]) if len(sys.argv) > 1 else 120_000
s = Workload.zipf(0.99, 1 << 16, k=1, views=3, window=64, seed=12).generate(n, logs=True)
eng = Engine(s.key_space, n=5)
eng.stage_logs([s])
eng.run()
r = eng.results()
off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc, s.fq_time)
go, gd = r["dep_off"], r["deps"]
print("dep totals", int(go[-1]), int(off[-1]))
cnt_g = np.diff(go.astype(np.int64)); cnt_o = np.diff(off.astype(np.int64))
bad = []
for c in range(s.n):
    a = gd[go[c]:go[c + 1]]; b = deps[off[c]:off[c + 1]]
    if len(a) != len(b) or not np.array_equal(a, b):
        bad.append(c)
        if len(bad) <= 8:
            print(c, "key", int(s.keys[c, 0]), "got", [hex(x) for x in a], "exp", [hex(x) for x in b])
print("bad", len(bad))
dmap = {int(d): i for i, d in enumerate(s.dots)}
for c in bad[:4]:
    a = gd[go[c]:go[c + 1]]; b = deps[off[c]:off[c + 1]]
    print(c, "got cmds", [dmap.get(int(x)) for x in a], "exp cmds", [dmap.get(int(x)) for x in b])
