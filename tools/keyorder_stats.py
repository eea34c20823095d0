#!/usr/bin/env python
"""keyorder_stats.py -- why the C4 graph runs in key order (engine.hip
cmd_views_keyorder): edge spans, ready-time excess H(v) - v and the tile
certificate's failure rate (graph_tile.hip: excess < R0, forward spans <
L - R0 with L = 2·R0) per (R0, core T), in arrival order and in (key,
arrival) order, on a prefix of the C4 stream.  CPU only (oracle KeyDeps +
scipy SCCs).

Usage: python tools/keyorder_stats.py [commands]   (default 5M, ~1 min)
Measured at 5M (round 5): arrival order max excess 728, forward spans <= 62,
5.4 % of T = 8192 tiles failing at R0 = 512; key order max excess 65,
forward spans <= 13, backward <= 20, no failure at R0 >= 128."""
import sys
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from fantoch_amd.workload import Workload  # noqa: E402
from oracle import oracle as O  # noqa: E402


def ready_times(pos, lab, nc, cs, cd):
    """H per vertex: the max position reachable (condensation fixpoint)."""
    mx = np.full(nc, -1, dtype=np.int64)
    np.maximum.at(mx, lab, pos)
    H = mx.copy()
    while True:
        Hn = H.copy()
        np.maximum.at(Hn, cs, H[cd])
        if np.array_equal(Hn, H):
            return H[lab]
        H = Hn


def tiles(ex, src, dst, N, label):
    f = dst > src
    print(f"{label}: max excess {ex.max()}, percentiles 50/90/99/99.9 "
          f"{np.percentile(ex, [50, 90, 99, 99.9]).tolist()}, max forward span "
          f"{(dst - src)[f].max()}, max backward span {(src - dst)[~f].max()}")
    for R0 in (64, 128, 256, 512):
        for T in (4096, 8192):
            L = 2 * R0
            nt = N // T
            e2 = ex[:nt * T].reshape(nt, T).max(1)
            lf = np.zeros(nt, dtype=bool)
            t_ = src[f & ((dst - src) >= L - R0)] // T
            lf[t_[t_ < nt]] = True
            fail = (e2 >= R0) | lf
            print(f"  R0={R0} T={T}: context {T + 2 * L} ({(T + 2 * L) / T:.3f} per core vertex), "
                  f"failing tiles {fail.mean() * 100:.2f}%")


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
    w = Workload.zipf(0.99, 1 << 20, k=1, views=3, window=64, seed=0xFA170C4000000004, n=5)
    s = w.generate(N)
    t = time.time()
    off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc, s.fq_time)
    print(f"oracle KeyDeps + union: {time.time() - t:.1f}s")
    order = np.argsort(s.dots)
    sd = s.dots[order]
    p = np.searchsorted(sd, deps)
    ok = (p < N) & (sd[np.minimum(p, N - 1)] == deps)
    src = np.repeat(np.arange(N), np.diff(off.astype(np.int64)))[ok]
    dst = order[np.minimum(p, N - 1)][ok]
    G = sp.csr_matrix((np.ones(len(src), dtype=np.int8), (src, dst)), shape=(N, N))
    nc, lab = connected_components(G, directed=True, connection="strong")
    cs, cd = lab[src], lab[dst]
    m = cs != cd
    cs, cd = cs[m], cd[m]
    print(f"{N} commands, {len(src)} in-batch edges, {nc} SCCs")
    ar = np.arange(N)
    tiles(ready_times(ar, lab, nc, cs, cd) - ar, src, dst, N, "arrival order")
    pof = np.empty(N, dtype=np.int64)
    pof[np.argsort(s.keys[:, 0], kind="stable")] = ar
    Hp = ready_times(pof, lab, nc, cs, cd)
    exv = np.zeros(N, dtype=np.int64)
    exv[pof] = Hp - pof
    tiles(exv, pof[src], pof[dst], N, "key order")


if __name__ == "__main__" and not (len(sys.argv) > 2 and sys.argv[2] == "groups"):
    main()


def group_stats(N=2_000_000):
    """Fraction of vertices in multi-member ready groups (the key-order
    epilogue's scattered records) and in non-singleton SCCs."""
    w = Workload.zipf(0.99, 1 << 20, k=1, views=3, window=64, seed=0xFA170C4000000004, n=5)
    s = w.generate(N)
    off, deps = O.views_run(0, 5, s.dots, s.key_off(), s.keys.reshape(-1), s.fq_proc, s.fq_time)
    order = np.argsort(s.dots)
    sd = s.dots[order]
    p = np.searchsorted(sd, deps)
    ok = (p < N) & (sd[np.minimum(p, N - 1)] == deps)
    src = np.repeat(np.arange(N), np.diff(off.astype(np.int64)))[ok]
    dst = order[np.minimum(p, N - 1)][ok]
    G = sp.csr_matrix((np.ones(len(src), dtype=np.int8), (src, dst)), shape=(N, N))
    nc, lab = connected_components(G, directed=True, connection="strong")
    cs, cd = lab[src], lab[dst]
    m = cs != cd
    H = ready_times(np.arange(N), lab, nc, cs[m], cd[m])
    gsize = np.bincount(H, minlength=N)[H]
    ssize = np.bincount(lab, minlength=nc)[lab]
    print(f"multi-member ready groups: {np.mean(gsize > 1) * 100:.1f}% of vertices; raised "
          f"{np.mean(H > np.arange(N)) * 100:.1f}%; non-singleton SCCs {np.mean(ssize > 1) * 100:.2f}%")


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "groups":
    group_stats(int(sys.argv[1]))
