"""C5 graph statistics on a prefix of the stream (CPU, numpy/scipy; analysis
only, nothing here is product code).

Builds the committed-deps graph of the first N commands of the C5 stream
(tests/fullsize.py's shard_union, the partial-replication dep union) and
reports what DESIGN.md §5.2 / §9 quote for the global SCC path:

* edge counts, forward / backward spans, SCC sizes;
* tile-local SCC contraction: SCCs of the subgraphs induced by 1024 / 2048 /
  4096-position tiles, and how many edges stay between classes (raw, after
  deduplicating each class's targets, as class-to-class edges);
* edges implied by a two-edge path (droppable without changing reachability
  or longest paths);
* how much edge work a frontier version of the coloring's H propagation
  would do (vertices re-evaluated only when a target's H changed).

Usage: python tools/c5_graph_stats.py [N]   (default 2,000,000; ~15 min, ~20 GB)
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def c5_graph(n):
    from fullsize import shard_union
    from fantoch_amd.workload import Workload
    w = Workload.zipf(0.99, 1 << 20, k=4, views=3, window=64, seed=0xFA170C4000000005, n=5,
                      shards=8)
    s = w.generate(n, logs=True)
    off, deps = shard_union(s)
    order = np.argsort(s.dots)
    dst = order[np.searchsorted(s.dots[order], deps)].astype(np.int64)
    src = np.repeat(np.arange(n), np.diff(off.astype(np.int64)))
    m = dst != src
    return src[m], dst[m]


def scc_labels(n, src, dst):
    a = sp.csr_matrix((np.ones(len(src), np.int8), (src, dst)), shape=(n, n))
    return connected_components(a, directed=True, connection="strong")[1]


def window_classes(n, src, dst, bs=128):
    """The engine's windows: SCCs of bs-position blocks and of the blocks
    shifted by bs / 2, united (k_windows' classes)."""
    def block(off):
        m = (src + off) // bs == (dst + off) // bs
        return scc_labels(n, src[m], dst[m])
    l1, l2 = block(0), block(bs // 2)
    n1 = l1.max() + 1
    u = sp.csr_matrix((np.ones(2 * n, np.int8), (np.r_[np.arange(n), np.arange(n)], np.r_[l1, n1 + l2])),
                      shape=(n, n1 + l2.max() + 1))
    g = sp.bmat([[None, u], [u.T, None]])
    return connected_components(g, directed=False)[1][:n]


def frontier_sweeps(n, src, dst, cls):
    """Round 1 of the coloring's H propagation (pull, class maxima, pointer
    jumping) as synchronous sweeps: per sweep the vertices whose H changed,
    and the edges a frontier version would touch (those of vertices with a
    target that changed in the previous sweep)."""
    e = len(src)
    mx = np.zeros(cls.max() + 1, np.int64)
    np.maximum.at(mx, cls, np.arange(n))
    h = mx[cls]
    deg = np.bincount(src, minlength=n)
    changed = np.ones(n, bool)
    full = front = 0
    for it in range(1, 64):
        need = np.zeros(n, bool)
        need[src[changed[dst]]] = True
        need |= changed
        front += int(deg[need].sum())
        full += e
        best = h.copy()
        np.maximum.at(best, src, h[dst])
        hc = np.zeros(cls.max() + 1, np.int64)
        np.maximum.at(hc, cls, best)
        nh = hc[cls]
        nh = np.maximum(nh, nh[np.minimum(nh, n - 1)])
        changed = nh != h
        print(f"  sweep {it}: {int(changed.sum())} vertices changed, frontier edges "
              f"{int(deg[need].sum())} of {e}")
        h = nh
        if not changed.any():
            break
    print(f"H propagation edge work: frontier / full = {front / full:.2f}")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    t = time.time()
    src, dst = c5_graph(n)
    e = len(src)
    fw = dst > src
    print(f"N {n} edges {e} forward {int(fw.sum())} ({time.time() - t:.0f} s)")
    print("forward span p50/p99/max", np.percentile(dst[fw] - src[fw], [50, 99, 100]))
    print("backward span p50/p99/max", np.percentile(src[~fw] - dst[~fw], [50, 99, 100]))
    lab = scc_labels(n, src, dst)
    sz = np.bincount(lab)
    print(f"sccs {len(sz)} largest {sz.max()} ({sz.max() / n:.1%}) singletons {int((sz == 1).sum())}")
    for bs in (1024, 2048, 4096):
        m = src // bs == dst // bs
        cl = scc_labels(n, src[m], dst[m])
        inter = cl[src] != cl[dst]
        cv = len(np.unique(cl[src[inter]].astype(np.int64) * n + dst[inter]))
        cc = len(np.unique(cl[src[inter]].astype(np.int64) * n + cl[dst[inter]]))
        print(f"tile {bs}: classes {len(np.unique(cl))} ({len(np.unique(cl)) / n:.1%}), "
              f"inter-class edges {inter.mean():.1%}, class->vertex rows {cv / e:.1%}, "
              f"class->class {cc / e:.1%}")
    a = sp.csr_matrix((np.ones(e, np.float32), (src, dst)), shape=(n, n))
    a.sum_duplicates()
    a.data[:] = 1
    a2 = a @ a
    a2.data[:] = 1
    red = a.multiply(a2).nnz
    print(f"distinct edges {a.nnz}, implied by a two-edge path {red} ({red / a.nnz:.1%})")
    frontier_sweeps(n, src, dst, window_classes(n, src, dst))


if __name__ == "__main__":
    main()
