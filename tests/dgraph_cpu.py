"""A CPU mirror of the fh_dgraph_* steps (csrc/dgraph.hip), test
infrastructure only: the world-size-2 gloo test runs fantoch_amd.dgraph's
orchestration and exchanges with these stages in place of the HIP ones and
compares the assembled outputs with the single-process oracle.  Same
interfaces and payload encodings as HipStages; the per-range computations are
plain restatements (per-process SequentialKeyDeps over element logs, the
per-command union, scipy SCCs, ready times / depths over the condensation in
topological order)."""
from __future__ import annotations

import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components

MARKER = 0x80000000


def _scc_order(nv, src, dst, key, dot):
    """SCCs of a graph (vertices 0..nv-1, edges src -> dst) with, per
    vertex: the SCC's representative (min vertex), its label (min dot), its
    ready time H = max key reachable, and its depth (longest path to a
    same-H successor SCC)."""
    if nv == 0:
        z = np.zeros(0, dtype=np.int64)
        return z, np.zeros(0, np.uint64), z, z
    g = csr_matrix((np.ones(len(src), np.int8), (src, dst)), shape=(nv, nv))
    nc, comp = connected_components(g, directed=True, connection="strong")
    rep = np.full(nc, nv, dtype=np.int64)
    np.minimum.at(rep, comp, np.arange(nv))
    lab = np.full(nc, np.iinfo(np.uint64).max, dtype=np.uint64)
    np.minimum.at(lab, comp, dot.astype(np.uint64))
    own = np.zeros(nc, dtype=np.int64)
    np.maximum.at(own, comp, key.astype(np.int64))
    cs, cd = comp[src], comp[dst]
    m = cs != cd
    cs, cd = cs[m], cd[m]
    succ = [[] for _ in range(nc)]
    indeg = np.zeros(nc, dtype=np.int64)
    for a, b in set(zip(cs.tolist(), cd.tolist())):
        succ[a].append(b)
        indeg[b] += 1
    # reverse topological order (Kahn on the condensation DAG)
    order, stack = [], [c for c in range(nc) if indeg[c] == 0]
    while stack:
        c = stack.pop()
        order.append(c)
        for b in succ[c]:
            indeg[b] -= 1
            if indeg[b] == 0:
                stack.append(b)
    assert len(order) == nc
    H = own.copy()
    depth = np.zeros(nc, dtype=np.int64)
    for c in reversed(order):
        for b in succ[c]:
            H[c] = max(H[c], H[b])
    for c in reversed(order):
        for b in succ[c]:
            if H[b] == H[c]:
                depth[c] = max(depth[c], depth[b] + 1)
    return rep[comp], lab[comp], H[comp], depth[comp]


class CpuStages:
    def __init__(self, rank: int, world: int, key_space: int, n: int = 5):
        self.rank, self.world, self.K = rank, world, key_space

    def stage(self, s, log_off, log_elem):
        self.s = s
        n, k, V = s.n, s.k, s.views
        S = self.S = k * V
        self.bounds = np.asarray([n * q // self.world for q in range(self.world + 1)], np.int64)
        self.a = int(self.bounds[self.rank])
        self.V = int(self.bounds[self.rank + 1]) - self.a
        self.log_off, self.log_elem = log_off.astype(np.int64), log_elem.astype(np.int64)
        self.mine = np.sort(self.log_elem)
        dest = np.searchsorted(self.bounds, self.mine // S, side="right") - 1
        send = np.bincount(dest, minlength=self.world)
        p = np.arange(self.a * S, (self.a + self.V) * S, dtype=np.int64)
        c, sl = p // S, p % k
        src = ((s.keys[c, sl] % np.uint64(s.shards)) % np.uint64(self.world)).astype(np.int64)
        o = np.lexsort((p, src))
        self.recv_pos = p[o] - self.a * S
        recv = np.bincount(src, minlength=self.world)
        hb = int(n).bit_length()
        self.hb = max(hb, 1)
        seq = s.dots & np.uint64((1 << 56) - 1)
        self.seqb = int(int(seq.max())).bit_length()
        return send.astype(np.int64), recv.astype(np.int64), (self.a, self.V)

    def keydeps(self, nsend):
        s, S, k = self.s, self.S, self.s.k
        code = {}
        for r in range(len(self.log_off) - 1):
            latest = {}
            for p in self.log_elem[self.log_off[r]:self.log_off[r + 1]].tolist():
                key = int(s.keys[p // S, p % k])
                code[p] = latest.get(key, 0)
                latest[key] = p // S + 1
        return np.asarray([code[p] for p in self.mine.tolist()], dtype=np.int32)

    def local(self, recv):
        s, S, a, V = self.s, self.S, self.a, self.V
        codes = np.zeros(V * S, dtype=np.int64)
        codes[self.recv_pos] = np.asarray(recv, dtype=np.int64) & 0xFFFFFFFF
        rows = codes.reshape(V, S)
        src, dst, off, deps = [], [], [0], []
        for v in range(V):
            vids = sorted(set(int(x) - 1 for x in rows[v] if x))
            deps.extend(sorted(int(d) for d in s.dots[vids]) if vids else [])
            off.append(len(deps))
            src.extend([v] * len(vids))
            dst.extend(vids)
        self.dep_off = np.asarray(off, np.uint32)
        self.deps = np.asarray(deps, np.uint64)
        src, dst = np.asarray(src, np.int64), np.asarray(dst, np.int64)
        loc = (dst >= a) & (dst < a + V)
        self.lsrc, self.ldst = src[loc], dst[loc] - a
        self.csrc, self.cdst = src[~loc], dst[~loc]
        self.rep, self.lab, self.H, self.depth = _scc_order(
            V, self.lsrc, self.ldst, np.arange(a, a + V), s.dots[a:a + V])
        # escaping: reaches a vertex with a cross-range edge
        esc = np.zeros(V, bool)
        esc[self.csrc] = True
        esc_rep = np.zeros(V, bool)
        esc_rep[self.rep[esc]] = True
        while True:
            e = esc_rep[self.rep]
            grow = np.zeros(V, bool)
            grow[self.lsrc[e[self.ldst]]] = True
            new = esc_rep.copy()
            new[self.rep[grow]] = True
            if np.array_equal(new, esc_rep):
                break
            esc_rep = new
        self.esc = esc_rep[self.rep]
        self.q = np.unique(self.cdst)
        owner = np.searchsorted(self.bounds, self.q, side="right") - 1
        return np.bincount(owner, minlength=self.world).astype(np.int64)

    def queries(self, nq):
        return self.q.astype(np.int32)

    def _code_of(self, lw):
        r = self.rep[lw]
        return np.where(self.esc[lw], self.a + r, MARKER | self.H[lw]).astype(np.int64)

    def answer(self, q):
        lw = np.asarray(q, dtype=np.int64) - self.a
        return self._code_of(lw).astype(np.uint32).view(np.int32)

    def condense(self, answers):
        a = self.a
        e = self.esc[self.lsrc]
        ls, ld = self.lsrc[e], self.ldst[e]
        keep = ~self.esc[ld] | (self.rep[ld] != self.rep[ls])
        ls, ld = ls[keep], ld[keep]
        rec = [((a + self.rep[ls]).astype(np.uint64) << np.uint64(32)) |
               self._code_of(ld).astype(np.uint64)]
        ans = np.asarray(answers, dtype=np.int64) & 0xFFFFFFFF
        idx = np.searchsorted(self.q, self.cdst)
        rec.append(((a + self.rep[self.csrc]).astype(np.uint64) << np.uint64(32)) |
                   ans[idx].astype(np.uint64))
        edges = np.unique(np.concatenate(rec))
        sup = np.nonzero(self.esc & (self.rep == np.arange(self.V)))[0]
        mx = np.zeros(self.V, np.int64)
        np.maximum.at(mx, self.rep[self.esc], np.nonzero(self.esc)[0] + a)
        verts = np.zeros(2 * len(sup), dtype=np.uint64)
        verts[0::2] = ((a + sup).astype(np.uint64) << np.uint64(32)) | mx[sup].astype(np.uint64)
        verts[1::2] = self.lab[sup]
        return verts.view(np.int64), edges.view(np.int64)

    def solve(self, verts, edges):
        s, a, V = self.s, self.a, self.V
        vv = np.asarray(verts).view(np.uint64)
        ee = np.asarray(edges).view(np.uint64)
        sid = (vv[0::2] >> np.uint64(32)).astype(np.int64)
        maxpos = (vv[0::2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        tgt = (ee & np.uint64(0xFFFFFFFF)).astype(np.int64)
        mk = (tgt & MARKER) != 0
        keys = np.unique(np.concatenate([maxpos << 1, ((tgt[mk] & ~MARKER) << 1) | 1]))
        cv = len(keys)
        so = np.argsort(sid)
        sid_s = sid[so]
        vid_s = np.searchsorted(keys, maxpos[so] << 1)
        dotv = np.full(cv, np.iinfo(np.uint64).max, dtype=np.uint64)
        dotv[vid_s] = vv[1::2][so]
        es = vid_s[np.searchsorted(sid_s, (ee >> np.uint64(32)).astype(np.int64))]
        ed = np.where(mk, np.searchsorted(keys, ((tgt & ~MARKER) << 1) | 1),
                      vid_s[np.minimum(np.searchsorted(sid_s, tgt), len(sid_s) - 1)] if len(sid_s) else 0)
        rep, lab, Hk, depth = _scc_order(cv, es, ed, np.arange(cv), dotv)
        okey = np.zeros(V, dtype=np.int64)
        label = np.zeros(V, dtype=np.uint64)
        for v in range(V):
            if self.esc[v]:
                x = vid_s[np.searchsorted(sid_s, a + self.rep[v])]
                okey[v] = (int(keys[Hk[x]] >> 1) << 32) | 0x80000000 | int(depth[x])
                label[v] = lab[x]
            else:
                okey[v] = (int(self.H[v]) << 32) | int(self.depth[v])
                label[v] = self.lab[v]
        self.label = label
        # elements by key owner: e0 = key << hb | H, e1 = cd << 32 | dot32
        k = s.k
        keys_v = s.keys[a:a + V].astype(np.int64)
        owner = (keys_v % s.shards) % self.world
        d = s.dots[a:a + V]
        d32 = ((d >> np.uint64(56)) << np.uint64(self.seqb)) | (d & np.uint64((1 << 56) - 1))
        e0 = (keys_v.astype(np.uint64) << np.uint64(self.hb)) | (okey >> 32).astype(np.uint64)[:, None]
        e1 = ((okey & 0xFFFFFFFF).astype(np.uint64) << np.uint64(32))[:, None] | d32[:, None]
        e1 = np.broadcast_to(e1, e0.shape)
        o = np.argsort(owner.reshape(-1), kind="stable")
        el = np.zeros(2 * V * k, dtype=np.uint64)
        el[0::2] = e0.reshape(-1)[o]
        el[1::2] = e1.reshape(-1)[o]
        return np.bincount(owner.reshape(-1), minlength=self.world).astype(np.int64), el.view(np.int64)

    def per_key(self, elems):
        el = np.asarray(elems).view(np.uint64)
        e0, e1 = el[0::2], el[1::2]
        o = np.lexsort((e1, e0))
        self.pk_key = (e0[o] >> np.uint64(self.hb)).astype(np.uint32)
        d = e1[o] & np.uint64(0xFFFFFFFF)
        self.pk_dot = ((d >> np.uint64(self.seqb)) << np.uint64(56)) | (d & np.uint64((1 << self.seqb) - 1))

    def results(self, count):
        return {"dep_off": self.dep_off, "deps": self.deps, "scc_label": self.label,
                "pk_key": self.pk_key, "pk_dot": self.pk_dot,
                "escaping": int(self.esc.sum()), "cross_edges": int(len(self.csrc))}
