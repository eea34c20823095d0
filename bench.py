#!/usr/bin/env python
"""bench.py -- commands ordered per second (deps+SCC+order) on MI355X.

Headline workload (BASELINE.json configs[3], "C4"): Atlas n=5 f=1 (fast quorum
3), 100M commands, Zipf s=0.99 over 2^20 keys, 1 key per command, replica
views (each replica's KeyDeps sees its commands in its own arrival order,
reorder window W=64).  One step orders the whole 100M-command stream from a
clean state, inputs resident in HBM:
  per-replica KeyDeps (sort by (replica, key) + previous element of each
  segment) -> QuorumDeps union -> dependency graph -> SCCs -> execution
  order -> per-key execution sequences,
and every output is materialised on the device inside the step: committed
deps as CSR of dots, SCC labels (min dot), execution ranks, per-key offsets
and per-key dot sequences (fh_engine_run).  Between steps fh_engine_rewind
clears the latest tables and executed clock on the engine stream.

Multi-GPU (`--gpus N`, one process per GPU under torch.distributed.run): the
stream is key-sharded by a work-balanced key map: every rank
counts the stream's commands per key, weights each key by its estimated cost
(a hot key's commands cost more: key_weights, measured on the 8 shards) and
packs keys largest-first onto the least loaded rank (fh_key_owners_balanced
over the weights; the same map on every rank).  With one key per
command every dependency joins two commands of one key, so a shard's graph is
closed: each rank orders its shard of the same global stream (global dots)
with no data-path collective; torch.distributed (RCCL) carries only the
barrier and the max-over-ranks time.  Total work is fixed: "scaling":
"strong", value = 100M x steps / max-over-ranks time.

The JSON line also carries the roofline of the dominant kernel (HIP events on
the engine stream around its launches in a probe pass), the CPU baseline (the
oracle restatement of the reference's per-replica SequentialKeyDeps +
QuorumDeps + incremental GraphExecutor on a bounded prefix, rank 0 at N=1)
and, as `secondary`, the C2 line (single-view KeyDeps, 1M-command batches).

`c5` (N=1, rank 0): BASELINE.json configs[4] at its stated size -- Atlas
partial replication over 8 key shards (shard = key mod 8), Zipf 0.99 over 2^20
keys, 4 keys per command, 100M commands -- with all 8 shards on the one GPU.
Shard h holds processes 5h+1..5h+5 (fantoch/src/util.rs:115-122); a command's
dot comes from its target shard (its first key's, id.rs:59-61) and every
shard it touches collects it with its own fast quorum and arrival order
(atlas.rs:214-328), so the 40 processes' KeyDeps each see only their shard's
keys of a command (element logs, FH_STREAM_ELEMENT_LOGS) and the committed
deps are the union over the shards (MShardCommit, atlas.rs:559-639).  Parity:
the committed-deps digest at 100M and every output on a 20k prefix equal the
oracle's shard-by-shard computation (tests/golden/make_digests.py,
tests/test_fullsize_gpu.py).

Roofline bytes are SURVEY.md §8(d)'s algorithmic bytes per command: the
dominant kernel's `achieved` = (its §8(d) term x commands per step) / (its
device time per step); the builder's own per-kernel byte counts ride along
as `*_builder` fields.  `cold_ms` = one run after fh_engine_forget_tuning
(the graph stage's learned reach bound / global-path entry dropped), and
`first_ms` = the first run of a fresh engine (buffer allocation included).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
METRIC = "commands ordered/sec (deps+SCC+order) at 1/2/4/8 GPUs; % HBM roofline"
C4_SEED = 0xFA170C4000000004
C2_SEED = 0xFA170C4000000002


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--commands", type=int, default=100_000_000, help="C4 stream length")
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=16_000_000,
                    help="C4 commands in the CPU-baseline prefix (~10 s of one host core)")
    ap.add_argument("--probe", default="sort_scatter,sort_scatter_dots,sort_scatter_v3,graph_tile,cmd_search,"
                    "view_records,cmd_pack,code_scatter,row_place,ko_final,"
                    "cmd_union,prev_bucket,place,log_keys",
                    help="kernels whose launches are timed in the probe pass")
    ap.add_argument("--no-phases", action="store_true", help="skip the per-phase profile pass")
    ap.add_argument("--no-secondary", action="store_true", help="skip the secondary C2 line")
    ap.add_argument("--no-streaming", action="store_true",
                    help="skip the small-batch executor line (tools/stream_bench)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other BASELINE configurations (C1, C3, C4 key shard, C5 12.5M)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 100M line")
    ap.add_argument("--c5-commands", type=int, default=100_000_000)
    ap.add_argument("--c5-steps", type=int, default=3)
    ap.add_argument("--one-gpu", action="store_true",
                    help="every rank on GPU 0 over gloo (a dry run of the N > 1 paths on a "
                         "one-GPU box; not a measurement)")
    ap.add_argument("--c5-backend", default="",
                    help="N > 1: exchange backend of the C5 leg (default: the process group's, "
                         "RCCL; gloo for a dry run of N ranks sharing one GPU)")
    ap.add_argument("--c5-solo", action="store_true",
                    help="dry runs: the C5 KeyDeps / local / condense / solve stages one rank at a "
                         "time, so their stage times are those of an unshared GPU (not a "
                         "throughput run)")
    ap.add_argument("--no-cpu-sharded", action="store_true",
                    help="skip the key-sharded multi-process CPU baseline")
    return ap.parse_args()


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/collect_pmc.py), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
            return json.load(fh).get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def c4_workload(keys):
    from fantoch_amd.workload import Workload
    return Workload.zipf(0.99, keys, k=1, views=3, window=64, seed=C4_SEED, n=5)


def cpu_baseline_c4(w, sample):
    """Oracle (C restatement of the reference CPU path: per-replica
    SequentialKeyDeps, QuorumDeps union, incremental GraphExecutor) on the
    first `sample` commands of the same stream, one thread; cmds/s."""
    from oracle import oracle as O
    s = w.generate(sample)
    key_off = s.key_off()
    keys = s.keys.reshape(-1)
    t0 = time.perf_counter()
    off, deps = O.views_run(0, 5, s.dots, key_off, keys, s.fq_proc, s.fq_time)
    ex, lab, kso, ks = O.graph_run(s.dots, key_off, keys, off, deps, s.key_space)
    dt = time.perf_counter() - t0
    assert len(ex) == s.n
    return s.n / dt, dt


def timed_steps(eng, steps, barrier, rewind=True):
    # eng.sync() = hipStreamSynchronize on the engine's stream: the library's
    # HIP runtime is not torch's, so torch.cuda.synchronize() would not wait
    # for the engine's kernels
    barrier()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        if rewind:
            eng.rewind()
        eng.run(sync=False)
    eng.sync()
    t1 = time.perf_counter()
    barrier()
    return t1 - t0


def probe_pass(eng, names, steps, rewind=True):
    import torch
    eng.set_probe(names)
    for _ in range(steps):
        if rewind:
            eng.rewind()
        eng.run(sync=False)
    eng.sync()
    probes = {}
    for name in [x for x in names.split(",") if x]:
        ms_, nl_, by_ = eng.probe_stats(name)
        if nl_:
            probes[name] = {"avg_launch_us": ms_ * 1e3, "launches": nl_,
                            "algorithmic_bytes_per_launch": by_,
                            "achieved_GBs": by_ / (ms_ * 1e-3) / 1e9 if ms_ > 0 else 0.0,
                            "traffic": pmc_traffic(name)}
    eng.set_probe(None)
    return probes


def sec8d_bytes(k, views, d, d_view=None):
    """SURVEY.md §8(d) algorithmic bytes per command, by term.  d_view: deps
    per command per view (<= k: the previous element of each key)."""
    dv = k if d_view is None else d_view
    b = {"deps": views * (8 * (1 + k) + 4 + 8 * dv),
         "union": (views * (4 + 8 * dv) + 4 + 8 * d) if views > 1 else 0.0,
         "exec": 4 + 4 * d + 8 + 4 + 4,
         "order": 8 + 8 * k}
    b["total"] = b["deps"] + b["union"] + b["exec"] + b["order"]
    return b


# the §8(d) term each probed kernel implements alone (the KeyDeps sort passes,
# the bucketing and the placement share B_deps between them: no single term)
SEC8D_TERM = {"graph_tile": "exec", "cmd_union": "union"}


def roofline(probes, fallback, commands, b8d, steps):
    if not probes:
        return {"bound": "hbm", "kernel": fallback, "achieved": 0.0, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": 0.0, "traffic": None}
    # dominant kernel: the most device time over the probe pass
    dom = max(probes, key=lambda k: probes[k]["avg_launch_us"] * probes[k]["launches"])
    p = probes[dom]
    per_step_s = p["avg_launch_us"] * 1e-6 * p["launches"] / steps
    term = SEC8D_TERM.get(dom)
    if dom == "graph_tile" and probes.get("ko_final", {}).get("launches"):
        # the key-order path: the tile kernel also writes the per-key
        # sequences, so it implements B_exec + B_order
        term = "exec+order"
    if term:
        per_cmd = sum(b8d[t] for t in term.split("+"))
        alg = per_cmd * commands  # bytes per step
        ach = alg / per_step_s / 1e9
        basis = f"SURVEY §8(d) B_{term} = {per_cmd:.2f} B/cmd x {commands} commands per step"
    else:
        alg = p["algorithmic_bytes_per_launch"] * p["launches"] / steps
        ach = p["achieved_GBs"]
        basis = "kernel's own algorithmic bytes (no single §8(d) term)"
    launches_per_step = p["launches"] / steps
    r = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": ach / HBM_PEAK_GBS, "traffic": p["traffic"], "launches": p["launches"],
         "launches_per_step": launches_per_step, "avg_launch_us": p["avg_launch_us"],
         "kernel_ms_per_step": per_step_s * 1e3,
         "algorithmic_bytes_per_step": alg,
         "algorithmic_bytes_per_launch": alg / launches_per_step, "basis": basis,
         "achieved_builder": p["achieved_GBs"],
         "frac_builder": p["achieved_GBs"] / HBM_PEAK_GBS,
         "algorithmic_bytes_per_launch_builder": p["algorithmic_bytes_per_launch"]}
    if p["traffic"] is not None:
        r["traffic_per_step"] = p["traffic"] * launches_per_step
    return r


def phases_of(eng, rewind=True):
    eng.set_profiling(True)
    acc = {}
    for _ in range(3):
        if rewind:
            eng.rewind()
        eng.run(sync=True)
        for name, ms in eng.kernel_times():
            acc.setdefault(name, []).append(ms)
    eng.set_profiling(False)
    return {k: round(float(np.median(v[1:] if len(v) > 1 else v)), 4) for k, v in acc.items()}


def path_roofline(value, k, views, d, world=1):
    b = sec8d_bytes(k, views, d)
    ach = value * b["total"] / 1e9 / world
    return {"bytes_per_cmd": b["total"], "terms": {t: b[t] for t in ("deps", "union", "exec", "order")},
            "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS}


def time_engine(s, local, steps):
    """One engine over the staged stream s: ms per step (rewind + run, after
    one warmup run), inputs resident, every output materialised."""
    from fantoch_amd.engine import Engine
    eng = Engine(s.key_space, n=5, device=local)
    eng.stage(s)
    eng.run(sync=True)  # warmup (also picks the graph path's entry)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.rewind()
        eng.run(sync=False)
    eng.sync()
    ms = (time.perf_counter() - t0) / steps * 1e3
    d = eng.dep_total() / s.n
    eng.close()
    v = s.n / (ms * 1e-3)
    return {"commands": int(s.n), "ms_per_step": round(ms, 3), "commands_per_s": v,
            "deps_per_cmd": d, "path_roofline": path_roofline(v, s.k, 3, d)}


def other_configs(local, steps=3):
    """The other BASELINE configurations on this GPU, each one engine pass over
    its whole staged stream per step (inputs resident, every output
    materialised): C1 (10k, plumbing), C3 (10M, one stream-wide SCC), C4's
    per-GPU key-shard size (12.5M) and the first 12.5M commands of C5's 4-key
    stream, unsharded.  Parity at these shapes: tests/test_fullsize_gpu.py."""
    from fantoch_amd.workload import Workload
    cfgs = {
        "c1": (Workload.conflict_rate_(10, k=1, views=3, window=64, seed=0xFA170C4000000001, n=5),
               10_000, "Atlas n=5 f=1, ConflictRate 10%, 1 key, replica views"),
        "c3": (Workload.conflict_pool(100, 16, k=2, views=3, window=64, seed=0xFA170C4000000003,
                                      n=5), 10_000_000,
               "EPaxos n=5, ConflictPool 100% (key 0 + 16-key pool), 2 keys, replica views"),
        "c4_shard": (Workload.zipf(0.99, 1 << 20, k=1, views=3, window=64, seed=C4_SEED, n=5),
                     12_500_000, "C4's critical key shard at 8 GPUs (work-weighted key map, "
                                 "global dots): Zipf 0.99 / 2^20 keys, 1 key"),
        "c5_12m": (Workload.zipf(0.99, 1 << 20, k=4, views=3, window=64,
                                 seed=0xFA170C4000000005, n=5), 12_500_000,
                   "first 12.5M commands of C5's stream, unsharded: Zipf 0.99 / 2^20 keys, "
                   "4 keys/cmd, replica views"),
    }
    out = {}
    for name, (w, n, desc) in cfgs.items():
        if name == "c4_shard":
            # the critical shard of the 100M stream over 8 GPUs under the
            # work-weighted key map (what rank q of bench.py --gpus 8
            # orders): of the shard holding the hottest key and the shard
            # with the most commands, the slower one (timed below)
            from fantoch_amd.workload import key_owners_weighted
            h = w.key_histogram(100_000_000)
            owner = key_owners_weighted(h, 8)
            loads = np.bincount(owner, weights=h.astype(np.float64), minlength=8)
            cands = sorted({int(owner[int(np.argmax(h))]), int(np.argmax(loads))})
            best = None
            for q in cands:
                s = w.generate_shard(100_000_000, 8, q, owner=owner)
                r = time_engine(s, local, steps)
                r["shard"] = q
                if best is None or r["ms_per_step"] > best["ms_per_step"]:
                    best = r
                del s
            best["workload"] = desc
            best["shards_timed"] = cands
            out[name] = best
            continue
        s = w.generate(n, logs=True, times=False)
        out[name] = time_engine(s, local, steps)
        out[name]["workload"] = desc
    return out


def c5_workload():
    from fantoch_amd.workload import Workload
    return Workload.zipf(0.99, 1 << 20, k=4, views=3, window=64, seed=0xFA170C4000000005, n=5,
                         shards=8)


def c5_line(args, local):
    """C5 at its stated size on one GPU (all 8 key shards, 40 processes): one
    engine pass over the 100M-command partially replicated stream per step,
    every output materialised."""
    from fantoch_amd.engine import Engine
    n = args.c5_commands
    t_gen = time.perf_counter()
    s = c5_workload().generate(n, logs=True, times=False)
    t_gen = time.perf_counter() - t_gen
    eng = Engine(s.key_space, n=5, device=local)
    eng.stage(s)
    first = eng.run(sync=True)
    steps = 3
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.rewind()
        eng.run(sync=False)
    eng.sync()
    ms = (time.perf_counter() - t0) / steps * 1e3
    d = eng.dep_total() / n
    r_out = eng.results()
    _, scc_sizes = np.unique(r_out["scc_label"], return_counts=True)
    del r_out
    eng.forget_tuning()
    eng.rewind()
    cold = eng.run(sync=True)
    phases = None
    if not args.no_phases:
        eng.set_profiling(True)
        eng.rewind()
        eng.run(sync=True)
        phases = {k: round(v, 3) for k, v in eng.kernel_times()}
        eng.set_profiling(False)
    eng.close()
    v = n / (ms * 1e-3)
    r = {"workload": "C5: Atlas partial replication, 8 key shards (key mod 8; shard h = processes "
                     "5h+1..5h+5, dots from the target shard, every shard its own collect and "
                     "arrival order), all on this GPU; Zipf 0.99 over 2^20 keys, 4 keys/cmd, fast "
                     "quorum 3, 100M commands; one step orders the whole stream, every output "
                     "materialised",
         "commands": n, "shards": 8, "processes": 40, "steps": steps, "warmup": 1,
         "ms_per_step": round(ms, 3), "commands_per_s": v, "first_ms": round(first, 3),
         "cold_ms": round(cold, 3), "deps_per_cmd": d, "sccs": int(len(scc_sizes)),
         "largest_scc": int(scc_sizes.max()), "generate_s": round(t_gen, 2),
         "path_roofline": path_roofline(v, 4, 3, d)}
    if phases:
        r["phases_ms"] = phases
    return r


def condensed_degrees(eg):
    """Out-degree profile of the condensed graph's edge records (src << 32 |
    target), for the solo measurement runs; {} otherwise."""
    if eg is None or len(eg) == 0:
        return {}
    e = eg.cpu().numpy() if hasattr(eg, "cpu") else np.asarray(eg)
    _, deg = np.unique((e.astype(np.uint64) >> np.uint64(32)), return_counts=True)
    deg = np.sort(deg)[::-1]
    return {"max_out_degree": int(deg[0]), "top8_out_degrees": [int(x) for x in deg[:8]],
            "sources": int(len(deg))}


def c5_dist_line(args, rank, world, local, group):
    """C5 across GPUs: fantoch_amd.dgraph.DistPartial -- KeyDeps by key shard
    (shard h on rank h % N), the per-command union and local SCCs by stream-
    position range, cross-range queries / answers, the condensed graph
    all-gathered and solved on every rank, per-key sequences at the keys'
    owners; exchanges over `group` (RCCL, or gloo for a dry run of N ranks
    sharing one GPU).  value = 100M x steps / max-over-ranks time."""
    import torch
    import torch.distributed as dist
    from fantoch_amd.dgraph import DistPartial
    n = args.c5_commands
    t_gen = time.perf_counter()
    s = c5_workload().generate(n, logs=True, times=False)
    t_gen = time.perf_counter() - t_gen
    p = DistPartial(rank, world, s.key_space, group=group, device=local,
                    solo=args.c5_solo)
    t_stage = time.perf_counter()
    p.stage(s)
    t_stage = time.perf_counter() - t_stage
    del s
    p.run()  # warmup
    steps = args.c5_steps
    dist.barrier(group=group)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        p.run()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    dist.barrier(group=group)
    t = torch.tensor([el], dtype=torch.float64)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    el = float(t.item())
    p.stages.set_profiling(True)
    p.run()
    stage_ms = p.stages.stage_times()
    p.stages.set_profiling(False)
    p.stages.close()
    v = n * steps / el
    return {"workload": "C5 across GPUs: Atlas partial replication, 8 key shards (key mod 8; shard "
                        "h = processes 5h+1..5h+5 on rank h % N), Zipf 0.99 over 2^20 keys, 4 "
                        "keys/cmd, fast quorum 3, 100M commands; every step orders the whole "
                        "stream (committed deps, SCC labels, per-key sequences)",
            "commands": n, "n_gpus": world, "steps": steps, "warmup": 1,
            "ms_per_step": round(el / steps * 1e3, 3), "commands_per_s": v, "scaling": "strong",
            "parallelism": f"KeyDeps by key shard x{world}; union + SCC by stream range x{world}",
            "backend": dist.get_backend(group), "generate_s": round(t_gen, 2),
            "stage_s": round(t_stage, 2), "rank0_stage_ms": stage_ms,
            # the graph every rank solves in step 4 (replicated work)
            "condensed_graph": {"super_vertices": int(p.condensed[0]),
                                "edges": int(p.condensed[1]),
                                **condensed_degrees(p.condensed_eg)},
            "solo_stages": bool(args.c5_solo)}


def streaming_line():
    """The executor drop-in at small batches (tools/stream_bench.cpp, built by
    tools/build_tools.sh): a C4-shaped committed stream fed to one fh_graph
    in stream order, `batch` Adds per call, drained after every call --
    GraphExecutor::handle + fetch_actions (executor.rs:76-145) as the runners
    call them (run/task/executor.rs:150-175); host arrays in and out, PCIe
    included.  None if the tool is not built."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "stream_bench")
    if not os.path.exists(exe):
        return None
    p = subprocess.run([exe, "1", "20000", "10", "100000", "1000", "2000000", "1000000",
                        "10000000"], capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        return {"error": p.stderr[-400:]}
    return [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]


def cpu_sharded_worker(arg):
    keys, nsh, sh, sample = arg
    import numpy as np
    from oracle import oracle as O
    from fantoch_amd.workload import key_owners_balanced
    w = c4_workload(keys)
    s = w.generate(sample)
    owner = key_owners_balanced(w.key_histogram(sample), nsh)
    mine = np.nonzero(owner[s.keys[:, 0]] == sh)[0]
    dots, kk = s.dots[mine], s.keys[mine].reshape(-1)
    ko = (np.arange(len(mine) + 1, dtype=np.uint64)).astype(np.uint32)
    fp, ft = s.fq_proc[mine], s.fq_time[mine]
    t0 = time.perf_counter()
    off, deps = O.views_run(0, 5, dots, ko, kk, fp, ft)
    O.graph_run(dots, ko, kk, off, deps, s.key_space)
    return len(mine), time.perf_counter() - t0


def cpu_baseline_sharded(keys, sample, procs):
    """The oracle on `procs` key shards of the same prefix (balanced key map,
    as on the GPUs) in parallel processes (one key per command: every shard's
    graph is closed): whole-prefix commands / the slowest shard's time."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(cpu_sharded_worker, [(keys, procs, i, sample) for i in range(procs)])
    slow = max(t for _, t in res)
    return sum(n for n, _ in res) / slow, slow


def secondary_c2(args, local):
    """C2: single-view KeyDeps + GraphExecutor, Zipf 0.7 over 1M keys, 1M-command
    batches of one continuing stream (state carried across batches)."""
    import torch
    from fantoch_amd.engine import Engine
    from fantoch_amd.workload import Workload
    batch, steps, warm = 1_000_000, 20, 5
    w = Workload.zipf(0.7, 1 << 20, k=1, seed=C2_SEED, n=5)
    s = w.generate(batch * (warm + steps))
    eng = Engine(s.key_space, n=5, device=local)
    from fantoch_amd.workload import Stream
    eng.stage_many([Stream(s.dots[i * batch:(i + 1) * batch], s.keys[i * batch:(i + 1) * batch],
                           None, None, s.key_space) for i in range(warm + steps)])
    for _ in range(warm):
        eng.run(sync=False)
    eng.sync()
    el = timed_steps(eng, steps, lambda: None, rewind=False)
    r = eng.results()
    eng.close()
    v = batch * steps / el
    d = int(r["dep_off"][-1]) / batch
    return {"metric": METRIC, "value": v, "unit": "commands/s",
            "path_roofline": path_roofline(v, 1, 1, d),
            "ms_per_step": el / steps * 1e3, "steps": steps, "warmup": warm,
            "config": {"workload": "C2: Zipf s=0.7 over 2^20 keys, 1 key/cmd, single replica view, "
                                   "1M-command batches of one stream, every output materialised",
                       "batch": batch},
            "deps_last_batch": int(r["dep_off"][-1])}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch
    if args.one_gpu:  # a dry run of N ranks on one GPU (gloo): the box has one
        local = 0
    if world > 1 or "RANK" in os.environ:
        import torch.distributed as dist_mod
        dist = dist_mod
        torch.cuda.set_device(local)
        if args.one_gpu:
            dist.init_process_group(backend="gloo")
        else:
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    from fantoch_amd.engine import Engine

    def barrier():
        if dist is not None:
            dist.barrier()

    w = c4_workload(args.keys)
    t_gen = time.perf_counter()
    owner = None
    if world == 1:
        s = w.generate(args.commands, logs=True, times=False)
    else:
        from fantoch_amd.workload import key_owners_weighted
        owner = key_owners_weighted(w.key_histogram(args.commands), world)
        s = w.generate_shard(args.commands, world, rank, owner=owner)
    t_gen = time.perf_counter() - t_gen
    eng = Engine(s.key_space, n=5, device=local)
    t_stage = time.perf_counter()
    eng.stage(s)
    eng.sync()
    t_stage = time.perf_counter() - t_stage
    first_ms = None
    for i in range(args.warmup):
        if i == 0:
            eng.rewind()
            first_ms = eng.run(sync=True)
            continue
        eng.rewind()
        eng.run(sync=False)
    eng.sync()
    elapsed = timed_steps(eng, args.steps, barrier)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cpu" if args.one_gpu else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = args.commands * args.steps / elapsed

    # outputs of the last run (read back outside the timed region)
    t_res = time.perf_counter()
    r = eng.results()
    t_res = time.perf_counter() - t_res
    n_local = s.n
    deps_total = int(r["dep_off"][-1])
    _, scc_sizes = np.unique(r["scc_label"], return_counts=True)
    probe_steps = min(args.steps, 10)
    probes = probe_pass(eng, args.probe, probe_steps)
    phases = None if (args.no_phases or rank != 0) else phases_of(eng)
    # cold run: the graph stage's learned tuning dropped (fresh-engine guesses)
    eng.forget_tuning()
    eng.rewind()
    cold_ms = eng.run(sync=True)
    eng.close()

    rank_commands = [n_local]
    if dist is not None:
        rank_commands = [None] * world
        dist.all_gather_object(rank_commands, int(n_local))
    d = deps_total / max(1, n_local)
    k, views = 1, 3
    b8d = sec8d_bytes(k, views, d)
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "commands/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": "C4: Atlas n=5 f=1 (fast quorum 3) replica views, 100M commands, "
                               "Zipf s=0.99 over 2^20 keys, 1 key/cmd, reorder window 64; one step "
                               "orders the whole stream, every output materialised on the device",
                   "commands": args.commands, "keys": args.keys, "zipf_s": 0.99, "views": views,
                   "parallelism": f"key-shard x{world}"},
        "roofline": roofline(probes, "sort_scatter", n_local, b8d, probe_steps),
        "kernels": probes,
        "path_roofline": path_roofline(value, k, views, d, world),
        "cold_ms": round(cold_ms, 3),
        "first_ms": round(first_ms, 3) if first_ms is not None else None,
        "stream": {"commands_this_rank": n_local, "commands_per_rank": rank_commands,
                   "partition": ("work-weighted key map (key_weights + fh_key_owners_balanced)"
                                 if world > 1
                                 else "whole stream"),
                   "deps_per_cmd": d, "sccs": int(len(scc_sizes)),
                   "largest_scc": int(scc_sizes.max()) if len(scc_sizes) else 0,
                   "generate_s": round(t_gen, 2)},
        # the same step with its PCIe legs -- the stream
        # staged from host memory (dots, keys, replica logs: H2D plus the
        # staging pass) and every output read back (D2H) -- measured once
        # each, outside the timed loop; not the metric
        "pcie_inclusive": {
            "stage_h2d_ms": round(t_stage * 1e3, 3),
            "results_d2h_ms": round(t_res * 1e3, 3),
            "ms": round(t_stage * 1e3 + elapsed / args.steps * 1e3 + t_res * 1e3, 3),
            "commands_per_s": n_local / (t_stage + elapsed / args.steps + t_res)},
    }
    if phases is not None:
        result["phases_ms"] = phases
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sample = min(args.cpu_sample, args.commands)
        v, dt = cpu_baseline_c4(w, sample)
        try:
            host = len(os.sched_getaffinity(0))
        except AttributeError:
            host = os.cpu_count()
        result["cpu_baseline"] = {"value": v, "unit": "commands/s", "cores": 1, "kind": "port",
                                  "host_nproc": os.cpu_count(), "host_cpus_usable": host,
                                  "sample": f"first {sample} commands of the same C4 stream: oracle "
                                            f"per-replica SequentialKeyDeps + QuorumDeps union + "
                                            f"incremental GraphExecutor, 1 thread, {dt:.2f}s"}
        if not args.no_cpu_sharded:
            procs = 16  # the GPU box's CPU share for one GPU
            vs, ts = cpu_baseline_sharded(args.keys, sample, procs)
            result["cpu_baseline_sharded"] = {
                "value": vs, "unit": "commands/s", "cores": procs, "kind": "port",
                "sample": f"the same {sample}-command prefix split into {procs} key shards "
                          f"(balanced key map), one oracle process per shard; slowest shard "
                          f"{ts:.2f}s"}
    if rank == 0 and world == 1 and not args.no_c5:
        result["c5"] = c5_line(args, local)
    if world > 1 and not args.no_c5:
        grp = dist.new_group(backend=args.c5_backend) if args.c5_backend else dist.group.WORLD
        result["c5"] = c5_dist_line(args, rank, world, local, grp)
    if rank == 0 and world == 1 and not args.no_secondary:
        result["secondary"] = secondary_c2(args, local)
    if rank == 0 and world == 1 and not args.no_streaming:
        result["streaming"] = streaming_line()
    if rank == 0 and world == 1 and not args.no_configs:
        result["configs"] = other_configs(local)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
