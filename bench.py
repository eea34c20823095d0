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
stream is key-sharded (owner = key mod N).  With one key per
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
    ap.add_argument("--probe", default="sort_scatter,sort_scatter_dots,graph_tile,prev_bucket,place,cmd_union,log_keys",
                    help="kernels whose launches are timed in the probe pass")
    ap.add_argument("--no-phases", action="store_true", help="skip the per-phase profile pass")
    ap.add_argument("--no-secondary", action="store_true", help="skip the secondary C2 line")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other BASELINE configurations (C1, C3, C4 key shard, C5 shard)")
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


def roofline(probes, fallback):
    if not probes:
        return {"bound": "hbm", "kernel": fallback, "achieved": 0.0, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": 0.0, "traffic": None}
    # dominant kernel: the most device time over the pass
    dom = max(probes, key=lambda k: probes[k]["avg_launch_us"] * probes[k]["launches"])
    p = probes[dom]
    ach = p["achieved_GBs"]
    return {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "traffic": p["traffic"], "launches": p["launches"],
            "avg_launch_us": p["avg_launch_us"],
            "algorithmic_bytes_per_launch": p["algorithmic_bytes_per_launch"]}


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


def other_configs(local, steps=3):
    """The other BASELINE configurations on this GPU, each one engine pass over
    its whole staged stream per step (inputs resident, every output
    materialised): C1 (10k, plumbing), C3 (10M, one stream-wide SCC), C4's
    per-GPU key-shard size (12.5M) and a C5 shard (12.5M commands of 4 keys).
    Parity at these shapes: tests/test_fullsize_gpu.py."""
    from fantoch_amd.engine import Engine
    from fantoch_amd.workload import Workload
    cfgs = {
        "c1": (Workload.conflict_rate_(10, k=1, views=3, window=64, seed=0xFA170C4000000001, n=5),
               10_000, "Atlas n=5 f=1, ConflictRate 10%, 1 key, replica views"),
        "c3": (Workload.conflict_pool(100, 16, k=2, views=3, window=64, seed=0xFA170C4000000003,
                                      n=5), 10_000_000,
               "EPaxos n=5, ConflictPool 100% (key 0 + 16-key pool), 2 keys, replica views"),
        "c4_shard": (Workload.zipf(0.99, 1 << 20, k=1, views=3, window=64, seed=C4_SEED, n=5),
                     12_500_000, "C4 per-GPU size at 8 GPUs: Zipf 0.99 / 2^20 keys, 1 key"),
        "c5_shard": (Workload.zipf(0.99, 1 << 20, k=4, views=3, window=64,
                                   seed=0xFA170C4000000005, n=5), 12_500_000,
                     "C5 shard: Zipf 0.99 / 2^20 keys, 4 keys/cmd, replica views"),
    }
    out = {}
    for name, (w, n, desc) in cfgs.items():
        s = w.generate(n, logs=True, times=False)
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
        eng.close()
        out[name] = {"workload": desc, "commands": n, "ms_per_step": round(ms, 3),
                     "commands_per_s": n / (ms * 1e-3)}
    return out


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
    return {"metric": METRIC, "value": batch * steps / el, "unit": "commands/s",
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
    if world > 1 or "RANK" in os.environ:
        import torch.distributed as dist_mod
        dist = dist_mod
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    from fantoch_amd.engine import Engine

    def barrier():
        if dist is not None:
            dist.barrier()

    w = c4_workload(args.keys)
    t_gen = time.perf_counter()
    if world == 1:
        s = w.generate(args.commands, logs=True, times=False)
    else:
        s = w.generate_shard(args.commands, world, rank)
    t_gen = time.perf_counter() - t_gen
    eng = Engine(s.key_space, n=5, device=local)
    eng.stage(s)
    for _ in range(args.warmup):
        eng.rewind()
        eng.run(sync=False)
    eng.sync()
    elapsed = timed_steps(eng, args.steps, barrier)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = args.commands * args.steps / elapsed

    # outputs of the last run (read back outside the timed region)
    r = eng.results()
    n_local = s.n
    deps_total = int(r["dep_off"][-1])
    _, scc_sizes = np.unique(r["scc_label"], return_counts=True)
    probes = probe_pass(eng, args.probe, min(args.steps, 10))
    phases = None if (args.no_phases or rank != 0) else phases_of(eng)
    eng.close()

    d = deps_total / max(1, n_local)
    k, views = 1, 3
    # SURVEY §8d algorithmic bytes per command with replica views: KeyDeps per
    # view (read dot + key ids, write offset + deps; d_v <= k), the union of
    # the views' reports into d committed deps, the executor (CSR as vertex
    # ids, dot for the tie-break, SCC id + exec rank) and the per-key order.
    b_deps = views * (8 * (1 + k) + 4 + 8 * k)
    b_union = views * (4 + 8 * k) + 4 + 8 * d
    b_exec = 4 + 4 * d + 8 + 4 + 4
    b_order = 8 + 8 * k
    bpc = b_deps + b_union + b_exec + b_order
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
        "roofline": roofline(probes, "sort_scatter"),
        "kernels": probes,
        "path_roofline": {"bytes_per_cmd": bpc,
                          "achieved_GBs": value * bpc / 1e9 / world,
                          "frac": value * bpc / 1e9 / world / HBM_PEAK_GBS},
        "stream": {"commands_this_rank": n_local, "deps_per_cmd": d, "sccs": int(len(scc_sizes)),
                   "largest_scc": int(scc_sizes.max()) if len(scc_sizes) else 0,
                   "generate_s": round(t_gen, 2)},
    }
    if phases is not None:
        result["phases_ms"] = phases
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sample = min(args.cpu_sample, args.commands)
        v, dt = cpu_baseline_c4(w, sample)
        result["cpu_baseline"] = {"value": v, "unit": "commands/s", "cores": 1, "kind": "port",
                                  "sample": f"first {sample} commands of the same C4 stream: oracle "
                                            f"per-replica SequentialKeyDeps + QuorumDeps union + "
                                            f"incremental GraphExecutor, 1 thread, {dt:.2f}s"}
    if rank == 0 and world == 1 and not args.no_secondary:
        result["secondary"] = secondary_c2(args, local)
    if rank == 0 and world == 1 and not args.no_configs:
        result["configs"] = other_configs(local)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
