#!/usr/bin/env python
"""bench.py -- commands ordered per second (deps + SCC + order) on MI355X.

Workload (BASELINE.json configs[1], "C2"): Zipf s=0.7 over 1M keys, 1 key per
command, one replica view, batches of 1M commands.  A step is one pass of the
fused engine over the next batch of the committed stream (inputs resident in
HBM, KeyDeps / executed-clock state carried from the previous batch): radix
sort -> per-key predecessor deps -> dependency graph certified acyclic ->
execution order -> per-key execution sequence -> executed-clock advance.

Multi-GPU (`--gpus N`, one process per GPU under torch.distributed.run): the
stream is key-sharded (owner = key mod N); with one key per
command a shard's commands depend only on that shard, so there is no data-path
collective (weak scaling: every rank orders ~1M commands per step).  Each
shard sequences its own dots, as fantoch's per-shard DotGen does
(fantoch/src/util.rs:115-122).

Output: one JSON line (rank 0) with the metric, the roofline of the dominant
kernel (HIP events around it inside the timed steps) and the CPU baseline
(the oracle restatement of SequentialKeyDeps + GraphExecutor on a bounded
sample, rank 0 at N=1 only).
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--zipf", type=float, default=0.7)
    ap.add_argument("--seed", type=int, default=0xFA170C4000000002)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=40_000_000,
                    help="commands in the CPU-baseline sample (~10 s of one host core)")
    ap.add_argument("--probe", default="kb_step,kb_partition,kb_order",
                    help="kernels whose launches are timed (comma-separated); the roofline "
                         "entry reports the one with the most device time")
    ap.add_argument("--no-phases", action="store_true", help="skip the per-phase profile pass")
    return ap.parse_args()


def shard_batches(args, rank, world, nbatches):
    """The rank's key shard of the global C2 stream (fantoch_amd/shard.py)."""
    from fantoch_amd.shard import shard_batches as sb
    from fantoch_amd.workload import Workload
    w = Workload.zipf(args.zipf, args.keys, k=1, seed=args.seed, n=5)
    return sb(w, rank, world, args.batch, nbatches)


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by tools/collect_pmc.py from
    separate FETCH_SIZE / WRITE_SIZE passes of this same command), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            return json.load(fh).get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(batch_stream, sample):
    """Oracle (C restatement of the reference CPU path) on `sample` commands,
    single-threaded; returns cmds/s."""
    from oracle import oracle as O
    from fantoch_amd.workload import Workload
    s = batch_stream
    dots, keys = s.dots[:sample], s.keys[:sample].reshape(-1)
    key_off = np.arange(len(dots) + 1, dtype=np.uint32)
    t0 = time.perf_counter()
    dep_off, deps = O.keydeps_run(dots, key_off, keys)
    ex, lab, kso, ks = O.graph_run(dots, key_off, keys, dep_off, deps, s.key_space)
    dt = time.perf_counter() - t0
    assert len(ex) == len(dots)
    return len(dots) / dt, dt


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or "RANK" in os.environ:
        import torch
        import torch.distributed as dist_mod
        dist = dist_mod
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl")
    import torch

    from fantoch_amd.engine import Engine

    # warmup + the timed steps + a probe pass of the same length (per-launch
    # HIP events cost ~3 us of stream time each, so they stay out of the
    # timed region)
    nb = args.warmup + 2 * args.steps
    batches = shard_batches(args, rank, world, nb)
    key_space = batches[0].key_space
    eng = Engine(key_space, n=5, device=local)
    eng.stage_many(batches)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        eng.run(sync=False)
    torch.cuda.synchronize()

    # timed region: exactly `steps` batches, no instrumentation
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run(sync=False)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    # probe pass: the next `steps` batches with HIP events on the stream of
    # every launch of the probed kernels (their own dispatch begin/end)
    eng.set_probe(args.probe)
    for _ in range(args.steps):
        eng.run(sync=False)
    torch.cuda.synchronize()
    probes = {}
    for name in [x for x in args.probe.split(",") if x]:
        ms_, nl_, by_ = eng.probe_stats(name)
        if nl_:
            probes[name] = {"avg_launch_us": ms_ * 1e3, "launches": nl_,
                            "algorithmic_bytes_per_launch": by_,
                            "achieved_GBs": by_ / (ms_ * 1e-3) / 1e9 if ms_ > 0 else 0.0}
    eng.set_probe(None)
    # dominant kernel: most device time over the pass (average x launches)
    dominant = (max(probes, key=lambda k: probes[k]["avg_launch_us"] * probes[k]["launches"])
                if probes else args.probe)
    pd = probes.get(dominant, {"avg_launch_us": 0.0, "launches": 0,
                               "algorithmic_bytes_per_launch": 0.0})
    probe_ms, probe_launches = pd["avg_launch_us"] * 1e-3, pd["launches"]
    probe_bytes = pd["algorithmic_bytes_per_launch"]
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_cmds = args.batch * args.steps * world
    value = total_cmds / elapsed

    # per-phase device times (separate profiled pass over a re-staged batch)
    phases = None
    if rank == 0 and not args.no_phases:
        eng2 = Engine(key_space, n=5, device=local)
        eng2.stage_many(batches[:4])
        eng2.set_profiling(True)
        acc = {}
        for _ in range(4):
            eng2.run(sync=True)
            for name, ms in eng2.kernel_times():
                acc.setdefault(name, []).append(ms)
        phases = {k: float(np.median(v[1:])) for k, v in acc.items()}
        eng2.close()

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "commands/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": "C2: batched KeyDeps+GraphExecutor, Zipf s=0.7 over 1M keys, "
                               "1 key/cmd, single replica view, 1M-command batches per GPU, "
                               "key-sharded across GPUs",
                   "batch_per_gpu": args.batch, "keys": args.keys, "zipf_s": args.zipf,
                   "parallelism": f"key-shard x{world}"},
    }
    achieved = probe_bytes / (probe_ms * 1e-3) / 1e9 if probe_ms > 0 else 0.0
    result["roofline"] = {"bound": "hbm", "kernel": dominant, "achieved": achieved,
                          "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                          "traffic": pmc_traffic(dominant), "launches": probe_launches,
                          "avg_launch_us": probe_ms * 1e3,
                          "algorithmic_bytes_per_launch": probe_bytes}
    for name, pr in probes.items():
        pr["traffic"] = pmc_traffic(name)
    result["kernels"] = probes
    # whole path against SURVEY §8d's 68 B/command (single view, k = 1)
    result["path_roofline"] = {"bytes_per_cmd": 68.0,
                               "achieved_GBs": value * 68.0 / 1e9 / world,
                               "frac": value * 68.0 / 1e9 / world / HBM_PEAK_GBS}
    if phases is not None:
        result["phases_ms"] = phases
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sample = min(args.cpu_sample, args.batch * nb)
        big = batches[0]
        if sample > big.n:
            from fantoch_amd.workload import Stream
            big = Stream(np.concatenate([b.dots for b in batches]),
                         np.concatenate([b.keys for b in batches]), None, None, key_space)
        v, dt = cpu_baseline(big, sample)
        result["cpu_baseline"] = {"value": v, "unit": "commands/s", "cores": 1, "kind": "port",
                                  "sample": f"first {sample} commands of the same C2 stream, "
                                            f"oracle SequentialKeyDeps + incremental "
                                            f"GraphExecutor, 1 thread, {dt:.2f}s"}
    if rank == 0:
        print(json.dumps(result))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
