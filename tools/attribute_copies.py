#!/usr/bin/env python
"""attribute_copies.py -- where __amd_rocclr_copyBuffer time comes from in a
rocprofv3 --kernel-trace run of bench.py.

A run spans from its first kernel (--run-start, default k_view_records: the
command-level KeyDeps pass that opens every C4 run; k_log_keys for the
chunked path) to its last one
(--run-end, default k_key_offsets: the per-key offsets that close it).  A
copyBuffer dispatch inside a run is in-step: a copy the run itself makes
(graph_tile's pass-2 core list, H2D; the small read-backs are k_fetch_u32
kernels, not copies).  One outside every run is staging or read-back: the
stream's upload (fh_engine_stage_logs) and results() between the timed loop
and the probe pass -- never inside a timed region.  Prints a JSON summary.

Usage: python tools/attribute_copies.py <run_kernel_trace.csv>
"""
from __future__ import annotations

import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--run-start", default="k_view_records", help="the kernel that opens a run")
    ap.add_argument("--run-end", default="k_key_offsets", help="the kernel that closes a run")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3  # us
    out = {"outside_runs": {"calls": 0, "us": 0.0}, "in_step": {"calls": 0, "us": 0.0}}
    total = sum(dur(r) for r in rows)
    inside, runs, run_us = False, 0, 0.0
    for r in rows:
        name = r["Kernel_Name"]
        if not inside and a.run_start in name:
            inside = True
            runs += 1
        if inside:
            run_us += dur(r)
        if "copyBuffer" in name:
            k = "in_step" if inside else "outside_runs"
            out[k]["calls"] += 1
            out[k]["us"] += dur(r)
        if inside and a.run_end in name:
            inside = False
    out["runs"] = runs
    out["run_device_us"] = run_us
    out["device_us_total"] = total
    for k in ("outside_runs", "in_step"):
        out[k]["frac_of_device_time"] = out[k]["us"] / total
    out["in_step"]["frac_of_run_device_time"] = out["in_step"]["us"] / run_us
    if runs:
        out["in_step"]["us_per_run"] = out["in_step"]["us"] / runs
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
