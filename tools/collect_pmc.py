#!/usr/bin/env python
"""collect_pmc.py -- HBM traffic per launch from rocprofv3 PMC passes.

Reads the counter CSVs of four separate `rocprofv3 --pmc` runs (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950, MI355X_MICROARCH.md §rocprofv3 PMC
slots):

  <root>/fetch        rocprofv3 --pmc FETCH_SIZE  -- python3 bench.py ...
  <root>/write        rocprofv3 --pmc WRITE_SIZE  -- python3 bench.py ...
  <root>/calib_fetch  rocprofv3 --pmc FETCH_SIZE  -- tools/pmc_calib
  <root>/calib_write  rocprofv3 --pmc WRITE_SIZE  -- tools/pmc_calib

FETCH_SIZE / WRITE_SIZE are in KiB.  FETCH_SIZE under-reports reads on gfx950
(½ for 16-B/lane streams; other widths uncalibrated, §HBM), so the
calibration kernels stream exactly 1 GiB at 4/8/16 B per lane and the
per-width factor counter/true is measured on the same box.  The engine's
kernels read and write 4-B-per-lane streams, so their raw bytes are divided
by the 4-B factors.

Writes profiles/pmc_traffic.json: {probe: {"hbm_bytes_per_launch": ...}, ...},
which bench.py reports as roofline.traffic.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

# probe name (fh_engine_set_probe) -> kernel-name pattern
PROBES = {
    # k_down<K, VT, DB, Src>: u32 or u64 values, any digit width (the balanced
    # 7 / 7 / 6-bit plan of 20-bit keys)
    "sort_scatter": r"k_down<unsigned int, unsigned int,",
    "sort_scatter_dots": r"k_down<unsigned int, unsigned long,",
    "sort_scatter_u64": r"k_down<unsigned long, unsigned int,",
    # the key-order path (round 5): V3 values, pass 0 reading through PackSrc
    "sort_scatter_v3": r"k_down<unsigned int, fh::(anonymous namespace)::V3, 7, fh::(anonymous namespace)::ArraySrc",
    "sort_scatter_v3_pack": r"k_down<unsigned int, fh::(anonymous namespace)::V3, 7, fh::(anonymous namespace)::PackSrc",
    "code_scatter": r"k_code_scatter<",
    "region_count": r"k_region_count<",
    "row_count": r"k_row_count<",
    "row_union": r"k_row_union<",
    "row_place": r"k_row_place<",
    "sv_rows": r"k_sv_rows",
    "run_place": r"k_run_place",
    "ko_final": r"k_ko_final",
    "key_counts": r"k_key_counts",
    "sort_up": r"k_up<",
    "graph_tile": r"k_graph_tile<",
    "prev_bucket": r"k_bucket_codes",
    "place": r"k_place",
    "cmd_union": r"k_cmd_engine<unsigned int>",
    "cmd_count": r"k_cmd_count<unsigned int>",
    "cmd_search": r"k_cmd_search<",
    "view_records": r"k_view_records<",
    "cmd_pack": r"k_cmd_pack",
    "cmd_tails": r"k_cmd_tails",
    "log_keys": r"k_log_keys",
    "tail_engine": r"k_tail_engine<unsigned int>",
    "exec_fill_dots": r"k_exec_fill_dots",
    "vid_fill_dots": r"k_vid_fill_dots",
    "exec_from_groups": r"k_exec_from_groups",
    # global graph path (C3 / C5)
    "kap_relax": r"k_kap_relax",
    "kap_init": r"k_kap_init",
    "fb_hprop": r"k_fb_hprop",
    "fb_reach": r"k_fb_reach",
    "fb_init": r"k_fb_init",
    "fb_merge": r"k_fb_merge",
    "windows": r"k_windows",
    "edge_rep": r"k_edge_rep",
    "edges_csr": r"k_edges_csr",
    "sort_scan": r"k_scan_fused",
    "sv_deps": r"k_sv_deps",
    "sv_tails": r"k_sv_tails",
    "kb_partition": r"k_kb_partition",
    "kb_order": r"k_kb_order",
    "kb_step": r"k_kb_step",
}
CALIB_BYTES = 1 << 30


def read_durations(d):
    """-> {kernel name: [per-dispatch duration in s]} from the counter CSVs'
    timestamps (ns)."""
    per = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                try:
                    t = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
                except (KeyError, ValueError):
                    continue
                per[row["Kernel_Name"]][(f, row.get("Dispatch_Id"))] = t
    return {k: list(v.values()) for k, v in per.items()}


def read_counters(d, counter):
    """-> {kernel name: [per-dispatch value]} for `counter` under dir `d`."""
    per = defaultdict(lambda: defaultdict(float))
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per[row["Kernel_Name"]][key] += float(row["Counter_Value"])
    return {k: list(v.values()) for k, v in per.items()}


def calib(root):
    out = {}
    for kind, sub, counter in (("read", "calib_fetch", "FETCH_SIZE"),
                               ("write", "calib_write", "WRITE_SIZE")):
        rows = read_counters(os.path.join(root, sub), counter)
        for name, vals in rows.items():
            m = re.search(r"calib_(read|write|gather|scatter)<(.*)>\s*\(", name)
            if not m:
                continue
            k = m.group(1)
            if (k in ("read", "gather")) != (kind == "read"):
                continue
            t = m.group(2)
            w = 16 if "4u" in t else 8 if "2u" in t else 4
            vals = sorted(vals)
            med = vals[len(vals) // 2] * 1024.0
            out[f"{k}{w}"] = med / CALIB_BYTES
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                  "pmc_traffic.json"))
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    cal = calib(a.root)
    fetch = read_counters(os.path.join(a.root, "fetch"), "FETCH_SIZE")
    write = read_counters(os.path.join(a.root, "write"), "WRITE_SIZE")
    rf, wf = cal.get("read4", 1.0), cal.get("write4", 1.0)
    res = {}
    if os.path.exists(a.out):  # keep the probes this run did not see
        with open(a.out) as fh:
            res = {k: v for k, v in json.load(fh).items() if not k.startswith("_")}
    res.update({"_calibration": {"counter_bytes_over_true_bytes": cal,
                            "note": "1 GiB per access width: read/write = coalesced streams, "
                                    "gather/scatter = one access per lane to a random line of "
                                    "the same buffer (counter bytes per algorithmic byte); raw "
                                    "engine counters are divided by read4 / write4"},
                "_units": "fabric bytes: FETCH_SIZE / WRITE_SIZE count the L2's memory-side "
                          "requests (Infinity-Cache hits included, MI355X_MICROARCH.md §HBM), "
                          "corrected by the stream factors; for gather-bound kernels they "
                          "are fabric traffic, not HBM bytes",
                "_command": a.command})
    dur = read_durations(os.path.join(a.root, "fetch"))
    for probe, pat in PROBES.items():
        fv = [v for k, vs in fetch.items() if pat in k for v in vs]
        wv = [v for k, vs in write.items() if pat in k for v in vs]
        if not fv or not wv:
            continue
        fr = sum(fv) / len(fv) * 1024.0
        wr = sum(wv) / len(wv) * 1024.0
        tv = [t for k, ts in dur.items() if pat in k for t in ts]
        e = {"hbm_bytes_per_launch": fr / rf + wr / wf,
             "fetch_bytes_raw": fr, "write_bytes_raw": wr,
             "read_bytes_corrected": fr / rf, "write_bytes_corrected": wr / wf,
             "launches": [len(fv), len(wv)]}
        if tv and sum(tv) > 0:
            t = sum(tv) / len(tv)
            e["avg_launch_s"] = t
            e["fabric_TBs"] = e["hbm_bytes_per_launch"] / t / 1e12
            # above the ~6.3 TB/s a copy achieves, the bytes cannot all be HBM
            # traffic: Infinity-Cache hits are in them
            e["exceeds_hbm_achievable"] = e["fabric_TBs"] > 6.3
        res[probe] = e
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
