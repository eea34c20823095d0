#!/usr/bin/env python
"""Per-kernel averages of rocprofv3 counter passes (tools/gpu_r05_prof.sh):
python tools/pmc_summary.py gpurun_out/pmcA_<tag> [gpurun_out/pmcB_<tag> ...]"""
import collections
import csv
import glob
import os
import re
import sys

for d in sys.argv[1:]:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for r in rows:
        m = re.search(r"(k_\w+<[^(]*>|k_\w+)\(", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for k, v in acc.items():
        n = len(dur[k])
        print(os.path.basename(d), k, "dispatches", n, "avg_us", round(sum(dur[k].values()) / n, 1),
              {c: round(x / n / 1e6, 2) for c, x in sorted(v.items())})
